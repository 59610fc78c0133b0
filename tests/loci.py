"""Fixture loci in the reference input formats (tests/golden/*), parsed like util.cpp."""
from __future__ import annotations

import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def read_locus(dirname, ldlist="ldfiles.txt", zlist="zfiles.txt", snp_map=None):
    d = os.path.join(GOLDEN, dirname) if not os.path.isabs(dirname) else dirname
    lds = [l.strip() for l in open(os.path.join(d, ldlist)) if l.strip()]
    zs = [l.strip() for l in open(os.path.join(d, zlist)) if l.strip()]
    ld, z, names = [], [], []
    for lf, zf in zip(lds, zs):
        vals = np.array(open(os.path.join(d, lf)).read().split(), dtype=np.float64)
        M = int(np.sqrt(vals.size))
        ld.append(vals[: M * M].reshape(M, M))
        nm, zz = [], []
        for line in open(os.path.join(d, zf)):
            p = line.split()
            nm.append(p[0])
            zz.append(float(p[1]))
        names.append(nm)
        z.append(np.array(zz))
    if snp_map is None:
        cands = [f for f in os.listdir(d) if "snp_map" in f]
        snp_map = cands[0]
    rows = [l.rstrip("\n").split(",") for l in open(os.path.join(d, snp_map)) if l.strip()]
    u2l = np.array([[int(r[1]) for r in rows], [int(r[2]) for r in rows]], dtype=np.int32)
    return dict(dir=d, ld=ld, z=z, names=names, snps=[r[0] for r in rows], u2l=u2l,
                files=[os.path.join(d, x) for x in lds] + [os.path.join(d, x) for x in zs]
                + [os.path.join(d, snp_map)])


EXAMPLE = dict(dirname="example", n=(334324, 6771), c=2, p=0.25)
SMALL = dict(dirname="small_example", n=(7000, 7000), c=3, p=0.75)
CONFIGS = dict(dirname="test_optional_configs", n=(7000, 7000), c=3, p=0.75)


def seam_for(spec, c=None, p=None, **kw):
    from pipsort_amd.engine import seam_from_arrays
    L = read_locus(spec["dirname"])
    return seam_from_arrays(L["ld"], L["z"], L["u2l"], spec["n"], max_causal=c if c is not None else spec["c"],
                            sharing_param=p if p is not None else spec["p"], **kw), L
