#!/usr/bin/env python3
"""Which EXACT-rerun checks of the k = 3 sweep fire (psx_timing.exact_rerun
bits: 1 = a set's / an a or c slot's notSharedLL group, 2 = an off-diagonal
unit's b-slot total) on loci with one strong shared SNP x, scanning the weaker
study's signal around the 900-bit floor.  Used to find a locus for the
SEP b-slot trigger test (tests/test_gpu_parity.py).
usage: tools/exact_bits.py M x z0 z1_lo z1_hi step"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pipsort_amd import engine as E  # noqa: E402


def locus(M, x, z0, z1, seed=9):
    idx = np.arange(M)
    ld, z = [], []
    for s, (rho, lamx) in enumerate(((0.5, z0), (0.3, z1))):
        sig = rho ** np.abs(idx[:, None] - idx[None, :])
        lam = np.zeros(M)
        lam[x] = lamx
        eps = np.random.default_rng(seed + s).standard_normal(M)
        z.append(sig @ lam + np.linalg.cholesky(sig) @ eps)
        ld.append(sig)
    u2l = np.stack([idx, idx]).astype(np.int32)
    return E.seam_from_arrays(ld, z, u2l, (12000, 9000), max_causal=3, sharing_param=0.3)


if __name__ == "__main__":
    M, x = int(sys.argv[1]), int(sys.argv[2])
    z0, lo, hi, step = (float(v) for v in sys.argv[3:7])
    for z1 in np.arange(lo, hi + 1e-9, step):
        pc = E.PostCal(locus(M, x, z0, z1))
        pc.run_exhaustive()
        t = pc.timing()
        print(f"M={M} x={x} z0={z0} z1={z1:.3f} bits={t['exact_rerun']} robust={t['robust_units']}", flush=True)
        pc.close()
