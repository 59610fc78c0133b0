"""One mixed-locus parity check against the oracle (developer tool; prints the
max PIP difference):  python tools/parity_one.py M0 M1 shared c"""
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

M0, M1, sh, c = (int(x) for x in sys.argv[1:5])
ld, z, _, _, u2l = synth.mixed_locus(M0, M1, sh, seed=M0 + M1)
seam = E.seam_from_arrays(ld, z, u2l, (5000, 9000), max_causal=c, sharing_param=0.5)
pc = E.PostCal(seam)
pc.run_exhaustive()
g = pc.accum()
r = O.postcal(seam)


def se(v, t):
    with np.errstate(over="ignore"):
        x = np.exp(v - t)
    x[v == 0] = 0
    return x


for f in ("post", "no_causal", "shared"):
    d = np.abs(se(getattr(g, f), g.total) - se(r[f], r["total"]))
    print(f, "max |dPIP|", d.max(), "at", int(d.argmax()))
for f in ("shared_ll", "notshared_ll"):
    a, b = getattr(g, f), r[f]
    m = b != 0
    print(f, "max rel", (np.abs(a[m] - b[m]) / np.abs(b[m])).max())
for f in ("post", "no_causal", "shared"):
    a, b = getattr(g, f), r[f]
    m = b != 0
    print(f, "raw log max abs diff", np.abs(a[m] - b[m]).max(), "median", np.median(np.abs(a[m] - b[m])))
print("configs", g.n_configs, r["n_configs"], "total", g.total, r["total"], "exact_rerun", pc.timing()["exact_rerun"])
