"""Time the GPU partial-pivot LU determinant (psx_lu_det_gpu) on random
matrices that need row swaps: blocked panels vs per-column launches
(PSX_LU_UNBLOCKED=1); results must be bit-identical."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from pipsort_amd import engine as E  # noqa: E402

for n in (500, 1000, 2000):
    a = np.random.default_rng(n).standard_normal((n, n))
    out = {}
    for mode in ("blocked", "unblocked", "blocked"):
        if mode == "unblocked":
            os.environ["PSX_LU_UNBLOCKED"] = "1"
        else:
            os.environ.pop("PSX_LU_UNBLOCKED", None)
        E.lu_det(a, gpu=True)
        t = time.perf_counter()
        d = E.lu_det(a, gpu=True)
        out[mode] = ((time.perf_counter() - t) * 1e3, d)
    same = np.float64(out["blocked"][1]).tobytes() == np.float64(out["unblocked"][1]).tobytes()
    print(f"n={n}: blocked {out['blocked'][0]:.2f} ms, unblocked {out['unblocked'][0]:.2f} ms, det bit-identical {same}",
          flush=True)
