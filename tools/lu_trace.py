"""Phase clocks of the tiled swap-free LU (PSX_LU_TRACE): the average per panel
of tiles (0, 0) and (1, 1) (operand loads + diagonal block + L pass | U solve |
delayed update), and each elimination's wall time, on SYN-v1 LDs."""
import os
import sys
import time

os.environ["PSX_LU_TRACE"] = "1"
sys.path.insert(0, ".")
import numpy as np  # noqa: E402
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

for M in (1000, 2000):
    ld, z, _, _, _ = synth.syn_v1(M)
    for rep in range(3):
        t = time.perf_counter()
        piv, zt, sw = E.elim_gpu(ld[0], z[0])
        print(f"M={M} rep {rep}: {1e3 * (time.perf_counter() - t):.2f} ms (incl. upload) swap={sw}", flush=True)

