"""Fit the k_sweep3 unit cost model (plan_units3c's `work`) to measured unit
durations, and show how evenly a world-N decomposition splits the time:
    python tools/unit_fit.py [--world 8] [--workload syn1000c3]
Runs every rank's shard synchronously with PSX_UNIT_TRACE set (lane 0 of each
unit records wall_clock64() at start / end, 100 MHz), then least-squares fits
duration = p + q * n_a separately for off-diagonal and diagonal units and
prints each rank's kernel span, unit count and summed unit time.
Diagnostics only."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
path = "/tmp/psx_unit_fit.bin"
os.environ["PSX_UNIT_TRACE"] = path
import torch  # noqa: E402,F401
import bench  # noqa: E402
from pipsort_amd import engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="syn1000c3")
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
pc = E.PostCal(bench.build_inputs(a.workload), device=0)
rows = []
for rank in range(a.world):
    pc.set_shard(rank, a.world)
    spans = []
    for _ in range(a.reps):
        pc.run_exhaustive()
        tr = np.fromfile(path, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
        spans.append((tr[:, 1].max() - tr[:, 0].min()) / 100.0)
    dur = (tr[:, 1] - tr[:, 0]) / 100.0
    diag = (tr[:, 3] >> 32) & 1
    na = (tr[:, 3] >> 33) & 0x7f
    redo = (tr[:, 3] >> 40) & 1
    rows.append((rank, min(spans), dur, diag, na, redo))
    print(f"rank {rank}: {len(dur)} units ({int(diag.sum())} diagonal, {int(redo.sum())} redone), "
          f"span {min(spans):.1f} us, sum of unit time {dur.sum():.0f} us, "
          f"sum / 512 slots {dur.sum() / 512:.1f} us", flush=True)
dur = np.concatenate([r[2] for r in rows])
diag = np.concatenate([r[3] for r in rows])
na = np.concatenate([r[4] for r in rows])
redo = np.concatenate([r[5] for r in rows])
fit = {}
for d in (0, 1):
    m = (diag == d) & (redo == 0)
    X = np.stack([np.ones(m.sum()), na[m]], axis=1)
    (p, q), *_ = np.linalg.lstsq(X, dur[m], rcond=None)
    fit[d] = (p, q)
    print(f"{'diagonal' if d else 'off-diag'}: duration = {p:.2f} + {q:.2f} * n_a us "
          f"(n={m.sum()}, residual rms {np.sqrt(np.mean((X @ [p, q] - dur[m]) ** 2)):.2f} us)")
q0 = fit[0][1]
print(f"model in off-diagonal-a units: off-diag {fit[0][0] / q0:.3f} + n_a; "
      f"diagonal {fit[1][0] / q0:.3f} + {fit[1][1] / q0:.3f} n_a")
if redo.any():
    print(f"redone units: n={int(redo.sum())}, mean {dur[redo == 1].mean():.1f} us")
pc.close()
