"""Run one shard's exhaustive pass repeatedly (for rocprofv3 --kernel-trace):
    python tools/pass_trace.py --rank 0 --world 8 --steps 20
then tools/trace_gaps.py on the kernel_trace.csv shows the per-pass timeline."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from pipsort_amd import engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="syn1000c3")
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
torch.cuda.set_device(0)
seam = bench.build_inputs(a.workload)
pc = E.PostCal(seam, device=0)
pc.set_shard(a.rank, a.world)
import time
for _ in range(3):
    pc.run_exhaustive()
t0 = time.perf_counter()
for _ in range(a.steps):
    pc.run_exhaustive()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / a.steps * 1e3
print(f"world {a.world} rank {a.rank}: {dt:.3f} ms per pass; last timing {pc.timing()}", flush=True)
pc.close()
