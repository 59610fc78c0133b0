"""Run one shard's step repeatedly (for rocprofv3 --kernel-trace):
    python tools/pass_trace.py --rank 0 --world 8 --steps 20
A step is the bench step: asynchronous pass + (world > 1) export, one copy
kernel standing in for the RCCL all-gather, merge.  tools/trace_gaps.py on the
kernel_trace.csv shows the per-step timeline."""
import argparse
import os
import sys
import time

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
stream = torch.cuda.Stream(priority=-1)
torch.cuda.set_stream(stream)
pc.set_stream(stream.cuda_stream)
pc.set_shard(a.rank, a.world)
nb = pc.partials_bytes()
mine = torch.empty(nb, dtype=torch.uint8, device="cuda")
gathered = torch.empty(nb * a.world, dtype=torch.uint8, device="cuda")
# the copies stand in for ranks 0..world-1: their plan tags get those ranks
tag_rank = (nb // 56 - 1) * 56 + 8
rank_bytes = torch.arange(a.world, dtype=torch.int32, device="cuda").view(torch.uint8).view(a.world, 4)


def step():
    pc.run_exhaustive_async()
    if a.world > 1:
        pc.export_partials(mine.data_ptr())
        gathered.view(a.world, nb).copy_(mine.view(1, nb).expand(a.world, nb))
        gathered.view(a.world, nb)[:, tag_rank:tag_rank + 4].copy_(rank_bytes)
        pc.merge_partials(gathered.data_ptr(), a.world)


for _ in range(3):
    step()
torch.cuda.synchronize()
pc.sync()
t0 = time.perf_counter()
for _ in range(a.steps):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / a.steps * 1e3
assert not pc.sync()
print(f"world {a.world} rank {a.rank}: {dt:.3f} ms per step; timing {pc.timing()}", flush=True)
pc.close()
