"""Host-side cost of one bench step (diagnostics): time each host call of the
world-N step loop (asynchronous pass, export, stand-in all-gather, merge of
partials) while the device runs, to see whether the host keeps ahead of the GPU.
    python tools/host_step.py --world 8 --steps 50"""
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
ap.add_argument("--steps", type=int, default=50)
a = ap.parse_args()
torch.cuda.set_device(0)
pc = E.PostCal(bench.build_inputs(a.workload), device=0)
stream = torch.cuda.Stream(priority=-1)
torch.cuda.set_stream(stream)
pc.set_stream(stream.cuda_stream)
pc.set_shard(a.rank, a.world)
nb = pc.partials_bytes()
mine = torch.empty(nb, dtype=torch.uint8, device="cuda")
gathered = torch.empty(nb * a.world, dtype=torch.uint8, device="cuda")
names = ["run_exhaustive_async", "export_partials", "all-gather stand-in", "merge_partials"]
acc = [0.0] * 4


def step(tally):
    t = [time.perf_counter()]
    pc.run_exhaustive_async()
    t.append(time.perf_counter())
    pc.export_partials(mine.data_ptr())
    t.append(time.perf_counter())
    gathered.view(a.world, nb).copy_(mine.view(1, nb).expand(a.world, nb))
    t.append(time.perf_counter())
    pc.merge_partials(gathered.data_ptr(), a.world)
    t.append(time.perf_counter())
    if tally:
        for i in range(4):
            acc[i] += t[i + 1] - t[i]


for _ in range(3):
    step(False)
torch.cuda.synchronize()
pc.sync()
t0 = time.perf_counter()
for _ in range(a.steps):
    step(True)
th = time.perf_counter() - t0
torch.cuda.synchronize()
dt = time.perf_counter() - t0
assert not pc.sync()
t = pc.timing()
print(f"world {a.world} rank {a.rank}: step {dt / a.steps * 1e3:.3f} ms, host loop {th / a.steps * 1e3:.3f} ms per step, "
      f"kernel {t['kernel_ms'] / max(t['kernel_launches'], 1):.3f} ms")
for n, v in zip(names, acc):
    print(f"  {n:22s} {v / a.steps * 1e6:8.1f} us per step")
pc.close()
