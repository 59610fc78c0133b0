"""Where the SSS proposal batch's time goes (bench.py sss_probe's batch: the
neighbourhood of a 4-SNP configuration on SYN-v1 M = 2000, -c 5): the whole
call from Python, the C-ABI call's own wall (psx_get_timing run_ms), the
staging copy (prepare_ms) and the k_eval_batch launch (HIP events), medians.
Run under rocprofv3 --kernel-trace --memory-copy-trace --stats for the merges
and copies.  Developer tool.

    python tools/batch_trace.py [--reps 50]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
M = 2000
ld, z, _, _, u2l = synth.syn_v1(M)
pc = E.PostCal(E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=5, sharing_param=0.25))
arr, npat = bench.sss_batch(M)
for _ in range(5):
    pc.eval_union_batch(arr, accumulate=True)
walls, runs, preps, kms = [], [], [], []
for _ in range(a.reps):
    t0 = time.perf_counter()
    pc.eval_union_batch(arr, accumulate=True)
    walls.append((time.perf_counter() - t0) * 1e3)
    t = pc.timing()
    runs.append(t["run_ms"])
    preps.append(t["prepare_ms"])
    kms.append(t["kernel_ms"])
pc.close()
med = statistics.median
print(f"batch of {len(arr)} sets ({npat} configurations): python call {med(walls):.4f} ms, C-ABI call "
      f"{med(runs):.4f} ms, staging copy {med(preps):.4f} ms, k_eval_batch5 {med(kms):.4f} ms (medians of {a.reps})",
      flush=True)
