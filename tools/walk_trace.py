"""The SSS walk on SYN-v1 M = 200, -c 5 (bench.py long_walks), run a few times
with PSX_SSS_PROFILE's host phases on stderr: the walk wall per run and its
iterations.  Run under rocprofv3 --kernel-trace for the device timeline
(tools/trace_timeline.py).  Developer tool.

    PSX_SSS_PROFILE=1 python tools/walk_trace.py [--reps 3] [--m 200]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--m", type=int, default=200)
a = ap.parse_args()
ld, z, _, _, u2l = synth.syn_v1(a.m)
pc = E.PostCal(E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=5, sharing_param=0.25))
for i in range(a.reps + 1):
    t0 = time.perf_counter()
    it = pc.run_sss()
    w = (time.perf_counter() - t0) * 1e3
    print(f"run {i}: {it} iterations, walk {w:.3f} ms ({w / max(it, 1) * 1e3:.1f} us per iteration), "
          f"kernel {pc.timing()['kernel_ms']:.3f} ms", flush=True)
pc.close()
