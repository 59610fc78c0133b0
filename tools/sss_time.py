"""Time the SSS path (sss_postcal.cpp:102-380) and the GPU Model setup on a
SYN-v1 locus:  python tools/sss_time.py --M 2000 --c 5"""
import argparse
import json
import os
import sys
import time

import torch  # noqa: F401  (HIP runtime first, as in bench.py)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=2000)
ap.add_argument("--c", type=int, default=5)
ap.add_argument("--reps", type=int, default=1)
a = ap.parse_args()
t0 = time.perf_counter()
ld, z, _, _, u2l = synth.syn_v1(a.M)
t1 = time.perf_counter()
mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=a.c, sharing_param=0.25)
pc = E.PostCal(mi)
t2 = time.perf_counter()
print(f"synth {t1 - t0:.2f} s; GPU setup+create {t2 - t1:.3f} s; info {pc.setup_info}", flush=True)
for r in range(a.reps):
    t3 = time.perf_counter()
    it = pc.run_sss()
    t4 = time.perf_counter()
    acc = pc.accum()
    tm = pc.timing()
    print(json.dumps({"M": a.M, "c": a.c, "iterations": it, "wall_s": t4 - t3, "configs": acc.n_configs,
                      "configs_per_s": acc.n_configs / (t4 - t3), "timing": tm}), flush=True)
pc.close()
