#!/usr/bin/env python3
"""Time the SSS proposal batch (bench.sss_batch, BASELINE configs[4] M = 2000)
through psx_eval_union_batch: REPS calls after a warm call, wall per call and
the k_eval_batch launch; run under rocprofv3 --kernel-trace --hip-runtime-trace
for the timeline (tools/trace_summary.py).  usage: tools/batch_trace.py [REPS]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
M = 2000
ld, z, _, _, u2l = synth.syn_v1(M)
mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=5, sharing_param=0.25)
pc = E.PostCal(mi)
arr, npat = bench.sss_batch(M)
for acc in (True, False):
    pc.eval_union_batch(arr, accumulate=acc)
    w, k, prep, run = [], [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        pc.eval_union_batch(arr, accumulate=acc)
        w.append((time.perf_counter() - t0) * 1e3)
        t = pc.timing()
        k.append(t["kernel_ms"])
        prep.append(t["prepare_ms"])
        run.append(t["run_ms"])
    w.sort()
    m = lambda v: sum(v) / len(v)  # noqa: E731
    print(f"accumulate={acc}: wall median {w[len(w) // 2]:.4f} ms min {w[0]:.4f} ms, "
          f"in the call {m(run):.4f} ms (validate + stage {m(prep):.4f} ms), "
          f"k_eval_batch {m(k):.4f} ms, {len(arr)} sets, {npat} configs")
pc.close()
