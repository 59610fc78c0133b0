"""Per-locus cost under a trace: a few warm creates of the SYN-v1 M = 1000 c = 3
locus (GPU Model setup) and each handle's first and second exhaustive pass.
Run it under `rocprofv3 --sys-trace` (or --kernel-trace --hip-trace) and read
the timeline with tools/trace_summary.py."""
import sys
import time

sys.path.insert(0, ".")
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
c = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ld, z, _, _, u2l = synth.syn_v1(M)
mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=c, sharing_param=0.25)
for rep in range(3):
    t0 = time.perf_counter()
    pc = E.PostCal(mi)
    t1 = time.perf_counter()
    pc.run_exhaustive()
    t2 = time.perf_counter()
    pc.run_exhaustive()
    t3 = time.perf_counter()
    pc.accum()
    t4 = time.perf_counter()
    print(f"rep {rep}: create {1e3 * (t1 - t0):.2f} first pass {1e3 * (t2 - t1):.2f} second {1e3 * (t3 - t2):.2f} "
          f"accum {1e3 * (t4 - t3):.2f} ms; setup {pc.setup_info}", flush=True)
    pc.close()
