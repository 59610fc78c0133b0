"""M = 2000 GPU Model setup (psx_create_from_ld) repeated, for rocprofv3
--kernel-trace: tools/trace_summary.py / the kernel_trace.csv show where a
warm setup's time goes (uploads, PSD loop, panels, copies)."""
import sys
import time

sys.path.insert(0, ".")
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
ld, z, _, _, u2l = synth.syn_v1(M)
mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=1, sharing_param=0.25)
for rep in range(4):
    t = time.perf_counter()
    pc = E.PostCal(mi)
    print(f"M={M} rep {rep}: create {1e3 * (time.perf_counter() - t):.2f} ms; setup_info {pc.setup_info}", flush=True)
    pc.close()
