"""GPU Model setup time (psx_create_from_ld: PSD shift loop, elimination,
upload) on the SYN-v1 loci, warm (the first create of the process is dropped)."""
import sys
import time

sys.path.insert(0, ".")
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

for M in (1000, 2000):
    ld, z, _, _, u2l = synth.syn_v1(M)
    mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=1, sharing_param=0.25)
    ms = []
    for rep in range(4):
        t = time.perf_counter()
        pc = E.PostCal(mi)
        wall = (time.perf_counter() - t) * 1e3
        ms.append((pc.setup_info["setup_ms"], wall))
        info = pc.setup_info
        pc.close()
    print(f"M={M}: setup_ms (engine, wall) per create {[(round(a, 2), round(b, 2)) for a, b in ms]}; "
          f"psd_iterations {info['psd_iterations']} eigen_route {info['eigen_route']}", flush=True)
