"""GPU Model setup time (psx_create_from_ld: PSD shift loop, elimination,
upload) on the SYN-v1 loci, warm (the first create of the process is dropped),
with the setup's phases and the first exhaustive pass of the handle (its plan /
layout preparation and kernel) — the per-locus cost beside the resident sweep."""
import json
import sys
import time

sys.path.insert(0, ".")
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

for M, c in ((1000, 3), (2000, 1)):
    ld, z, _, _, u2l = synth.syn_v1(M)
    mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=c, sharing_param=0.25)
    rows = []
    for rep in range(4):
        t = time.perf_counter()
        pc = E.PostCal(mi)
        wall = (time.perf_counter() - t) * 1e3
        info = pc.setup_info
        row = {"setup_ms": round(info["setup_ms"], 2), "create_wall_ms": round(wall, 2),
               "alloc": round(info["alloc_ms"], 2), "studies": round(info["studies_ms"], 2),
               "tail": round(info["tail_ms"], 2), "upload": [round(x, 2) for x in info["study_upload_ms"]],
               "psd_lu": [round(x, 2) for x in info["study_psd_ms"]],
               "finish": [round(x, 2) for x in info["study_finish_ms"]]}
        if c == 3:
            t = time.perf_counter()
            pc.run_exhaustive()
            tm = pc.timing()
            row["first_pass_wall_ms"] = round((time.perf_counter() - t) * 1e3, 2)
            row["pass_prepare_ms"] = round(tm["prepare_ms"], 2)
            row["pass_kernel_ms"] = round(tm["kernel_ms"], 3)
            t = time.perf_counter()
            pc.run_exhaustive()
            row["second_pass_wall_ms"] = round((time.perf_counter() - t) * 1e3, 2)
        pc.close()
        rows.append(row)
    print(f"M={M} c={c}: psd_iterations {info['psd_iterations']} eigen_route {info['eigen_route']}", flush=True)
    for r in rows:
        print("  " + json.dumps(r), flush=True)
