#!/usr/bin/env python3
"""Summarise tools/gpu_pmc.sh output into profiles/pmc_latest.json (read by bench.py).

usage: tools/pmc_summary.py gpurun_out/<TAG>/pmc WORKLOAD [KERNEL_SUBSTRING]

Per-dispatch averages of every counter for the dominant kernel, plus derived
figures.  HBM traffic per launch follows MI355X_MICROARCH.md (HBM/rocprofv3):
FETCH_SIZE (KB) counts 64 B per 128 B request of a coalesced read, so it is
doubled; WRITE_SIZE (KB) is taken as is.
"""
import collections
import csv
import glob
import json
import os
import sys

d, workload = sys.argv[1], sys.argv[2]
ksub = sys.argv[3] if len(sys.argv) > 3 else "k_sweep3"
agg = collections.defaultdict(float)
cnt = collections.Counter()
name = None
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if ksub not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        key = (os.path.basename(os.path.dirname(f)), r["Counter_Name"], r["Dispatch_Id"])
        agg[key] += float(r["Counter_Value"])
per = collections.defaultdict(list)
for (p, c, disp), v in agg.items():
    per[c].append(v)
c = {k: sum(v) / len(v) for k, v in per.items()}
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402  (kernel_src_sha: which build these counters describe)

out = {"workload": workload, "kernel": name, "kernel_src_sha": bench.kernel_src_sha(), "counters_per_dispatch": c}
if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
    out["hbm_bytes_per_launch"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
    out["hbm_bytes_note"] = "2 x FETCH_SIZE + WRITE_SIZE (KB -> B), gfx950 FETCH_SIZE half-count correction"
if "SQ_INSTS_VALU_FLOPS_FP64" in c:
    out["fp64_flop_insts_per_launch"] = c["SQ_INSTS_VALU_FLOPS_FP64"]  # per wave instruction (FMA = 2); x 64 lanes = FP64 operations
if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
    # every wave64 VALU instruction occupies its SIMD for 4 cycles; 1024 SIMDs.
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs (8 x 2.4 GHz x kernel time), so
    # the kernel's cycle count is GRBM_GUI_ACTIVE / 8.
    out["gpu_cycles_per_launch"] = c["GRBM_GUI_ACTIVE"] / 8.0
    out["valu_busy"] = 4.0 * c["SQ_INSTS_VALU"] / (1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0)
    out["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]  # wave64 VALU instructions of one launch
    f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                      "SQ_INSTS_VALU_TRANS_F64"))
    if f64:
        out["fp64_valu_insts_per_launch"] = f64
        out["fp64_valu_share"] = f64 / c["SQ_INSTS_VALU"]
for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
    if k in c and "SQ_WAVE_CYCLES" in c:
        out[k.lower() + "_frac"] = c[k] / c["SQ_WAVE_CYCLES"]
# the SSS proposal batch's evaluator (bench.py sss_probe: one k_eval_batch
# launch over the whole neighbourhood): the largest-grid k_eval_batch dispatches
ev = collections.defaultdict(float)
grids, names = {}, {}
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "k_eval_batch" not in r["Kernel_Name"]:
            continue
        key = (os.path.basename(os.path.dirname(f)), r["Counter_Name"], r["Dispatch_Id"])
        ev[key] += float(r["Counter_Value"])
        grids[r["Dispatch_Id"]] = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        names[r["Dispatch_Id"]] = "k_eval_batch5" if "k_eval_batch5" in r["Kernel_Name"] else "k_eval_batch"
if ev:
    gmax = max(grids.values())
    per_ev = collections.defaultdict(list)
    for (p, cn, disp), v in ev.items():
        if grids[disp] == gmax:
            per_ev[cn].append(v)
    ce = {k: sum(v) / len(v) for k, v in per_ev.items()}
    kname = sorted({names[x] for x in grids if grids[x] == gmax})
    out["sss_eval"] = {"kernel": "/".join(kname), "grid_size": gmax, "eval_src_sha": bench.eval_src_sha(),
                       "counters_per_dispatch": ce}
    if "SQ_INSTS_VALU_FLOPS_FP64" in ce:
        out["sss_eval"]["fp64_flop_insts_per_launch"] = ce["SQ_INSTS_VALU_FLOPS_FP64"]
json.dump(out, open(os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_latest.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "counters_per_dispatch"}, indent=1))
