"""Timeline of a rocprofv3 --kernel-trace --hip-runtime-trace csv directory:
HIP API calls longer than a threshold and kernels (grouped runs of one name),
in start order, times relative to the first event (ms).

usage: tools/trace_summary.py DIR [min_api_us=40] [t_from_ms] [t_to_ms]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 40.0
t_from = float(sys.argv[3]) if len(sys.argv) > 3 else -1e18
t_to = float(sys.argv[4]) if len(sys.argv) > 4 else 1e18


def rows(pat):
    f = glob.glob(os.path.join(d, pat))
    return list(csv.DictReader(open(f[0]))) if f else []


api = rows("*hip_api_trace.csv")
ker = rows("*kernel_trace.csv")
cpy = rows("*memory_copy_trace.csv")
ev = []
for r in api:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ev.append((s, e, "api", f'{r["Function"]} [t{r["Thread_Id"]}]'))
for r in ker:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    ev.append((s, e, "ker", nm.split("(")[0][-48:]))
for r in cpy:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ev.append((s, e, "cpy", f'{r.get("Direction", "copy")} {int(r.get("Bytes", 0) or 0)} B'))
ev.sort()
t0 = ev[0][0]
run = None


def flush():
    global run
    if run:
        s, e, name, n, busy = run
        print(f"{(s - t0) / 1e6:10.3f} {(e - s) / 1e3:9.1f} us  ker x{n:<4d} busy {busy / 1e3:8.1f} us  {name}")
    run = None


for s, e, kind, name in ev:
    t = (s - t0) / 1e6
    if t < t_from or t > t_to:
        continue
    if kind == "ker":
        if run and run[2] == name:
            run = (run[0], e, name, run[3] + 1, run[4] + e - s)
        else:
            flush()
            run = (s, e, name, 1, e - s)
        continue
    if kind == "api" and (e - s) / 1e3 < thr:
        continue
    flush()
    print(f"{t:10.3f} {(e - s) / 1e3:9.1f} us  {kind}  {name}")
flush()
