"""Summarise a rocprofv3 kernel_trace.csv as a per-pass timeline: for the last
few passes print each kernel's start offset, duration and the gap before it."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
# a pass begins at the fill (memset) kernel
starts = [i for i, k in enumerate(ks) if "fillBuffer" in k[2]]
show = starts[-4:] if len(starts) >= 4 else starts
for si, s in enumerate(show):
    e = show[si + 1] if si + 1 < len(show) else len(ks)
    t0 = ks[s][0]
    print(f"--- pass at {t0}")
    prev_end = t0
    for st, en, name in ks[s:e]:
        print(f"  +{(st - t0) / 1e3:8.1f} us  dur {(en - st) / 1e3:8.1f} us  gap {(st - prev_end) / 1e3:6.1f}  {name[:70]}")
        prev_end = max(prev_end, en)
    print(f"  pass span {(prev_end - t0) / 1e3:.1f} us")
