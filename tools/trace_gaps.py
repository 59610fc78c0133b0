"""Summarise a rocprofv3 kernel_trace.csv as a per-step timeline: for the last
few steps print each kernel's start offset, duration and the gap before it.
A step begins at the dominant sweep kernel (k_sweep3)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
starts = [i for i, k in enumerate(ks) if "k_sweep3" in k[2]]
show = starts[-4:] if len(starts) >= 4 else starts
for si, s in enumerate(show):
    e = show[si + 1] if si + 1 < len(show) else len(ks)
    t0 = ks[s][0]
    print(f"--- step at {t0}")
    prev_end = t0
    for st, en, name in ks[s:e]:
        print(f"  +{(st - t0) / 1e3:8.1f} us  dur {(en - st) / 1e3:8.1f} us  gap {(st - prev_end) / 1e3:6.1f}  {name[:70]}")
        prev_end = max(prev_end, en)
    nxt = ks[show[si + 1]][0] if si + 1 < len(show) else prev_end
    print(f"  step span {(nxt - t0) / 1e3:.1f} us")
