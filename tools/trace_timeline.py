"""The last N kernel dispatches and memory copies of a rocprofv3 --kernel-trace
--memory-copy-trace run (its rocpd SQLite output) in time order: start
relative to the first shown, duration, gap after the previous one.  Developer
tool.

    python tools/trace_timeline.py gpurun_out/<tag>/prof [--last 40]
"""
import argparse
import glob
import os
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--last", type=int, default=40)
a = ap.parse_args()
db = sorted(glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True))[0]
c = sqlite3.connect(db)
ev = [(s, e, n[:70]) for n, s, e in c.execute("select name, start, end from kernels")]
ev += [(s, e, n) for n, s, e in c.execute("select name, start, end from memory_copies")]
ev.sort()
shown = ev[-a.last:]
t0, prev = shown[0][0], None
for s, e, n in shown:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  {n}")
    prev = e
