"""Unit timeline of the k = 3 sweep kernel for one shard (diagnostics):
    python tools/unit_trace.py --world 8 --rank 3
Runs synchronous passes with PSX_UNIT_TRACE set (each k_sweep3 unit's lane 0
records wall_clock64() at start / end, 100 MHz) and prints the kernel span,
unit durations and how many units run concurrently over time."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
path = "/tmp/psx_unit_trace.bin"
os.environ["PSX_UNIT_TRACE"] = path
import torch  # noqa: E402,F401
import bench  # noqa: E402
from pipsort_amd import engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="syn1000c3")
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--world", type=int, default=8)
a = ap.parse_args()
pc = E.PostCal(bench.build_inputs(a.workload), device=0)
pc.set_shard(a.rank, a.world)
for _ in range(3):
    pc.run_exhaustive()
tr = np.fromfile(path, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
st, en = tr[:, 0], tr[:, 1]
t0 = st.min()
span = (en.max() - t0) / 100.0
dur = (en - st) / 100.0
print(f"world {a.world} rank {a.rank}: {len(tr)} units, kernel span {span:.1f} us (wall_clock64)")
print(f"unit duration us: mean {dur.mean():.1f} p10 {np.percentile(dur, 10):.1f} p50 {np.median(dur):.1f} "
      f"p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f}")
print(f"first-unit starts: {((st - t0) / 100.0)[:5]}; last start {(st.max() - t0) / 100.0:.1f} us; "
      f"first end {(en.min() - t0) / 100.0:.1f} us")
edges = np.linspace(0, span, 21)
mid = 0.5 * (edges[1:] + edges[:-1])
conc = [int(((st - t0) / 100.0 <= m).sum() - ((en - t0) / 100.0 <= m).sum()) for m in mid]
print("concurrent units over time (20 bins):", conc)
order = np.argsort(st)
print("start time by unit index decile (us):",
      [round(float((st[order][int(q * (len(st) - 1))] - t0) / 100.0), 1) for q in np.linspace(0, 1, 11)])
uid = tr[:, 3] & 0xffffffff
redo = (tr[:, 3] >> 40) & 1
print(f"units redone by the robust variant: {int(redo.sum())} (mean duration {dur[redo == 1].mean() if redo.any() else 0:.1f} us); "
      f"busy unit-us {dur.sum():.0f}")
diag = (tr[:, 3] >> 32) & 1
na = tr[:, 3] >> 33
for dflag in (0, 1):
    for k in sorted(set(na[diag == dflag].tolist())):
        m = (diag == dflag) & (na == k)
        print(f"{'diagonal' if dflag else 'off-diag'} units with {k} a: n={m.sum()} mean {dur[m].mean():.1f} us")
ph = tr[:, 4:8]
pro = (ph[:, 0] - st) / 100.0
apro = (ph[:, 1] - ph[:, 0]) / 100.0
steps = (ph[:, 2] - ph[:, 1]) / 100.0
fold = (ph[:, 3] - ph[:, 2]) / 100.0
fn = tr[:, 8:14]
for dflag in (0, 1):
    m = diag == dflag
    print(f"{'diagonal' if dflag else 'off-diag'} first-a phases (us, mean): unit prologue {pro[m].mean():.2f}, "
          f"a prologue {apro[m].mean():.2f}, steps {steps[m].mean():.1f}, a fold+record {fold[m].mean():.2f}, "
          f"rest {((en - ph[:, 3]) / 100.0)[m].mean():.2f}")
    if fn[m, 0].any():
        d = lambda x, y: float(((x - y) / 100.0)[m].mean())
        print(f"   a prologue split: loads+barrier {d(fn[:, 0], ph[:, 0]):.2f}, per-study terms {d(fn[:, 1], fn[:, 0]):.2f}, "
              f"vectors+shifts+slot max {d(fn[:, 2], fn[:, 1]):.2f}, closed forms {d(fn[:, 3], fn[:, 2]):.2f}, "
              f"scale+barrier {d(ph[:, 1], fn[:, 3]):.2f}; fold {d(fn[:, 4], ph[:, 2]):.2f}, record {d(ph[:, 3], fn[:, 4]):.2f}")
la = (tr[:, 15] - tr[:, 14]) / 100.0
for dflag in (0, 1):
    m = (diag == dflag) & (tr[:, 14] > 0)
    if m.any():
        print(f"{'diagonal' if dflag else 'off-diag'} LAST-a prologue (units of > 1 a, us, mean): {la[m].mean():.2f}")
bu = np.array([d.mean() for d in np.array_split(dur[np.argsort(uid)], 10)])
print("mean duration by unit-index decile:", np.round(bu, 1).tolist())

# first-a walk time and unit duration by start-time decile (cold-start effects)
sdec = np.array_split(np.argsort(st), 10)
print("first-a steps (us) by start-time decile:", [round(float(steps[i].mean()), 1) for i in sdec])
print("unit duration (us) by start-time decile:", [round(float(dur[i].mean()), 1) for i in sdec])
print("units with 4 a: later-a time per a (us) by start decile:",
      [round(float(((en[i] - ph[i, 3]) / 100.0)[na[i] == 4].mean() / 3.0), 1) if (na[i] == 4).any() else None
       for i in sdec])

# per unit class (off-diagonal / diagonal) and tile: unit-us and a-walks, to
# check the shard split's cost model (psx_sweep.hip plan_units3c)
tK = (tr[:, 2] >> 40) & 0xff
tC = (tr[:, 2] >> 48) & 0xff
for dflag in (0, 1):
    m = diag == dflag
    if m.any():
        print(f"{'diagonal' if dflag else 'off-diag'}: units {int(m.sum())}, a-walks {int(na[m].sum())}, "
              f"busy unit-us {dur[m].sum():.0f}, us per a-walk {dur[m].sum() / max(1, na[m].sum()):.2f}")
m = diag == 0
if m.any():
    rows = []
    for k in sorted(set(tK[m].tolist())):
        mk = m & (tK == k)
        rows.append((k, round(float(dur[mk].sum() / na[mk].sum()), 2)))
    print("off-diag us per a-walk by K:", rows)
m = diag == 1
if m.any():
    rows = []
    for k in sorted(set(tK[m].tolist())):
        mk = m & (tK == k)
        rows.append((k, round(float(dur[mk].sum() / na[mk].sum()), 2)))
    print("diagonal us per a-walk by K:", rows)
xcc = (tr[:, 2] >> 32) & 0xf
print("XCC of unit index (first 16):", xcc[:16].tolist(), "; fraction with XCC == index % 8:",
      round(float((xcc == (np.arange(len(xcc)) % 8)).mean()), 3))
# per XCD (blocks are dealt round-robin over the 8 XCDs): the span ends with
# the slowest XCD; busy / (slots x span) is the occupancy the drain leaves
print(f"ideal span at 2048 wave slots: {dur.sum() / 2048:.1f} us (busy unit-us / slots) vs span {span:.1f} us")
for x in range(8):
    m = xcc == x
    if m.any():
        print(f"  XCC {x}: units {int(m.sum())}, busy unit-us {dur[m].sum():.0f} (ideal {dur[m].sum() / 256:.1f} us), "
              f"last end {(en[m].max() - t0) / 100.0:.1f} us, last start {(st[m].max() - t0) / 100.0:.1f} us")
pc.close()
