"""End-to-end wall time of the drop-in PIPSORT on a SYN-v1 locus written in
the reference's input formats (developer tool):
    python tools/cli_e2e.py --M 1000 --c 3 [--q 1]"""
import argparse
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=1000)
ap.add_argument("--c", type=int, default=3)
ap.add_argument("--q", type=int, default=0)
ap.add_argument("--bin", default=E.PIPSORT_BIN, help="PIPSORT executable (A/B builds)")
ap.add_argument("--reps", type=int, default=1)
a = ap.parse_args()
with tempfile.TemporaryDirectory() as d:
    ld, z, names, rows, _ = synth.syn_v1(a.M)
    t0 = time.time()
    synth.write_locus(d, ld, z, names, rows)
    t1 = time.time()
    args = [a.bin, "-c", str(a.c), "-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "snp_map", "-n",
            "10000,8000", "-p", "0.25", "-o", "out"] + (["-q", str(a.q)] if a.q else [])
    best = None
    for _ in range(a.reps):
        t2 = time.time()
        r = subprocess.run(args, cwd=d, capture_output=True, text=True)
        t3 = time.time()
        best = t3 - t2 if best is None else min(best, t3 - t2)
    t2, t3 = 0.0, best
    sizes = sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d) if f.endswith(".ld"))
    print(f"M={a.M} c={a.c} q={a.q}: write {t1 - t0:.2f} s ({sizes / 1e6:.0f} MB LD text); PIPSORT wall {t3 - t2:.3f} s rc={r.returncode}")
    for line in r.stdout.splitlines():
        if "Time" in line or "psd shift" in line or "configurations" in line.lower():
            print("   ", line)
    if r.returncode:
        print(r.stdout[-2000:], r.stderr[-2000:])
