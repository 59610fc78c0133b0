"""How long a HIP process takes to go away after _exit: tools/init_probe (a
bare HIP start-up, optionally holding device / pinned memory) and the drop-in
CLI on tests/example, each in fresh processes; the exit is the child's
monotonic clock at _exit (its end_ms / PSX_TIMING "end") to the parent's
return from wait.  Developer tool.

    python tools/exit_probe.py [--reps 4]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=4)
a = ap.parse_args()
probe = os.path.join(ROOT, "tools", "init_probe")
for args in ([], ["0", "0"], ["1024", "0"], ["16384", "0"], ["0", "256"], ["0", "0", "1"], ["0", "0", "3"],
             ["0", "0", "6"]):
    ex = []
    for _ in range(a.reps):
        p = subprocess.Popen([probe, "0"] + args, stdout=subprocess.PIPE, text=True)
        line = p.stdout.readline()
        p.wait()
        t = time.monotonic() * 1e3
        d = json.loads(line)
        ex.append(t - d["end_ms"])
    print(f"init_probe {' '.join(args) or '(bare)'}: exit {statistics.median(ex):.1f} ms "
          f"(min {min(ex):.1f}, of {a.reps}); device MiB / pinned MiB / streams held: {args or ['0', '0']}", flush=True)

import bench  # noqa: E402

for sq in ("1", "0", "1", "0"):  # the CLI's one queue (default) against the engine's own streams
    os.environ["PSX_SINGLE_QUEUE"] = sq
    w, same, ph = bench.example_wall()
    print(f"CLI tests/example (PSX_SINGLE_QUEUE={sq}): wall {w:.3f} s, outputs match {same}, exit_ms {ph.get('exit_ms') if ph else None}",
          flush=True)
