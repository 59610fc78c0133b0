"""Time process exit of tools/exit_probe.bin per mode (5 reps each): the gap
between the epoch the probe prints just before _exit(0) and the parent seeing
it end.  python tools/exit_probe.py"""
import json
import os
import subprocess
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for mode in (0, 1, 2, 3):
    ex, tot = [], []
    for _ in range(5):
        t0 = time.time()
        r = subprocess.run([os.path.join(ROOT, "tools", "exit_probe.bin"), str(mode)], capture_output=True, text=True)
        t1 = time.time()
        d = json.loads(r.stdout.strip().splitlines()[-1])
        ex.append(t1 * 1e3 - d["exit_epoch_ms"])
        tot.append((t1 - t0) * 1e3)
    print(json.dumps({"mode": mode, "exit_ms": sorted(ex), "wall_ms": sorted(tot), "last": d}), flush=True)
