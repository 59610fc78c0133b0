"""HIP start-up / exit cost of the drop-in CLI's device path under runtime
environment settings (tools/exit_probe.bin mode 2 = HIP runtime + the warm-up
of a c = 2 run, then _exit): 5 runs each, medians.  python tools/init_env_probe.py"""
import json
import os
import statistics
import subprocess
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENVS = [{}, {"HSA_ENABLE_SDMA": "0"}, {"GPU_MAX_HW_QUEUES": "1"}, {"HIP_FORCE_DEV_KERNARG": "1"},
        {"HSA_ENABLE_SDMA": "0", "GPU_MAX_HW_QUEUES": "1"}, {}]
for extra in ENVS:
    rt, wm, ex, wall = [], [], [], []
    for _ in range(5):
        t0 = time.time()
        r = subprocess.run([os.path.join(ROOT, "tools", "exit_probe.bin"), "2"], capture_output=True, text=True,
                           env=dict(os.environ, **extra))
        t1 = time.time()
        d = json.loads(r.stdout.strip().splitlines()[-1])
        rt.append(d["runtime_ms"])
        wm.append(d["warm_ms"])
        ex.append(t1 * 1e3 - d["exit_epoch_ms"])
        wall.append((t1 - t0) * 1e3)
    med = statistics.median
    print(json.dumps({"env": extra, "runtime_ms": med(rt), "warm_ms": med(wm), "exit_ms": med(ex),
                      "wall_ms": med(wall)}), flush=True)
