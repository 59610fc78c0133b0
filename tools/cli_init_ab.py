"""tests/example through the drop-in CLI in fresh processes under environment
variants, alternating, with the CLI's phase split (PSX_TIMING): where the cold
start of a one-locus run goes (HIP runtime, first allocation / launch, setup,
exit).  Developer tool.

    python tools/cli_init_ab.py [--reps 4] [VAR=VALUE[,VAR=VALUE] ...]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("variants", nargs="*")
a = ap.parse_args()
variants = [""] + a.variants
res = {v: [] for v in variants}
base = dict(os.environ)
for rep in range(a.reps):
    for v in variants:
        os.environ.clear()
        os.environ.update(base)
        for kv in filter(None, v.split(",")):
            k, val = kv.split("=", 1)
            os.environ[k] = val
        w, same, ph = bench.example_wall()
        res[v].append((w, same, ph))
os.environ.clear()
os.environ.update(base)
keys = ("hip_runtime_ms", "context_and_code_load_ms", "wait_for_gpu_ms", "gpu_setup_ms", "exit_ms")
for v in variants:
    rows = res[v]
    walls = [r[0] for r in rows if r[0]]
    med = {k: statistics.median([r[2][k] for r in rows if r[2]]) for k in keys}
    em = statistics.median([r[2]["context_and_code_load_split"]["engine_module_ms"] for r in rows
                            if r[2] and r[2].get("context_and_code_load_split")])
    sp = {k: statistics.median([r[2]["context_and_code_load_split"].get("engine_module_split", {}).get(k, 0.0)
                                for r in rows if r[2] and r[2].get("context_and_code_load_split")])
          for k in ("first_alloc_ms", "first_launch_enqueue_ms", "first_launch_complete_ms")}
    ss = [r[2].get("gpu_setup_split") for r in rows if r[2] and r[2].get("gpu_setup_split")]
    if ss:
        print(f"  gpu_setup_split (last): {ss[-1]}")
    print(f"[{v or 'default'}] wall median {statistics.median(walls):.3f} s (min {min(walls):.3f}), outputs match "
          f"{all(r[1] for r in rows)}; " + ", ".join(f"{k} {med[k]:.1f}" for k in keys) + f", engine_module {em:.1f} ({', '.join(f'{k} {x:.1f}' for k, x in sp.items())})",
          flush=True)
