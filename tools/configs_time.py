"""Time the -b configs-file path at scale (bench.configs_probe: 4,826,809 rows
of SYN-v1 M = 1000, c = 3): python tools/configs_time.py  (PSX_ENGINE_LIB
selects an A/B build).  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402,F401
import bench  # noqa: E402

print(json.dumps(bench.configs_probe()), flush=True)
