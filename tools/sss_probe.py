#!/usr/bin/env python3
"""The bench line's SSS section alone (bench.sss_probe: BASELINE configs[4]
walk, proposal batch with its k_eval_sets roofline, the long walks), printed
as JSON.  usage: python tools/sss_probe.py [REPS]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
print(json.dumps(bench.sss_probe(reps), indent=1))
