#!/usr/bin/env python3
"""A/B of the SSS walk's eval wait (psx_engine.hip run_sss): PSX_SSS_FLAG=0
waits for the eval's stop event before reading the neighbours' mark words, 1
(the default) polls the words as the eval publishes them.  Modes alternate per
round on one handle; every walk's accumulators must be bitwise identical to
the first walk's.  usage: python tools/sss_flag_ab.py [ROUNDS] [M ...]"""
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (HIP runtime first, as in bench.py)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
loci = [int(x) for x in sys.argv[2:]] or [100, 200]
modes = ("0", "1")
for M in loci:
    ld, z, _, _, u2l = synth.syn_v1(M)
    mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=5, sharing_param=0.25)
    pc = E.PostCal(mi)
    pc.run_sss()  # first-call costs
    ref = None
    ms = {m: [] for m in modes}
    same = {m: True for m in modes}
    for r in range(rounds):
        order = modes if r % 2 == 0 else modes[::-1]
        for m in order:
            os.environ["PSX_SSS_FLAG"] = m
            t0 = time.perf_counter()
            it = pc.run_sss()
            ms[m].append((time.perf_counter() - t0) * 1e3)
            a = pc.accum()
            v = np.concatenate([a.post, a.no_causal, a.shared, a.shared_ll, [float(a.n_configs), float(it)]])
            if ref is None:
                ref = v
            same[m] &= bool(np.array_equal(v.view(np.uint64), ref.view(np.uint64)))
    pc.close()
    print(json.dumps({"M": M, "iterations": it,
                      "walk_ms": {m: {"min": min(x), "median": float(np.median(x))} for m, x in ms.items()},
                      "bitwise_same_as_first": same}), flush=True)
