"""Time the SSS walk (psx_run_sss, sss_postcal.cpp:102-380) on SYN-v1 loci:
iterations, configurations, walk wall time, kernel time and the host share.

    python tools/sss_walk_probe.py [--loci 100,200,2000] [--c 5] [--reps 2]

PSX_ENGINE_LIB selects the engine library (A/B).  Developer tool: one JSON
line per locus.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loci", default="100,200,2000")
    ap.add_argument("--c", type=int, default=5)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    for M in [int(x) for x in args.loci.split(",")]:
        ld, z, _, _, u2l = synth.syn_v1(M)
        mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=args.c, sharing_param=0.25)
        pc = E.PostCal(mi)
        best = None
        for _ in range(args.reps):
            t0 = time.perf_counter()
            it = pc.run_sss()
            dt = (time.perf_counter() - t0) * 1e3
            if best is None or dt < best[0]:
                best = (dt, it, pc.timing())
        dt, it, tm = best
        n = pc.accum().n_configs
        pc.close()
        print(json.dumps({"locus": f"SYN-v1 M={M} -c {args.c}", "iterations": it, "configs": n,
                          "walk_ms": round(dt, 2), "kernel_ms": round(tm["kernel_ms"], 2),
                          "host_and_sync_ms": round(dt - tm["kernel_ms"], 2),
                          "ms_per_iteration": round(dt / max(it, 1), 3),
                          "configs_per_s": n / (dt / 1e3)}), flush=True)


if __name__ == "__main__":
    main()
