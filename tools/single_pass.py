"""Single-locus latency on ONE GPU: one exhaustive pass of one shard, from the
host call to merged accumulators the host can read, for world = 1, 2, 4, 8.

    python tools/single_pass.py [--workload syn1000c3] [--passes 20] [--worlds 1,2,4,8]

A pass of rank r at world w = psx_run_exhaustive_async (its shard) + (w > 1)
one copy of the rank's partial image (read in place, psx_partials_device_ptr;
--export: exported first) standing in for the RCCL all-gather, merge_partials
+ psx_sync (the one host synchronisation: EXACT flag, status).  Nothing
overlaps the next pass: this is the latency of sweeping a locus once, which is
what the CLI and a real per-locus run see (the bench's pipelined passes hide
the merge and the exchange under the next pass's sweep).  Each (world, rank)
is timed in rounds that alternate the rank order; the line reports the
slowest rank's median and the speed-up over world 1.  Developer tool.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from pipsort_amd import engine as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syn1000c3")
    ap.add_argument("--passes", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--sync-api", action="store_true", help="psx_run_exhaustive (host readback per pass) instead")
    ap.add_argument("--export", action="store_true", help="export the image (a copy) instead of reading it in place")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    seam = bench.build_inputs(args.workload)
    stream = torch.cuda.Stream(priority=-1)
    torch.cuda.set_stream(stream)
    out = {"workload": args.workload, "mode": "sync_api" if args.sync_api else "async+sync", "worlds": {}}
    for world in [int(w) for w in args.worlds.split(",")]:
        pc = E.PostCal(seam, device=0)
        pc.set_stream(stream.cuda_stream)
        nb = pc.partials_bytes()
        mine = torch.empty(nb, dtype=torch.uint8, device="cuda") if args.export else pc.partials_tensor()
        gathered = torch.empty(nb * world, dtype=torch.uint8, device="cuda")
        tag_rank = (nb // 56 - 1) * 56 + 8
        rank_bytes = torch.arange(world, dtype=torch.int32, device="cuda").view(torch.uint8).view(world, 4)
        gv = gathered.view(world, nb)

        def one_pass():
            if args.sync_api:
                pc.run_exhaustive()
            else:
                pc.run_exhaustive_async()
            if world > 1:
                if args.export:
                    pc.export_partials(mine.data_ptr())
                gv.copy_(mine.view(1, nb).expand(world, nb))
                gv[:, tag_rank:tag_rank + 4].copy_(rank_bytes)
                pc.merge_partials(gathered.data_ptr(), world)
            assert not pc.sync()

        per = [[] for _ in range(world)]
        kern = [[] for _ in range(world)]
        for rd in range(args.rounds):
            order = range(world) if rd % 2 == 0 else range(world - 1, -1, -1)
            for rank in order:
                pc.set_shard(rank, world)
                for _ in range(3):
                    one_pass()
                torch.cuda.synchronize()
                for _ in range(args.passes):
                    t0 = time.perf_counter()
                    one_pass()
                    per[rank].append((time.perf_counter() - t0) * 1e3)
                    t = pc.timing()
                    kern[rank].append(t["kernel_ms"] / max(t["kernel_launches"], 1))
        pc.close()
        ranks = [{"rank": r, "pass_ms": statistics.median(per[r]), "kernel_ms": statistics.median(kern[r])}
                 for r in range(world)]
        worst = max(r["pass_ms"] for r in ranks)
        out["worlds"][world] = {"single_pass_ms": worst, "ranks": ranks}
        print(f"world {world}: single pass {worst:.3f} ms (slowest rank, median of {args.passes * args.rounds}); "
              f"pass ms per rank {[round(r['pass_ms'], 3) for r in ranks]}; "
              f"kernel ms per rank {[round(r['kernel_ms'], 3) for r in ranks]}", flush=True)
    base = out["worlds"].get(1, {}).get("single_pass_ms")
    if base:
        for w, d in out["worlds"].items():
            d["speedup"] = base / d["single_pass_ms"]
        print("speed-up over world 1: " + ", ".join(f"{w}: {d['speedup']:.2f}x" for w, d in out["worlds"].items()))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
