"""Strong-scaling rehearsal on ONE GPU: time every rank's shard of the exhaustive
sweep for world = 1, 2, 4, 8 (one after another on the same device) and report
the slowest rank's step time, i.e. the step time an N-GPU node would see minus
the RCCL all-gather (latency-bound, ~56 KB per rank at M = 1000).

    python tools/shard_rehearsal.py [--workload syn1000c3] [--steps 10]

Each rank's step = run_exhaustive (its shard) + export_partials + merge of
`world` images (the gathered buffer is filled with this rank's image, which
costs the same to fold).  Developer tool (not the bench): prints one JSON line.
"""
import argparse
import json
import os
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=4,
                    help="timed rounds over the ranks, alternating forward / reverse rank order")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reverse", action="store_true", help="start the rounds in reverse rank order")
    ap.add_argument("--sync", action="store_true",
                    help="single passes: each step = async pass + exchange + psx_sync, nothing overlapping the next "
                         "(the latency of sweeping one locus once; tools/single_pass.py times each pass alone)")
    ap.add_argument("--no-exchange", action="store_true", help="world > 1 without the export / all-gather / merge")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    seam = bench.build_inputs(args.workload)
    stream = torch.cuda.Stream(priority=-1)  # high: merges + exchange ahead of the sweeps
    torch.cuda.set_stream(stream)
    out = {"workload": args.workload, "worlds": {}}
    for world in [int(w) for w in args.worlds.split(",")]:
        # One handle, its shard switched per rank, timed in rounds that alternate
        # the rank order: a rank measured first ran ~8 % slower than the same
        # shard measured later (r05q), whatever its rank.  (One handle per rank
        # put some ranks' compute streams on the hardware queue of the exchange
        # stream, GPU_MAX_HW_QUEUES = 4: +20-30 % on those ranks, r05s.)
        pc = E.PostCal(seam, device=0)
        pc.set_stream(stream.cuda_stream)
        nb = pc.partials_bytes()
        mine = torch.empty(nb, dtype=torch.uint8, device="cuda")
        gathered = torch.empty(nb * world, dtype=torch.uint8, device="cuda")
        # the copies of this rank's image stand in for ranks 0..world-1: their plan
        # tags (image slot ldg + 1: magic, world, rank, ...) get those ranks, or the
        # merge refuses them
        tag_rank = (nb // 56 - 1) * 56 + 8
        rank_bytes = torch.arange(world, dtype=torch.int32, device="cuda").view(torch.uint8).view(world, 4)

        def step(pc):
            pc.run_exhaustive_async()
            if world > 1 and not args.no_exchange:
                pc.export_partials(mine.data_ptr())
                # one copy kernel stands in for the RCCL all-gather
                gathered.view(world, nb).copy_(mine.view(1, nb).expand(world, nb))
                gathered.view(world, nb)[:, tag_rank:tag_rank + 4].copy_(rank_bytes)
                pc.merge_partials(gathered.data_ptr(), world)
            if args.sync:
                assert not pc.sync()

        acc = [{"step": [], "kernel": [], "sweep": [], "span": []} for _ in range(world)]
        for rd in range(args.rounds):
            fwd = (rd % 2 == 0) != args.reverse
            for rank in (range(world) if fwd else range(world - 1, -1, -1)):
                pc.set_shard(rank, world)
                for _ in range(3):
                    step(pc)
                torch.cuda.synchronize()
                pc.sync()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    step(pc)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) * 1e3 / args.steps
                assert not pc.sync()
                t = pc.timing()
                a = acc[rank]
                a["step"].append(dt)
                a["kernel"].append(t["kernel_ms"] / max(t["kernel_launches"], 1))
                a["sweep"].append(t["sweep_ms"])
                a["span"].append(t.get("span_ms", 0.0))
        ranks = [{"rank": r, "step_ms": sum(a["step"]) / len(a["step"]), "kernel_ms": sum(a["kernel"]) / len(a["kernel"]),
                  "sweep_ms": sum(a["sweep"]) / len(a["sweep"]), "span_ms": sum(a["span"]) / len(a["span"])}
                 for r, a in enumerate(acc)]
        pc.close()
        worst = max(r["step_ms"] for r in ranks)
        ks = [r["kernel_ms"] for r in ranks]
        out["worlds"][world] = {"max_step_ms": worst, "kernel_spread": max(ks) / min(ks) - 1.0, "ranks": ranks}
        print(f"world {world}: max step {worst:.3f} ms; kernel ms per rank "
              f"{[round(r['kernel_ms'], 3) for r in ranks]} (spread {100 * (max(ks) / min(ks) - 1):.1f} %); "
              f"step ms per rank {[round(r['step_ms'], 3) for r in ranks]}; "
              f"span ms per pass {[round(r['span_ms'], 3) for r in ranks]}; "
              f"sweep ms {[round(r['sweep_ms'], 3) for r in ranks]}",
              flush=True)
    base = out["worlds"].get(1, {}).get("max_step_ms")
    if base:
        for w, d in out["worlds"].items():
            d["predicted_speedup_excl_allgather"] = base / d["max_step_ms"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
