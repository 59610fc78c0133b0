"""Sharded SSS walk rehearsal on ONE GPU: the M = 200 c = 5 SYN-v1 walk (and
BASELINE configs[4], M = 2000) at world 1 (psx_run_sss) and at world 2 with two
rank threads on the same device, their per-iteration all-gather either
host-staged (psx_run_sss_sharded: scores D2H, bytes, H2D) or kept on the device
(psx_run_sss_sharded_dev: pack -> copies through two alternating shared device buffers on
each rank's engine stream -> unpack), the walk time per rank (median of reps).
On one device the two ranks share the GPU, so this checks the exchange path's
cost and correctness (same walk, same accumulators), not a speed-up: the
threads' Python callbacks and barriers (GIL) dominate both exchange forms here;
with RCCL the device form's callback only enqueues the collective.

    python tools/sss_shard_rehearsal.py [--reps 5]
"""
import argparse
import os
import statistics
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402


def walk_world2(seam, dev, reps):
    world = 2
    pcs = []
    for r in range(world):
        pc = E.PostCal(seam)
        pc.set_shard(r, world)
        pcs.append(pc)
    bar = threading.Barrier(world, timeout=60)
    slots = [None] * world
    shared = torch.empty(world * (1 << 22), dtype=torch.uint8, device="cuda")
    times = [[] for _ in range(world)]
    iters = [None] * world
    errs = []

    def ag_host(r):
        def ag(b):
            slots[r] = b
            bar.wait()
            out = b"".join(slots)
            bar.wait()
            return out
        return ag

    def ag_dev(r):
        n_call = [0]

        def ag(send, recv, nbytes, stream):
            # two shared buffers, alternating (see tests/test_gpu_sss_shard.py)
            buf = shared[(n_call[0] % 2) * (shared.numel() // 2):]
            n_call[0] += 1
            ext = torch.cuda.ExternalStream(stream)
            with torch.cuda.stream(ext):
                buf[r * nbytes:(r + 1) * nbytes].copy_(E.device_bytes(send, nbytes))
            ext.synchronize()
            bar.wait()
            with torch.cuda.stream(ext):  # enqueued: the engine's stream orders it
                E.device_bytes(recv, world * nbytes).copy_(buf[:world * nbytes])
        return ag

    def run(r):
        try:
            torch.cuda.set_device(0)
            f = ag_dev(r) if dev else ag_host(r)
            for i in range(reps + 1):
                bar.wait()
                t0 = time.perf_counter()
                iters[r] = pcs[r].run_sss_sharded_dev(f) if dev else pcs[r].run_sss_sharded(f)
                if i:
                    times[r].append((time.perf_counter() - t0) * 1e3)
        except BaseException as ex:  # noqa: BLE001
            errs.append(ex)
            bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errs, errs
    nb = pcs[0].partials_bytes()
    buf = torch.empty(nb * world, dtype=torch.uint8, device="cuda")
    for r, pc in enumerate(pcs):
        pc.export_partials(buf.data_ptr() + r * nb)
    torch.cuda.synchronize()
    pcs[0].merge_partials(buf.data_ptr(), world)
    acc = pcs[0].accum()
    for pc in pcs:
        pc.close()
    return iters, [statistics.median(t) for t in times], acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sizes", default="200,2000")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    for M in [int(x) for x in a.sizes.split(",")]:
        ld, z, _, _, u2l = synth.syn_v1(M)
        seam = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=5, sharing_param=0.25)
        pc = E.PostCal(seam)
        ws = []
        for i in range(a.reps + 1):
            t0 = time.perf_counter()
            it1 = pc.run_sss()
            if i:
                ws.append((time.perf_counter() - t0) * 1e3)
        one = pc.accum()
        pc.close()
        print(f"M={M} c=5 world 1: {it1} iterations, walk {statistics.median(ws):.2f} ms (median of {a.reps})",
              flush=True)
        for dev in (False, True):
            iters, t, acc = walk_world2(seam, dev, a.reps)
            same = acc.n_configs == one.n_configs and all(
                np.allclose(getattr(acc, f), getattr(one, f), rtol=1e-11, atol=0)
                for f in ("post", "no_causal", "shared", "shared_ll", "notshared_ll"))
            print(f"M={M} c=5 world 2 ({'device' if dev else 'host-staged'} exchange): iterations {iters}, "
                  f"walk ms per rank {[round(x, 2) for x in t]}; merged accumulators match world 1: {same}",
                  flush=True)


if __name__ == "__main__":
    main()
