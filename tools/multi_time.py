"""In-process multi-GPU exchange timing (psx_multi_*), developer tool.

    python tools/multi_time.py [--workload syn1000c3] [--devices 0,0,0,0,0,0,0,0] [--reps 10]

Times psx_multi_run_exhaustive over the device list (entries may repeat: on a
one-GPU box every shard shares device 0, so the shards' sweeps run concurrently
on one GPU) against the same shards run one after another on one handle
(psx_set_shard(r, n) + psx_run_exhaustive each, then one export / merge of the
n images), i.e. what the multi layer adds on top of the shards' own work: host
threads, per-shard exports into the gather buffer, the fold on the first
device.  Prints one JSON line.
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
    ap.add_argument("--devices", default="0,0,0,0,0,0,0,0")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    devs = [int(d) for d in args.devices.split(",")]
    n = len(devs)
    torch.cuda.set_device(0)
    mi = bench.build_inputs(args.workload)

    many = E.MultiPostCal(mi, devs)
    many.run_exhaustive()  # warm-up: plans, buffers
    t = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        many.run_exhaustive()
        t.append((time.perf_counter() - t0) * 1e3)
    multi_ms = sorted(t)[len(t) // 2]
    acc_multi = many.accum()
    many.close()

    one = E.PostCal(mi, device=devs[0])
    nb = one.partials_bytes()
    mine = torch.empty(nb, dtype=torch.uint8, device="cuda")
    gathered = torch.empty(nb * n, dtype=torch.uint8, device="cuda")

    def serial():
        for r in range(n):
            one.set_shard(r, n)
            one.run_exhaustive()
            one.export_partials(gathered[r * nb:].data_ptr())
        one.merge_partials(gathered.data_ptr(), n)
        torch.cuda.synchronize()

    def timed(f):
        f()
        t = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            f()
            t.append((time.perf_counter() - t0) * 1e3)
        return sorted(t)[len(t) // 2]

    serial_ms = timed(serial)
    acc_serial = one.accum()

    # the shard rehearsal's form (tools/shard_rehearsal.py): asynchronous passes
    # back to back on one handle, exports / merge ordered on the caller's stream
    stream = torch.cuda.Stream(priority=-1)
    torch.cuda.set_stream(stream)
    one.set_stream(stream.cuda_stream)

    def serial_async():
        for r in range(n):
            one.set_shard(r, n)
            one.run_exhaustive_async()
            one.export_partials(gathered[r * nb:].data_ptr())
        one.merge_partials(gathered.data_ptr(), n)
        torch.cuda.synchronize()
        assert not one.sync()

    serial_async_ms = timed(serial_async)
    one.close()
    same = bool((acc_multi.pips()[0] == acc_serial.pips()[0]).all()) and acc_multi.n_configs == acc_serial.n_configs
    out = {"workload": args.workload, "devices": devs, "multi_ms": multi_ms, "serial_shards_ms": serial_ms,
           "serial_async_shards_ms": serial_async_ms, "multi_over_serial": multi_ms / serial_ms,
           "multi_over_serial_async": multi_ms / serial_async_ms, "results_bit_identical": same,
           "note": "median of %d; multi = psx_multi_run_exhaustive (shards concurrent, exports from the shards' "
                   "threads, fold on the first device); serial = the same n shards one after another on one "
                   "handle + one merge; serial_async = the same with asynchronous passes (the shard rehearsal's step)" % args.reps}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
