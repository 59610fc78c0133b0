"""N > 1 path on CPU with torch.distributed gloo, world_size 2: the config-shard
plan covers every union set exactly once across ranks, and the exchange step
(all-gather of partial accumulator images, folded in rank order) gives every
rank the same result as folding all images in one process."""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pipsort_amd import engine as E
from pipsort_amd import synth


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _image(rank, world=2, ldg=256):
    rng = np.random.default_rng(100 + rank)
    a = np.zeros(ldg + 2, dtype=E.ACC5_DTYPE)
    for f in ("mP", "mS", "mN"):
        a[f] = rng.integers(-2000, 2000, ldg + 2)
    for f in ("post0", "post1", "shared", "sll", "nsll"):
        a[f] = rng.random(ldg + 2) * (rng.random(ldg + 2) > 0.3)
    raw = bytearray(a.tobytes())
    s = np.zeros(1, dtype=E.SETREC_DTYPE)
    s["m"], s["m0"], s["m1"] = rank * 3, -rank, 2 * rank
    s["tot"], s["nc0"], s["nc1"], s["score"], s["npat"] = 1.0 + rank, 0.5, 0.25, -rank, 10 + rank
    raw[ldg * 56: ldg * 56 + s.itemsize] = s.tobytes()
    raw[(ldg + 1) * 56:] = E.plan_tag(rank, world, 200, 0xABC)
    return np.frombuffer(bytes(raw), dtype=np.uint8)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, _, _, _, u2l = synth.mixed_locus(150, 170, 120, seed=5)
        m = np.array([(u2l[0] >= 0).sum(), (u2l[1] >= 0).sum()], dtype=np.int32)
        seam = E.Seam(m=m, B=np.zeros(1), s_prime=np.zeros(1), union_to_local=u2l,
                      sample_sizes=np.array([1, 1], dtype=np.int32), max_causal=3)
        # 1) shard plan: sum over ranks of this rank's union sets / configurations
        cnt = []
        for k in (1, 2, 3):
            s, c = seam.shard_stats(k, rank, world)
            cnt += [float(s), c]
        t = torch.tensor(cnt, dtype=torch.float64)
        dist.all_reduce(t)
        # 2) exchange: all-gather this rank's partial image, fold in rank order
        mine = torch.from_numpy(_image(rank).copy())
        out = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(out, mine)
        folded = E.fold_partials_host(np.stack([o.numpy() for o in out]))
        q.put((rank, t.tolist(), folded.tobytes(), u2l.shape[1], seam.count_configs()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shard_and_exchange():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    U = res[0][3]
    tot = res[0][1]
    for k, (s, c) in zip((1, 2, 3), zip(tot[0::2], tot[1::2])):
        assert s == math.comb(U, k)
    assert abs(sum(tot[1::2]) + 1 - res[0][4]) < 0.5  # + null configuration
    # every rank folded the same bytes, equal to a single-process fold
    assert res[0][2] == res[1][2]
    single = E.fold_partials_host(np.stack([_image(r) for r in range(world)]))
    assert res[0][2] == single.tobytes()
