"""Sharded SSS walk (psx_run_sss_sharded): `world` engines on one
device stand in for the ranks, in one thread each, their all-gather a barrier
over shared buffers (the bench / a real job binds it to torch.distributed).
Every rank must walk the same path as the single-GPU walk, and the merged
accumulators must match the oracle's SSS (sss_postcal.cpp:102-380).  Marked
gpu; run on an MI355X."""
import threading

import numpy as np
import pytest

import loci
from oracle import oracle as O
from pipsort_amd import engine as E
from pipsort_amd import synth
from test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


def _sharded(seam, world):
    import torch

    pcs = []
    for r in range(world):
        pc = E.PostCal(seam)
        pc.set_shard(r, world)
        pcs.append(pc)
    bar = threading.Barrier(world, timeout=60)
    slots = [None] * world
    iters = [None] * world
    errs = []

    def gather(r):
        def ag(b):
            slots[r] = b
            bar.wait()
            out = b"".join(slots)
            bar.wait()
            return out
        return ag

    def run(r):
        try:
            iters[r] = pcs[r].run_sss_sharded(gather(r))
        except BaseException as ex:  # noqa: BLE001
            errs.append(ex)
            bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    nb = pcs[0].partials_bytes()
    buf = torch.empty(nb * world, dtype=torch.uint8, device="cuda")
    for r, pc in enumerate(pcs):
        pc.export_partials(buf.data_ptr() + r * nb)
    torch.cuda.synchronize()
    pcs[0].merge_partials(buf.data_ptr(), world)
    got = pcs[0].accum()
    for pc in pcs:
        pc.close()
    return iters, got


def _seams():
    out = [("small_c3", loci.seam_for(loci.SMALL, c=3)[0]), ("example_c2", loci.seam_for(loci.EXAMPLE, c=2)[0])]
    ld, z, _, _, u2l = synth.syn_v1(60)
    out.append(("syn60_c5", E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=5, sharing_param=0.25)))
    return out


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["small_c3", "example_c2", "syn60_c5"])
def test_sss_sharded_matches_single_walk_and_oracle(gpu, name, world):
    seam = dict(_seams())[name]
    one = E.PostCal(seam)
    it1 = one.run_sss()
    single = one.accum()
    one.close()
    iters, got = _sharded(seam, world)
    assert iters == [it1] * world  # the same walk on every rank
    assert got.n_configs == single.n_configs
    assert_parity(got, O.postcal(seam, "sss"), ll_rtol=1e-11)


def test_sss_sharded_callback_error_is_reported(gpu):
    seam = dict(_seams())["small_c3"]
    pc = E.PostCal(seam)
    pc.set_shard(0, 2)

    def broken(_b):
        raise RuntimeError("collective failed")

    with pytest.raises(RuntimeError, match="collective failed"):
        pc.run_sss_sharded(broken)
    pc.close()


def test_sss_sharded_world1_is_run_sss(gpu):
    seam = dict(_seams())["small_c3"]
    a = E.PostCal(seam)
    ia = a.run_sss()
    ra = a.accum()
    b = E.PostCal(seam)
    ib = b.run_sss_sharded(lambda x: x)
    rb = b.accum()
    assert ia == ib and ra.n_configs == rb.n_configs
    for f in ("post", "no_causal", "shared", "shared_ll", "notshared_ll"):
        assert np.array_equal(getattr(ra, f), getattr(rb, f)), f
    a.close()
    b.close()
