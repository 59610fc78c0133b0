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


def _sharded(seam, world, dev=False):
    """dev: psx_run_sss_sharded_dev, the all-gather on device buffers ordered on
    each rank's engine stream (here: copies through one shared device buffer,
    a barrier between the ranks' copy-in and copy-out)."""
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
    shared = torch.empty(world * (1 << 22), dtype=torch.uint8, device="cuda") if dev else None

    def gather(r):
        def ag(b):
            slots[r] = b
            bar.wait()
            out = b"".join(slots)
            bar.wait()
            return out
        return ag

    def gather_dev(r):
        n_call = [0]

        def ag(send, recv, nbytes, stream):
            # two shared buffers, alternating: a rank refills one only after the
            # next call's barrier, which every rank reaches after its engine
            # synchronised the copy-out of the previous use
            assert world * nbytes <= shared.numel() // 2
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
            iters[r] = (pcs[r].run_sss_sharded_dev(gather_dev(r)) if dev else
                        pcs[r].run_sss_sharded(gather(r)))
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


@pytest.mark.parametrize("dev", [False, True], ids=["host_exchange", "device_exchange"])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["small_c3", "example_c2", "syn60_c5"])
def test_sss_sharded_matches_single_walk_and_oracle(gpu, name, world, dev):
    seam = dict(_seams())[name]
    one = E.PostCal(seam)
    it1 = one.run_sss()
    single = one.accum()
    one.close()
    iters, got = _sharded(seam, world, dev)
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


def test_sss_sharded_dev_exchange_bitwise_host_exchange(gpu):
    """The device exchange walks the same path and folds the same values as
    the host-staged one: merged accumulators bitwise equal."""
    seam = dict(_seams())["syn60_c5"]
    ih, gh = _sharded(seam, 2, False)
    idv, gd = _sharded(seam, 2, True)
    assert ih == idv and gh.n_configs == gd.n_configs and gh.total == gd.total
    for f in ("post", "no_causal", "shared", "shared_ll", "notshared_ll"):
        assert np.array_equal(getattr(gh, f), getattr(gd, f)), f


def test_sss_sharded_dev_callback_error_is_reported(gpu):
    seam = dict(_seams())["small_c3"]
    pc = E.PostCal(seam)
    pc.set_shard(0, 2)

    def broken(*_a):
        raise RuntimeError("collective failed")

    with pytest.raises(RuntimeError, match="collective failed"):
        pc.run_sss_sharded_dev(broken)
    pc.close()
