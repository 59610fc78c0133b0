"""Asynchronous exhaustive passes (psx_run_exhaustive_async + psx_sync): the
no-host-sync pipeline bench.py times.  Same results as the synchronous pass,
sharded exchange included, and the EXACT flag survives to psx_sync (and across
ranks through psx_merge_partials).  Marked gpu; run on an MI355X."""
import numpy as np
import pytest

from pipsort_amd import engine as E
from pipsort_amd import synth
from test_gpu_parity import _sexp

pytestmark = pytest.mark.gpu

FIELDS = ("post", "no_causal", "shared", "shared_ll", "notshared_ll")


def _inputs(M=300, c=3):
    ld, z, _, _, u2l = synth.mixed_locus(M, M + 20, M - 40, seed=M)
    return E.model_inputs(ld, z, u2l, (5000, 9000), max_causal=c, sharing_param=0.4)


@pytest.mark.parametrize("c", [2, 3])
def test_async_passes_bitwise_equal_sync(gpu, c):
    mi = _inputs(c=c)
    a = E.PostCal(mi)
    a.run_exhaustive()
    ra = a.accum()
    b = E.PostCal(mi)
    for _ in range(5):  # back-to-back passes, no host sync in between
        b.run_exhaustive_async()
    assert b.sync() is False
    t = b.timing()
    assert t["kernel_launches"] == 5 and t["kernel_ms"] > 0
    rb = b.accum()
    assert rb.n_configs == ra.n_configs and rb.total == ra.total
    for f in FIELDS:
        assert np.array_equal(getattr(ra, f), getattr(rb, f)), f


def test_async_ring_wraps(gpu):
    """More passes than the event ring holds (64) before one sync."""
    mi = _inputs(M=100, c=2)
    pc = E.PostCal(mi)
    for _ in range(150):
        pc.run_exhaustive_async()
    assert pc.sync() is False
    assert pc.timing()["kernel_launches"] == 150


@pytest.mark.parametrize("world", [2, 5, 8])
def test_async_sharded_exchange(gpu, world):
    """Sharded asynchronous passes with the exchange; at world >= 8 the handles
    overlap their passes on CU-masked streams by default (one XCD kept for the
    merges and the exchange), below it they do not."""
    import torch
    mi = _inputs()
    ref = E.PostCal(mi)
    ref.run_exhaustive()
    r = ref.accum()
    nb = ref.partials_bytes()
    stream = torch.cuda.Stream()
    buf = torch.empty(nb * world, dtype=torch.uint8, device="cuda")
    pcs = []
    for k in range(world):
        pc = E.PostCal(mi)
        pc.set_stream(stream.cuda_stream)
        pc.set_shard(k, world)
        pcs.append(pc)
    for step in range(2):
        for k, pc in enumerate(pcs):
            pc.run_exhaustive_async()
            pc.export_partials(buf.data_ptr() + k * nb)
        for pc in pcs:
            pc.merge_partials(buf.data_ptr(), world)
    for pc in pcs:
        assert pc.sync() is False
        assert (pc.overlap_cus() > 0) == (world >= 8), pc.overlap_cus()
        g = pc.accum()
        assert g.n_configs == r.n_configs
        for f in ("post", "no_causal", "shared"):
            d = np.abs(_sexp(getattr(g, f), g.total) - _sexp(getattr(r, f), r.total)).max()
            assert d <= 1e-12, f
        for f in ("shared_ll", "notshared_ll"):
            np.testing.assert_allclose(getattr(g, f), getattr(r, f), rtol=1e-12)


def _extreme():
    M = 80
    idx = np.arange(M)
    ld, z = [], []
    for s, rho in enumerate((0.5, 0.3)):
        sig = rho ** np.abs(idx[:, None] - idx[None, :])
        lam = np.zeros(M)
        lam[20] = 45.0
        lam[60] = 6.0 if s == 0 else 0.0
        eps = np.random.default_rng(9 + s).standard_normal(M)
        z.append(sig @ lam + np.linalg.cholesky(sig) @ eps)
        ld.append(sig)
    u2l = np.stack([idx, idx]).astype(np.int32)
    return E.model_inputs(ld, z, u2l, (12000, 9000), max_causal=3, sharing_param=0.3)


def test_async_reports_exact_flag_and_sync_path_recovers(gpu):
    import torch
    mi = _extreme()
    ref = E.PostCal(mi)
    ref.run_exhaustive()  # synchronous: reruns the exact variant itself
    assert ref.timing()["exact_rerun"] != 0
    r = ref.accum()
    assert ref.sync() is False  # handled: the sticky copy was cleared
    pc = E.PostCal(mi)
    pc.run_exhaustive_async()
    assert pc.sync() is True
    assert pc.sync() is False  # cleared by the previous sync
    pc.run_exhaustive()
    g = pc.accum()
    for f in FIELDS:
        assert np.array_equal(getattr(g, f), getattr(r, f)), f
    # across ranks: whichever shard raises the flag, after the exchange every rank sees it
    nb = pc.partials_bytes()
    buf = torch.empty(nb * 2, dtype=torch.uint8, device="cuda")
    ranks = []
    for k in range(2):
        x = E.PostCal(mi)
        x.set_shard(k, 2)
        x.run_exhaustive_async()
        x.export_partials(buf.data_ptr() + k * nb)
        ranks.append(x)
    torch.cuda.synchronize()
    flags = []
    for x in ranks:
        x.merge_partials(buf.data_ptr(), 2)
        flags.append(x.sync())
    assert flags == [True, True]


@pytest.mark.parametrize("c", [2, 3])
def test_overlapped_passes_bitwise_equal_sync(gpu, c, monkeypatch):
    """PSX_OVERLAP: consecutive asynchronous sweeps on two CU-masked compute
    streams (overlapping), merges on the reserved CUs: every pass still equals
    the synchronous one bit for bit, and the per-pass span is reported."""
    monkeypatch.setenv("PSX_OVERLAP", "8")
    mi = _inputs(c=c)
    a = E.PostCal(mi)
    a.run_exhaustive()
    ra = a.accum()
    b = E.PostCal(mi)
    for _ in range(7):
        b.run_exhaustive_async()
    assert b.sync() is False
    t = b.timing()
    assert t["kernel_launches"] == 7 and 0 < t["span_ms"] <= t["kernel_ms"]
    rb = b.accum()
    assert rb.n_configs == ra.n_configs and rb.total == ra.total
    for f in FIELDS:
        assert np.array_equal(getattr(ra, f), getattr(rb, f)), f
    a.close()
    b.close()
