"""Several devices in one process (psx_multi_*, the drop-in CLI's PSX_DEVICES):
one shard per device entry, folded on the first device.  A test box has one
GPU, so the entries repeat device 0 — the same code path as a node, with the
peer copies replaced by same-device copies."""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

import loci
from oracle import oracle as O
from pipsort_amd import engine as E
from pipsort_amd import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _same(a, b, pip_tol=1e-12, ll_rtol=1e-12):
    assert a.n_configs == b.n_configs
    pa, na, sa = a.pips()
    pb, nb, sb = b.pips()
    assert max(np.abs(pa - pb).max(), np.abs(na - nb).max(), np.abs(sa - sb).max()) <= pip_tol
    for f in ("shared_ll", "notshared_ll"):
        np.testing.assert_allclose(getattr(a, f), getattr(b, f), rtol=ll_rtol, atol=0, err_msg=f)


@pytest.mark.parametrize("n", [2, 3])
def test_multi_handle_matches_single(gpu, n):
    """Exhaustive (fused k = 3 pass), configs file and the sharded SSS walk over
    n shards in one process equal one handle; the exhaustive result is also at
    oracle parity."""
    ld, z, _, _, u2l = synth.mixed_locus(70, 60, 40, seed=5)
    seam = E.seam_from_arrays(ld, z, u2l, (5000, 9000), max_causal=3, sharing_param=0.5)
    one = E.PostCal(seam)
    many = E.MultiPostCal(seam, [0] * n)
    one.run_exhaustive()
    many.run_exhaustive()
    _same(many.accum(), one.accum())
    ref = O.postcal(seam)
    got = many.accum()
    assert got.n_configs == ref["n_configs"]
    assert np.abs(got.pips()[0] - np.where(ref["post"] == 0, 0, np.exp(ref["post"] - ref["total"]))).max() <= 1e-9
    assert many.timing()["configs"] == got.n_configs
    rows = synth.all_configs_rows(seam.union_to_local, seam.m, 2)
    one.run_configs(rows)
    many.run_configs(rows)
    _same(many.accum(), one.accum())
    it1, itn = one.run_sss(), many.run_sss()
    assert it1 == itn
    _same(many.accum(), one.accum())
    one.close()
    many.close()


def test_multi_handle_gpu_setup(gpu):
    """psx_multi_create_from_ld: every device runs the Model setup (PSD shift
    LU, SYN-v1 M = 300), then the sharded sweep."""
    ld, z, _, _, u2l = synth.syn_v1(300)
    mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=3, sharing_param=0.25)
    one = E.PostCal(mi)
    many = E.MultiPostCal(mi, [0, 0])
    assert many.setup_info["psd_added"] == one.setup_info["psd_added"]
    one.run_exhaustive()
    many.run_exhaustive()
    _same(many.accum(), one.accum())


FILES = ("study0_post", "study1_post", "study0_set", "study1_set", "nocausal", "shared_pips")


def _cli(tmp_path, src, args, devices):
    d = tmp_path / f"{src}_{devices.replace(',', '_')}"
    shutil.copytree(os.path.join(loci.GOLDEN, src), d)
    env = dict(os.environ, PSX_DEVICES=devices)
    r = subprocess.run([E.PIPSORT_BIN] + args, cwd=d, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return d, r.stdout


@pytest.mark.parametrize("src,args", [
    ("example", ["-c", "2", "-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "snp_map", "-n", "334324,6771",
                 "-p", "0.25", "-o", "out"]),
    ("small_example", ["-q", "1", "-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "eur_afr_small_test_snp_map",
                       "-n", "7000,7000", "-o", "out"]),
    ("test_optional_configs", ["-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "eur_afr_small_test_snp_map",
                               "-n", "7000,7000", "-b", "all_configs_int16", "-d", "72", "-e", "5", "-o", "out"]),
])
def test_cli_two_devices_byte_identical(gpu, tmp_path, src, args):
    """The drop-in CLI driving two devices in one process (PSX_DEVICES=0,0)
    writes the same files, byte for byte, as one device; on tests/example those
    are the reference's expected files."""
    d1, _ = _cli(tmp_path, src, args, "0")
    d2, out2 = _cli(tmp_path, src, args, "0,0")
    assert "devices = 2" in out2
    for f in FILES:
        assert open(d2 / f"out_{f}.txt").read() == open(d1 / f"out_{f}.txt").read(), f
    if src == "example":
        for f in ("study0_post", "study1_post", "study0_set", "study1_set", "nocausal"):
            assert open(d2 / f"out_{f}.txt").read() == open(d2 / f"expected_{f}.txt").read(), f


@pytest.mark.parametrize("c", [1, 4])
def test_multi_count_off_the_fused_path(gpu, c):
    """max_causal 1 / 4 are not fused-pass shapes: each shard runs the
    synchronous sweep.  The folded count (timing) must still be every shard's,
    i.e. equal the merged accumulators' count and one handle's."""
    ld, z, _, _, u2l = synth.mixed_locus(40, 36, 28, seed=7)
    seam = E.seam_from_arrays(ld, z, u2l, (5000, 9000), max_causal=c, sharing_param=0.5)
    one = E.PostCal(seam)
    one.run_exhaustive()
    many = E.MultiPostCal(seam, [0, 0, 0])
    many.run_exhaustive()
    got = many.accum()
    _same(got, one.accum())
    assert got.n_configs == seam.count_configs()
    assert many.timing()["configs"] == got.n_configs
    one.close()
    many.close()


def test_multi_exact_rerun_matches_single_sync(gpu):
    """The extreme-signal locus raises the EXACT flag inside the asynchronous
    multi-shard pass, which then reruns the step synchronously on every shard:
    the folded result equals one synchronous handle (to rounding: a shard
    without a flagged set keeps the fast variant), the flag is
    reported and the count is the whole locus's."""
    from test_gpu_async import _extreme
    mi = _extreme()
    one = E.PostCal(mi)
    one.run_exhaustive()
    assert one.timing()["exact_rerun"] != 0
    r = one.accum()
    many = E.MultiPostCal(mi, [0, 0])
    many.run_exhaustive()
    g = many.accum()
    t = many.timing()
    assert t["exact_rerun"] != 0
    assert t["configs"] == g.n_configs == r.n_configs
    _same(g, r)  # shards without a flagged set keep the fast variant: equal to rounding
    one.close()
    many.close()


def _bitwise(a, b):
    """Every accumulator bit for bit (the 0-sentinel entries included)."""
    assert a.n_configs == b.n_configs
    for f in ("post", "no_causal", "shared", "shared_ll", "notshared_ll"):
        x, y = np.asarray(getattr(a, f)), np.asarray(getattr(b, f))
        assert np.array_equal(x.view(np.uint64), y.view(np.uint64)), f
    assert np.float64(a.total).view(np.uint64) == np.float64(b.total).view(np.uint64)


def _device_lists(n_dev):
    """Device lists the multi-device tests run: both orders of two devices, every
    device in order and reversed, and a repeated-device mix."""
    out = [[0, 1], [1, 0], list(range(min(n_dev, 8))), list(reversed(range(min(n_dev, 8)))), [1, 0, 1, 0]]
    uniq = []
    for d in out:
        if d not in uniq:
            uniq.append(d)
    return uniq


def test_multi_distinct_devices(gpu):
    """Shards on distinct devices (peer copies of the partial images into
    device 0's gather buffer over xGMI) give, for every device list, the SAME
    BITS as the same number of shards on one device (same plan, same rank-order
    fold: the result may not depend on which device ran a shard), and one
    handle's results to rounding.  Runs where the box has two or more GPUs (the
    driver's node); skipped on a one-GPU box, so this path is unverified until a
    multi-GPU run records it passing."""
    if E.device_count() < 2:
        pytest.skip("one device visible")
    ld, z, _, _, u2l = synth.syn_v1(300)
    seam = E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=3, sharing_param=0.25)
    one = E.PostCal(seam)
    one.run_exhaustive()
    ref = {}
    for devs in _device_lists(E.device_count()):
        n = len(devs)
        if n not in ref:
            same = E.MultiPostCal(seam, [0] * n)
            same.run_exhaustive()
            ref[n] = same.accum()
            same.close()
        many = E.MultiPostCal(seam, devs)
        many.run_exhaustive()
        g = many.accum()
        _bitwise(g, ref[n])
        _same(g, one.accum())
        assert many.timing()["configs"] == g.n_configs
        many.close()
    one.close()


def test_multi_device_lists_fold_identically_on_one_gpu(gpu):
    """The bitwise claim of test_multi_distinct_devices on a one-GPU box: two
    multi-handles with the same shard count fold to the same bits (the fold is
    deterministic, whatever ran first)."""
    ld, z, _, _, u2l = synth.syn_v1(200)
    seam = E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=3, sharing_param=0.25)
    a = E.MultiPostCal(seam, [0, 0, 0])
    a.run_exhaustive()
    b = E.MultiPostCal(seam, [0, 0, 0])
    b.run_exhaustive()
    b.run_exhaustive()
    _bitwise(a.accum(), b.accum())
    a.close()
    b.close()


def test_pool_trim_releases_cached_blocks(gpu):
    """Freed engine buffers stay cached for the next handle; psx_pool_trim gives
    them back (a co-resident framework can then allocate the memory)."""
    ld, z, _, _, u2l = synth.syn_v1(150)
    seam = E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=3, sharing_param=0.25)
    pc = E.PostCal(seam)
    pc.run_exhaustive()
    pc.close()
    assert E.pool_cached_bytes() > 0
    E.pool_trim()
    assert E.pool_cached_bytes() == 0
    pc = E.PostCal(seam)  # the pool refills from the runtime
    pc.run_exhaustive()
    assert pc.accum().n_configs == seam.count_configs()
    pc.close()


@pytest.mark.parametrize("mod", ["test_gpu_async.py", "test_gpu_dist.py::test_refused_merge_leaves_handle_usable"])
def test_poisoned_pool(gpu, mod):
    """The caching pool hands out recycled blocks with old contents: with
    PSX_POOL_POISON=1 every block comes filled with 0xFF bytes (NaN doubles,
    -1 ints), so code that relied on fresh memory being zero would fail here."""
    import subprocess
    env = dict(os.environ, PSX_POOL_POISON="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", mod)], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
