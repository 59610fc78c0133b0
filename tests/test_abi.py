"""C-ABI library: loads, exports every declared symbol, refuses to run without a
GPU, and its host-only helpers are exact.  CPU only (no compute calls)."""
import math
import os
import re
import subprocess

import numpy as np
import pytest

import loci
from pipsort_amd import engine as E
from pipsort_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in ("pipsort_engine.h", "pipsort_model.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"\b(psx_\w+)\s*\(", txt))
    return names


def test_library_exports_every_declared_symbol():
    lib = E.load_library()
    decl = _declared()
    assert decl == set(E.EXPORTED)
    dyn = subprocess.run(["nm", "-D", "--defined-only", E.LIB_PATH], capture_output=True, text=True).stdout
    for name in decl:
        assert re.search(rf"\bT {name}\b", dyn), name
        assert getattr(lib, name)
    assert lib.psx_abi_version() == 4  # 3: psx_timing.prepare_ms / run_ms, setup phases, partial-image PlanTag; 4: psx_partials_device_ptr


def test_no_cpu_fallback():
    if E.device_count() > 0:
        pytest.skip("a HIP device is present")
    seam, _ = loci.seam_for(loci.SMALL)
    with pytest.raises(E.EngineError) as ei:
        E.PostCal(seam)
    assert ei.value.code == E.PSX_ENODEV


def _count_seam(u2l, c):
    U = u2l.shape[1]
    m = np.array([(u2l[0] >= 0).sum(), (u2l[1] >= 0).sum()], dtype=np.int32)
    return E.Seam(m=m, B=np.zeros(1), s_prime=np.zeros(1), union_to_local=u2l,
                  sample_sizes=np.array([1, 1], dtype=np.int32), max_causal=c)


def test_configuration_counts_match_survey():
    L = loci.read_locus("example")
    assert _count_seam(L["u2l"], 2).count_configs() == 216_817
    for M, c, n in ((200, 2, 179_701), (500, 3, 560_253_751), (1000, 3, 4_491_007_501)):
        u2l = np.stack([np.arange(M), np.arange(M)]).astype(np.int32)
        assert _count_seam(u2l, c).count_configs() == n


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shards_partition_every_level(world):
    _, _, _, _, u2l = synth.mixed_locus(150, 170, 120, seed=3)
    U = u2l.shape[1]
    w = np.where((u2l[0] >= 0) & (u2l[1] >= 0), 3, 1)
    seam = _count_seam(u2l, 3)
    for k in (1, 2, 3):
        tot_sets, tot_cfg = 0, 0.0
        for r in range(world):
            s, c = seam.shard_stats(k, r, world)
            tot_sets += s
            tot_cfg += c
        assert tot_sets == math.comb(U, k)
        # e_k of the per-SNP pattern weights
        e = np.zeros(k + 1)
        e[0] = 1
        for x in w:
            e[1:] = e[1:] + e[:-1] * x
        assert abs(tot_cfg - e[k]) < 0.5


@pytest.mark.parametrize("U", [3, 63, 64, 65, 129, 1000])
@pytest.mark.parametrize("world", [1, 8])
def test_k3_block_pattern_plan_counts(U, world):
    """The k = 3 plan (off-diagonal tiles + folded diagonal tiles with a before,
    after or inside the block) covers C(U, 3) sets and sum 27 configurations
    per set for a fully shared locus, at block-boundary sizes."""
    u2l = np.stack([np.arange(U), np.arange(U)]).astype(np.int32)
    seam = _count_seam(u2l, 3)
    sets, cfg = 0, 0.0
    for r in range(world):
        s, c = seam.shard_stats(3, r, world)
        sets += s
        cfg += c
    assert sets == math.comb(U, 3)
    assert abs(cfg - 27 * math.comb(U, 3)) < 0.5


def _tagged(raw, rank, world, U=100, h=0x1234):
    """An image with its PlanTag slot (the last 56 bytes) set."""
    return np.frombuffer(bytes(raw[:-56]) + E.plan_tag(rank, world, U, h), dtype=np.uint8)


def test_partial_fold_is_associative_and_order_fixed():
    rng = np.random.default_rng(0)
    ldg = 128
    imgs = []
    for r in range(4):
        a = np.zeros(ldg + 2, dtype=E.ACC5_DTYPE)
        for f in ("mP", "mS", "mN"):
            a[f] = rng.integers(-3000, 3000, ldg + 2)
        for f in ("post0", "post1", "shared", "sll", "nsll"):
            a[f] = rng.random(ldg + 2) * (rng.random(ldg + 2) > 0.2)
        s = np.zeros(1, dtype=E.SETREC_DTYPE)
        s["m"], s["m0"], s["m1"] = rng.integers(-50, 50), -70, 3
        s["tot"], s["nc0"], s["nc1"], s["score"], s["npat"] = 1.5, 0.5, 0.25, -3.0, 7
        raw = a.tobytes()
        raw = raw[: ldg * 56] + s.tobytes() + E.plan_tag(r, 4, 100, 0x1234)
        imgs.append(np.frombuffer(raw, dtype=np.uint8))
    imgs = np.stack(imgs)
    full = E.fold_partials_host(imgs)
    # a fold is a world-1 image: the halves are re-tagged as shards 0 / 1 of 2
    pair = [np.stack([_tagged(imgs[i], 0, 2), _tagged(imgs[i + 1], 1, 2)]) for i in (0, 2)]
    halves = [_tagged(E.fold_partials_host(pair[0]), 0, 2), _tagged(E.fold_partials_host(pair[1]), 1, 2)]
    left = E.fold_partials_host(np.stack(halves))
    A = np.frombuffer(full[: ldg * 56].tobytes(), dtype=E.ACC5_DTYPE)
    B = np.frombuffer(left[: ldg * 56].tobytes(), dtype=E.ACC5_DTYPE)

    def val(x, m, s):
        return np.where(x[s] > 0, x[m] + np.log2(np.where(x[s] > 0, x[s], 1)), -np.inf)
    for m, s in (("mP", "post0"), ("mP", "post1"), ("mS", "sll"), ("mN", "nsll")):
        np.testing.assert_allclose(val(A, m, s), val(B, m, s), rtol=0, atol=1e-12)
    sa = np.frombuffer(full[ldg * 56: ldg * 56 + 56].tobytes(), dtype=E.SETREC_DTYPE)[0]
    assert sa["npat"] == 28 and sa["score"] == -3.0
    tag = np.frombuffer(full[-56:].tobytes(), dtype=E.PLANTAG_DTYPE)[0]
    assert (tag["magic"], tag["world"], tag["rank"], tag["hash"]) == (E.PLAN_MAGIC, 1, 0, 0x1234)


def test_mismatched_plan_images_are_refused():
    """Images of ranks that cut different plans (another hash: other PSX_K3_*
    knobs or build), out of rank order, of another world size, or without a
    tag are refused by the fold (the device merge checks the same tags)."""
    ldg = 64
    base = np.zeros((ldg + 2) * 56, dtype=np.uint8)
    good = [_tagged(base, r, 3) for r in range(3)]
    E.fold_partials_host(np.stack(good))
    bad_cases = {
        "hash": [good[0], good[1], _tagged(base, 2, 3, h=0x1235)],
        "order": [good[1], good[0], good[2]],
        "world": [good[0], good[1], _tagged(base, 2, 4)],
        "untagged": [good[0], good[1], base],
    }
    for name, imgs in bad_cases.items():
        with pytest.raises(E.EngineError, match="one plan"):
            E.fold_partials_host(np.stack(imgs))


def test_model_inputs_shape_helpers_without_gpu():
    """ModelInputs (the psx_create_from_ld route) exposes the same host-only
    helpers as Seam; creating an engine from it without a GPU fails loudly."""
    L = loci.read_locus("example")
    mi = E.model_inputs(L["ld"], L["z"], L["u2l"], (334324, 6771), max_causal=2, sharing_param=0.25)
    assert mi.count_configs() == 216_817
    assert mi.N == 441 and mi.n_union == L["u2l"].shape[1]
    if E.device_count() > 0:
        pytest.skip("a HIP device is present")
    with pytest.raises(E.EngineError) as ei:
        E.PostCal(mi)
    assert ei.value.code == E.PSX_ENODEV
    with pytest.raises(E.EngineError):
        E.lu_det(np.eye(3), gpu=True)


def test_host_lu_det_matches_numpy_and_underflows_like_gsl():
    rng = np.random.default_rng(1)
    a = rng.standard_normal((30, 30))
    assert math.isclose(E.lu_det(a), np.linalg.det(a), rel_tol=1e-10)
    idx = np.arange(1800)
    # index-order product of U_ii = 0.64 sticks at the smallest subnormal; 0.19 flushes to 0
    assert E.lu_det(0.6 ** np.abs(idx[:, None] - idx[None, :])) == 5e-324
    assert E.lu_det(0.9 ** np.abs(idx[:, None] - idx[None, :])) == 0.0


@pytest.mark.parametrize("U", [3, 65, 300, 1000])
@pytest.mark.parametrize("world", [1, 2, 8])
def test_k3_units_cover_every_walk_step_once(U, world):
    """The k = 3 work units of all shards cover every (a, tile, b-walk step) of
    the block-pattern decomposition exactly once (a units may split a b-walk:
    the ranges of one (a, tile) must tile [0, 64); the tail split cuts the last
    units into single-a units, PSX_K3_TAIL2 into half walks).  The a-chunk sizes
    are sized for 256 CUs whatever the device, so every rank cuts the same list."""
    ldg = (U + 63) // 64 * 64
    pad = ldg - U
    seen = {}
    n_units = 0
    for r in range(world):
        units = E.plan_units_k3(U, r, world)
        n_units += len(units)
        for a0, a1, z, w in units:
            K, C, j0, j1 = z & 0xFFFF, w & 0xFFFF, z >> 16, w >> 16
            assert K <= C and pad <= a0 < a1 and j0 < j1 <= 64
            if K == C:  # folded diagonal walk: half steps, even bounds
                assert j0 % 2 == 0 and j1 % 2 == 0
            for a in range(a0, a1):
                seen.setdefault((a, K, C), []).append((j0, j1))
    nblk = ldg // 64
    want = {(a, K, C) for C in range(nblk) if 64 * C + 64 > pad for K in range(C + 1)
            for a in range(pad, 64 * K if K < C else ldg)}
    assert set(seen) == want
    for key, ranges in seen.items():
        ranges.sort()
        assert ranges[0][0] == 0 and ranges[-1][1] == 64, (key, ranges)
        for (x0, x1), (y0, y1) in zip(ranges, ranges[1:]):
            assert x1 == y0, (key, ranges)
    assert n_units >= 1
