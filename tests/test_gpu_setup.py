"""GPU Model setup (psx_create_from_ld; model.h:171-264, util.cpp:195-263).

* The PSD-shift determinant on the GPU is bit-identical to the host
  restatement of GSL's elimination (model.cpp lu_det), including the
  index-order product's underflow behaviour.
* PostCal built from LD + z on the GPU (no eigendecomposition when Sigma' is
  positive definite) matches PostCal built from the reference's own low-rank
  B / S' (host eigen route) and the oracle.
Marked gpu; run on an MI355X."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import loci
from oracle import oracle as O
from pipsort_amd import engine as E
from pipsort_amd import synth
from test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


def _bits(x):
    return np.float64(x).view(np.uint64)


def _det_cases():
    rng = np.random.default_rng(5)
    cases = {
        "n1": np.array([[0.3]]),
        "n2_swap": np.array([[1e-3, 2.0], [3.0, 4.0]]),
        "rand64": rng.standard_normal((64, 64)),
        "rand257": rng.standard_normal((257, 257)),
        "ties": rng.integers(-3, 4, (96, 96)).astype(np.float64),  # equal |pivots|: first one wins
        "singular": np.ones((40, 40)),
        "ar1_sticky": 0.6 ** np.abs(np.arange(2000)[:, None] - np.arange(2000)[None, :]),  # sticks at 5e-324
        "ar1_zero": 0.9 ** np.abs(np.arange(1200)[:, None] - np.arange(1200)[None, :]),  # underflows to 0
    }
    for d in ("example", "small_example"):
        L = loci.read_locus(d)
        for s in range(2):
            cases[f"{d}{s}"] = L["ld"][s]
            cases[f"{d}{s}_shift"] = L["ld"][s] + 0.01 * np.eye(L["ld"][s].shape[0])
    return cases


@pytest.mark.parametrize("name", sorted(_det_cases()))
def test_lu_det_bit_identical(gpu, name):
    a = _det_cases()[name]
    h = E.lu_det(a)
    g = E.lu_det(a, gpu=True)
    assert _bits(h) == _bits(g), (name, h, g)


@pytest.mark.parametrize("d", ["example", "small_example"])
def test_psd_shift_gpu_matches_host(gpu, d):
    L = loci.read_locus(d)
    for s in range(2):
        sh, ah = E.psd_shift(L["ld"][s])
        sg, ag = E.psd_shift_gpu(L["ld"][s])
        assert ah == ag
        assert np.array_equal(sh, sg)


def _both(ld, z, u2l, n, **kw):
    seam = E.seam_from_arrays(ld, z, u2l, n, **kw)
    mi = E.model_inputs(ld, z, u2l, n, **kw)
    return seam, mi


def _run(x):
    pc = E.PostCal(x)
    pc.run_exhaustive()
    return pc, pc.accum()


@pytest.mark.parametrize("spec", ["example", "small_example"])
def test_ld_route_matches_eigen_route(gpu, spec):
    sp = loci.EXAMPLE if spec == "example" else loci.SMALL
    L = loci.read_locus(sp["dirname"])
    seam, mi = _both(L["ld"], L["z"], L["u2l"], sp["n"], max_causal=sp["c"], sharing_param=sp["p"])
    pc, got = _run(mi)
    info = pc.setup_info
    assert info["eigen_route"] == [0, 0]
    for s in range(2):
        assert info["psd_added"][s] == E.psd_shift(L["ld"][s])[1]
    assert_parity(got, O.postcal(seam), pip_tol=1e-9, ll_rtol=1e-9)
    _, ref = _run(seam)
    assert_parity(got, ref.__dict__, pip_tol=1e-9, ll_rtol=1e-9)


@pytest.mark.parametrize("M0,M1,shared,c", [(90, 110, 60, 3), (130, 70, 5, 2), (1, 3, 1, 3)])
def test_ld_route_mixed_loci(gpu, M0, M1, shared, c):
    ld, z, _, _, u2l = synth.mixed_locus(M0, M1, shared, seed=M0 + M1)
    seam, mi = _both(ld, z, u2l, (5000, 9000), max_causal=c, sharing_param=0.5)
    _, got = _run(mi)
    assert_parity(got, O.postcal(seam), pip_tol=1e-9, ll_rtol=1e-9)


def test_ld_route_syn1000(gpu):
    """The bench locus: GPU setup vs host eigen route, full sweep, PIPs 1e-9."""
    ld, z, _, _, u2l = synth.syn_v1(1000)
    seam, mi = _both(ld, z, u2l, (10000, 8000), max_causal=2, sharing_param=0.25)
    pc, got = _run(mi)
    assert pc.setup_info["eigen_route"] == [0, 0]
    _, ref = _run(seam)
    assert_parity(got, ref.__dict__, pip_tol=1e-9, ll_rtol=1e-9)


def test_ld_route_fused_lu_shift_loop_and_asymmetric(gpu):
    """The swap-free fused elimination (blocked panels, z's forward
    solve riding along, step 2 skipped for an exactly symmetric LD):
    * study 0: AR(1) rho = 0.95, M = 400, whose determinant underflows to 0,
      so util.cpp:195-226 adds 0.01 several times; the shift must equal the
      host restatement of GSL's elimination exactly;
    * study 1: a symmetric LD with one upper entry moved by one ulp (not
      exactly symmetric: step 2 runs on the lower triangle, as the reference's
      eigensolver reads it).
    PIPs against the host eigen route."""
    M = 400
    idx = np.arange(M)
    ar = 0.95 ** np.abs(idx[:, None] - idx[None, :])
    assert E.lu_det(ar) == 0.0  # the loop must iterate
    ld1 = 0.5 ** np.abs(idx[:, None] - idx[None, :])
    ld1[3, 17] = np.nextafter(ld1[3, 17], 1.0)
    rng = np.random.default_rng(9)
    z = [rng.standard_normal(M) * 1.5, rng.standard_normal(M) * 1.5]
    z[0][M // 2] = 5.0
    z[1][M // 2] = 4.0
    u2l = np.stack([idx, idx]).astype(np.int32)
    seam, mi = _both([ar, ld1], z, u2l, (6000, 7000), max_causal=2, sharing_param=0.25)
    pc, got = _run(mi)
    info = pc.setup_info
    assert info["eigen_route"] == [0, 0]
    assert info["psd_added"][0] == E.psd_shift(ar)[1] > 0
    assert info["psd_added"][1] == E.psd_shift(ld1)[1]
    _, ref = _run(seam)
    assert_parity(got, ref.__dict__, pip_tol=1e-9, ll_rtol=1e-9)


def test_indefinite_sigma_takes_eigen_route(gpu):
    """det > 0 with two negative eigenvalues: the PSD loop stops at a = 0 and the
    reference's |W| differs from Sigma'; the engine must take the eigen route."""
    rng = np.random.default_rng(3)
    M = 40
    q, _ = np.linalg.qr(rng.standard_normal((M, M)))
    w = np.linspace(0.2, 3.0, M)
    w[:2] = [-0.3, -0.5]
    sig = (q * w) @ q.T
    sig = (sig + sig.T) / 2
    assert E.lu_det(sig) > 0
    ld = [sig, 0.5 ** np.abs(np.arange(M)[:, None] - np.arange(M)[None, :])]
    z = [rng.standard_normal(M) * 2, rng.standard_normal(M) * 2]
    u2l = np.stack([np.arange(M), np.arange(M)]).astype(np.int32)
    seam, mi = _both(ld, z, u2l, (6000, 7000), max_causal=2, sharing_param=0.4)
    pc, got = _run(mi)
    assert pc.setup_info["eigen_route"] == [1, 0]
    assert_parity(got, O.postcal(seam), pip_tol=1e-9, ll_rtol=1e-9)


def _indefinite(M, seed):
    """A symmetric Sigma with two negative eigenvalues and det > 0 (the PSD loop
    of util.cpp:195-226 stops at a = 0, so the eigen route must take |W|)."""
    rng = np.random.default_rng(seed)
    q, _ = np.linalg.qr(rng.standard_normal((M, M)))
    w = np.linspace(0.05, 4.0, M)
    w[:2] = [-0.3, -0.5]
    sig = (q * w) @ q.T
    return (sig + sig.T) / 2, rng


def test_indefinite_sigma_gpu_eigen_route_m500(gpu):
    """The eigen route on the GPU (rocSOLVER dsyevd, psx_eigen.hip) at M = 500:
    PIPs and LL columns of the host route's seam (the restated model.h:213-259
    eigen route) through the oracle."""
    M = 500
    sig, rng = _indefinite(M, 11)
    assert E.lu_det(sig) > 0
    ld = [sig, 0.5 ** np.abs(np.arange(M)[:, None] - np.arange(M)[None, :])]
    z = [rng.standard_normal(M) * 2, rng.standard_normal(M) * 2]
    z[0][M // 3] += 6.0
    u2l = np.stack([np.arange(M), np.arange(M)]).astype(np.int32)
    seam, mi = _both(ld, z, u2l, (6000, 7000), max_causal=2, sharing_param=0.4)
    pc, got = _run(mi)
    assert pc.setup_info["eigen_route"] == [1, 0]
    assert_parity(got, O.postcal(seam), pip_tol=1e-9, ll_rtol=1e-9)


def test_indefinite_sigma_m1000_sets_up_under_a_second(gpu):
    """An indefinite M = 1000 LD through the GPU eigen route: the whole Model
    setup + PostCal construction (psx_create_from_ld) in < 1 s."""
    M = 1000
    sig, rng = _indefinite(M, 12)
    ld = [sig, 0.5 ** np.abs(np.arange(M)[:, None] - np.arange(M)[None, :])]
    z = [rng.standard_normal(M), rng.standard_normal(M)]
    u2l = np.stack([np.arange(M), np.arange(M)]).astype(np.int32)
    mi = E.model_inputs(ld, z, u2l, (6000, 7000), max_causal=2, sharing_param=0.4)
    E.PostCal(mi).close()  # first create of the process: runtime / library start-up
    pc = E.PostCal(mi)
    assert pc.setup_info["eigen_route"] == [1, 0]
    assert pc.setup_info["setup_ms"] < 1000.0, pc.setup_info


def test_cli_host_setup_route_still_reproduces_goldens(gpu, tmp_path):
    """PSX_HOST_SETUP=1 keeps the reference's eigen route in the drop-in CLI."""
    d = tmp_path / "example"
    shutil.copytree(os.path.join(loci.GOLDEN, "example"), d)
    env = dict(os.environ, PSX_HOST_SETUP="1")
    r = subprocess.run([E.PIPSORT_BIN, "-c", "2", "-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "snp_map", "-n",
                        "334324,6771", "-p", "0.25", "-o", "pipsort_results"], cwd=d, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Time for eigen decomp" in r.stdout
    for f in ("study0_post", "study1_post", "study0_set", "study1_set", "nocausal"):
        assert open(d / f"pipsort_results_{f}.txt").read() == open(d / f"expected_{f}.txt").read(), f


def test_example_pipeline_end_to_end(gpu, tmp_path):
    """tests/example/run_example.sh end to end with the drop-in pieces: PIPSORT
    (GPU setup + sweep) then global / not-shared PIPs; the post-processed files
    equal what the reference's utils make from the reference's expected files."""
    from pipsort_amd import postprocess as PP
    d = tmp_path / "example"
    shutil.copytree(os.path.join(loci.GOLDEN, "example"), d)
    r = subprocess.run([E.PIPSORT_BIN, "-c", "2", "-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "snp_map", "-n",
                        "334324,6771", "-p", "0.25", "-o", "pipsort_results"], cwd=d, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    PP.global_pips(str(d / "pipsort_results_study0_post.txt"), str(d / "pipsort_results_study1_post.txt"),
                   str(d / "pipsort_results_shared_pips.txt"), str(d / "global_pips.txt"))
    PP.not_shared_pips(str(d / "pipsort_results_shared_pips.txt"), str(d / "global_pips.txt"),
                       str(d / "not_shared_pips.txt"))
    gold = os.path.join(loci.GOLDEN, "postprocess")
    g = [l.split("\t") for l in (d / "global_pips.txt").read_text().splitlines()]
    e = [l.split("\t") for l in open(os.path.join(gold, "example_global_pips.txt")).read().splitlines()]
    assert [x[0] for x in g] == [x[0] for x in e]
    # global PIPs column: from byte-identical post / shared-PIP files -> identical
    assert [x[3] for x in g] == [x[3] for x in e]
    # LL columns: race-affected in the reference (postcal.cpp:1012-1017), 1 line may differ
    bad = sum(1 for x, y in zip(g[1:], e[1:]) if x[1:3] != y[1:3])
    assert bad <= 1


def test_warmup_entry_point(gpu):
    """psx_warmup (the CLI overlaps it with input parsing): brings the device up
    and loads device code; a bad device index is an
    error, not a crash; the engine works afterwards."""
    lib = E.load_library()
    assert lib.psx_warmup(0) == E.PSX_OK
    assert lib.psx_warmup(E.device_count() + 3) == E.PSX_EINVAL
    seam, _ = loci.seam_for(loci.SMALL, c=2)
    pc = E.PostCal(seam)
    pc.run_exhaustive()
    assert_parity(pc.accum(), O.postcal(seam))


def _elim_pivots(a):
    """Host restatement of the swap-free right-looking elimination (GSL's
    operation order: l = a_ij / a_jj, then a_ik - l * u_jk, not fused; a zero
    pivot skips the column): the U diagonal."""
    a = np.array(a, dtype=np.float64, copy=True)
    n = a.shape[0]
    for j in range(n - 1):
        if a[j, j] == 0.0:
            continue
        l = a[j + 1:, j] / a[j, j]
        a[j + 1:, j + 1:] -= np.outer(l, a[j, j + 1:])
    return np.diag(a).copy()


def _elim_spsq(a, z):
    """||S'||^2 of the setup's step 2: the same unpivoted elimination with z's
    forward solve riding along (z_i - l_ij z_j, unfused), then sum z~_i^2 / D_i
    in index order."""
    a = np.array(a, dtype=np.float64)
    z = np.array(z, dtype=np.float64)
    n = a.shape[0]
    for j in range(n - 1):
        l = a[j + 1:, j] / a[j, j]
        a[j + 1:, j + 1:] -= np.outer(l, a[j, j + 1:])
        z[j + 1:] -= l * z[j]
    piv = np.diag(a)
    q = 0.0
    for i in range(n):
        q += float(z[i]) * float(z[i]) / float(piv[i])
    return q


def _elim(a, z, check=True):
    """Host restatement of the tiled kernels' contract (psx_elim_gpu): the
    per-column elimination without pivoting (a zero pivot skips its step, as
    GSL does), z's forward solve riding along, and whether GSL's pivot search
    would have swapped some row (some |a_ij| > |a_jj| below the diagonal, NaNs
    never chosen)."""
    a = np.array(a, dtype=np.float64, copy=True)
    z = np.array(z, dtype=np.float64, copy=True)
    n = a.shape[0]
    swap = False
    for j in range(n - 1):
        if check and a[j, j] == a[j, j] and (np.abs(a[j + 1:, j]) > abs(a[j, j])).any():
            swap = True
        if a[j, j] == 0.0:
            continue
        l = a[j + 1:, j] / a[j, j]
        a[j + 1:, j + 1:] -= np.outer(l, a[j, j + 1:])
        z[j + 1:] -= l * z[j]
    return np.diag(a).copy(), z, swap


def _tiled_cases():
    cases = []
    for n in (1, 2, 15, 16, 17, 31, 32, 33, 63, 64, 65, 79, 80, 81, 96, 97, 129, 200, 333):
        idx = np.arange(n)
        rng = np.random.default_rng(n)
        a = 0.9 ** np.abs(idx[:, None] - idx[None, :]) + 0.01 * rng.standard_normal((n, n))
        a[idx, idx] += 0.5
        cases.append((f"ld{n}", a))
    # zero pivots (steps skipped, no swap needed: the column below is zero too)
    n = 70
    a = np.eye(n) * 2.0 + 0.1 * np.random.default_rng(7).standard_normal((n, n))
    for j in (3, 16, 17, 40, 69):
        a[j, :] = 0.0
        a[:, j] = 0.0
    cases.append(("zero-pivots", a))
    # a row swap needed in a diagonal block, and one below it (check mode flags both)
    b = cases[13][1].copy()  # n = 81
    b[5, 2] = 10.0
    cases.append(("swap-in-block", b))
    c = cases[13][1].copy()
    c[70, 20] = 10.0
    cases.append(("swap-below-block", c))
    return cases


@pytest.mark.parametrize("name,a", _tiled_cases(), ids=[c[0] for c in _tiled_cases()])
def test_tiled_elimination_bit_identical(gpu, name, a):
    """The tiled swap-free elimination (k_lu_diag + one k_lu_tile per 16-column
    panel, every tile recomputing its rows' L chains and columns' U solves from
    the published diagonal block) gives every pivot U_ii and every z~_i of the
    per-column elimination bit for bit, on sizes around the panel / tile edges,
    with skipped (zero) pivots, and raises the swap flag exactly when GSL's
    pivot search would swap; with the check off (the setup's step 2) the
    pivots are the unpivoted elimination's."""
    z = np.random.default_rng(11).standard_normal(a.shape[0])
    for check in (True, False):
        piv, zt, sw = E.elim_gpu(a, z, check=check)
        hp, hz, hs = _elim(a, z, check=check)
        assert sw == hs, (name, check, sw, hs)
        if sw:
            continue
        assert np.array_equal(piv.view(np.uint64), hp.view(np.uint64)), (name, check, np.flatnonzero(piv != hp)[:5])
        assert np.array_equal(zt.view(np.uint64), hz.view(np.uint64)), (name, check, np.flatnonzero(zt != hz)[:5])


@pytest.mark.parametrize("M", [1, 2, 15, 16, 17, 33, 300, 1000, 2000])
def test_blocked_swap_free_elimination_bit_identical(gpu, M):
    """The tiled swap-free elimination of psx_setup.hip gives the per-column
    elimination's pivots bit for bit inside the setup: the setup's min pivot
    ratio equals the host restatement's exactly, on sizes around the 16-column
    panel and on the SYN-v1 LDs."""
    if M >= 1000:
        ld, z, _, _, u2l = synth.syn_v1(M)
    else:
        idx = np.arange(M)
        a0 = 0.95 ** np.abs(idx[:, None] - idx[None, :])
        a1 = 0.5 ** np.abs(idx[:, None] - idx[None, :])
        rng = np.random.default_rng(M)
        ld = [a0, a1]
        z = [rng.standard_normal(M), rng.standard_normal(M)]
        u2l = np.stack([idx, idx]).astype(np.int32)
    mi = E.model_inputs(ld, z, u2l, (6000, 7000), max_causal=1, sharing_param=0.25)
    pc = E.PostCal(mi)
    info = pc.setup_info
    for s in range(2):
        add = E.psd_shift(ld[s])[1]
        assert info["psd_added"][s] == add
        if info["eigen_route"][s]:
            continue
        a = ld[s] + add * np.eye(ld[s].shape[0])
        piv = _elim_pivots(a)
        dmax = np.abs(np.diag(a)).max()
        assert info["min_pivot_ratio"][s] == piv.min() / dmax, (s, info["min_pivot_ratio"][s], piv.min() / dmax)
        # the tiled kernels alone: no swap flagged (more tiles than resident blocks
        # at M >= 1000) and every pivot bit for bit
        gp, _, sw = E.elim_gpu(a)
        assert not sw and np.array_equal(gp.view(np.uint64), piv.view(np.uint64)), (s, sw)
        if M <= 300:  # z's forward solve (it feeds K = -||S'||^2 / 2): bit-identical too
            assert _bits(info["spsq"][s]) == _bits(_elim_spsq(a, z[s])), (s, info["spsq"][s], _elim_spsq(a, z[s]))
    pc.close()


@pytest.mark.parametrize("M0,M1", [(17, 300), (300, 33), (1000, 129), (1, 64)])
def test_joint_study_elimination_bit_identical(gpu, M0, M1):
    """The two studies' first elimination runs in joint launches (one
    k_lu_step per panel index for both matrices, blockIdx.z = study; the grid
    covers the larger one and the smaller study's blocks past its trailing part
    return).  Studies of different sizes: each study's shift, min pivot ratio
    and (M <= 300) ||S'||^2 equal the host restatement's bit for bit."""
    lds, zs = [], []
    rng = np.random.default_rng(M0 * 7 + M1)
    for M, r in ((M0, 0.6), (M1, 0.8)):  # determinants > 0 at these sizes: no shift
        idx = np.arange(M)
        lds.append(r ** np.abs(idx[:, None] - idx[None, :]))
        zs.append(rng.standard_normal(M) * 1.5)
    U = max(M0, M1)
    u2l = -np.ones((2, U), dtype=np.int32)
    u2l[0, :M0] = np.arange(M0)
    u2l[1, :M1] = np.arange(M1)
    mi = E.model_inputs(lds, zs, u2l, (6000, 7000), max_causal=1, sharing_param=0.25)
    pc = E.PostCal(mi)
    info = pc.setup_info
    for s in range(2):
        a = lds[s]
        assert info["eigen_route"][s] == 0 and info["psd_added"][s] == E.psd_shift(a)[1] == 0.0
        piv = _elim_pivots(a)
        assert info["min_pivot_ratio"][s] == piv.min() / np.abs(np.diag(a)).max(), s
        if a.shape[0] <= 300:
            assert _bits(info["spsq"][s]) == _bits(_elim_spsq(a, zs[s])), (s, info["spsq"][s])
    pc.close()


@pytest.mark.parametrize("n", [2, 16, 17, 33, 300])
def test_blocked_pivoting_lu_det_bit_identical(gpu, n, monkeypatch):
    """The blocked partial-pivot elimination (LDS panel with row swaps, swaps
    replayed on the trailing columns, delayed updates) gives the host
    restatement's determinant bit for bit on random matrices that need row
    swaps, and so does the per-column path (PSX_LU_UNBLOCKED=1)."""
    a = np.random.default_rng(100 + n).standard_normal((n, n))
    h = E.lu_det(a)
    g = E.lu_det(a, gpu=True)
    monkeypatch.setenv("PSX_LU_UNBLOCKED", "1")
    u = E.lu_det(a, gpu=True)
    assert _bits(h) == _bits(g) == _bits(u), (n, h, g, u)


def test_blocked_step2_elimination_bit_identical(gpu):
    """Step 2 (no pivoting, on the lower triangle mirrored) through the blocked
    panels with the pivot check off: the min pivot ratio equals the host
    restatement's exactly, for an LD one ulp off symmetric (M = 300) and for
    tests/example's LDs (they need row swaps, so step 1 took the pivoting
    path)."""
    M = 300
    idx = np.arange(M)
    ld1 = 0.5 ** np.abs(idx[:, None] - idx[None, :])
    ld1[3, 17] = np.nextafter(ld1[3, 17], 1.0)
    rng = np.random.default_rng(5)
    cases = [([ld1, ld1.copy()], [rng.standard_normal(M), rng.standard_normal(M)],
              np.stack([idx, idx]).astype(np.int32), (6000, 7000))]
    L = loci.read_locus(loci.EXAMPLE["dirname"])
    cases.append((L["ld"], L["z"], L["u2l"], loci.EXAMPLE["n"]))
    for ld, z, u2l, n in cases:
        mi = E.model_inputs(ld, z, u2l, n, max_causal=1, sharing_param=0.25)
        pc = E.PostCal(mi)
        info = pc.setup_info
        for s in range(2):
            if info["eigen_route"][s]:
                continue
            a = np.asarray(ld[s], dtype=np.float64)
            add = info["psd_added"][s]
            sym = np.tril(a) + np.tril(a, -1).T + add * np.eye(a.shape[0])
            piv = _elim_pivots(sym)
            dmax = np.abs(np.diag(sym)).max()
            assert info["min_pivot_ratio"][s] == piv.min() / dmax, (s, info["min_pivot_ratio"][s], piv.min() / dmax)
            zs = np.asarray(z[s], dtype=np.float64)
            assert _bits(info["spsq"][s]) == _bits(_elim_spsq(sym, zs)), (s, info["spsq"][s], _elim_spsq(sym, zs))
        pc.close()
