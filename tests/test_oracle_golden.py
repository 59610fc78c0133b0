"""The oracle (CPU restatement, oracle/) pinned against the reference's own
golden vectors: /root/reference/tests/example/expected_* (copied to
tests/golden/example/).  CPU only."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import loci
from oracle import oracle as O
from pipsort_amd import engine as E

FILES = ("study0_post", "study1_post", "study0_set", "study1_set", "nocausal", "shared_pips")


def _run_cli(tmp_path, args, src="example"):
    d = tmp_path / src
    shutil.copytree(os.path.join(loci.GOLDEN, src), d)
    r = subprocess.run([O.CLI] + args, cwd=d, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return d


def test_example_reproduces_reference_goldens(tmp_path):
    # tests/example/run_example.sh:1 invocation
    d = _run_cli(tmp_path, ["-c", "2", "-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "snp_map", "-n",
                            "334324,6771", "-p", "0.25", "-o", "pipsort_results"])
    for f in FILES:
        got = open(d / f"pipsort_results_{f}.txt").read()
        exp = open(d / f"expected_{f}.txt").read()
        if f != "shared_pips":
            assert got == exp, f
        else:
            # shared_ll / notshared_ll are updated without a lock in the reference
            # (postcal.cpp:1012-1017): compare the PIP column exactly, LL columns numerically
            g = [l.split("\t") for l in got.splitlines()[1:]]
            e = [l.split("\t") for l in exp.splitlines()[1:]]
            assert [x[:2] for x in g] == [x[:2] for x in e]
            gl = np.array([[float(x[2]), float(x[3])] for x in g])
            el = np.array([[float(x[2]), float(x[3])] for x in e])
            bad = np.abs(gl - el) > 1e-6 * np.maximum(1.0, np.abs(el))
            assert bad.any(axis=1).sum() <= 1
    # _log.txt is appended, never overwritten (util.cpp:183-187)
    assert len(open(d / "pipsort_results_log.txt").read().splitlines()) == 1


def test_literal_nxn_equals_reduced_kxk():
    """The k x k reduction used by the oracle equals the reference's N x N
    Woodbury formulation (postcal.cpp:214-304) on the rank-deficient small locus."""
    for c in (1, 2, 3):
        seam, _ = loci.seam_for(loci.SMALL, c=c)
        a = O.postcal(seam)
        b = O.postcal(seam, literal=True)
        for k in ("post", "no_causal", "shared", "shared_ll", "notshared_ll"):
            np.testing.assert_allclose(a[k], b[k], rtol=1e-12, atol=1e-9)
        assert abs(a["total"] - b["total"]) < 1e-9
        assert a["n_configs"] == b["n_configs"]


def test_configs_file_and_sss_paths():
    seam, L = loci.seam_for(loci.CONFIGS)
    rows = np.fromfile(os.path.join(L["dir"], "all_configs_int16"), dtype=np.int16).reshape(72, 5)
    r = O.postcal(seam, "configs", rows)
    assert r["n_configs"] == 72
    pip = np.where(r["post"] == 0, 0.0, np.exp(np.minimum(r["post"] - r["total"], 0)))
    assert np.all(pip <= 1 + 1e-12) and (r["post"] == 0).sum() == 4
    seam, _ = loci.seam_for(loci.SMALL)
    s = O.postcal(seam, "sss")
    # the walk hits "no new configurations" after 2 iterations and the null
    # configuration is accumulated twice (sss_postcal.cpp:202 then as a minus-neighbour)
    assert s["n_configs"] == 25


@pytest.mark.parametrize("spec_c", [("small", 3), ("mixed", 3), ("syn", 2)])
def test_member_sums_checker_matches_whole_oracle(spec_c):
    """oracle.member_sums (the per-SNP checker used at loci too large for the
    whole-sweep oracle) reproduces the whole-sweep oracle's post / shared /
    sharedLL / notSharedLL entries of every union SNP."""
    from pipsort_amd import synth
    name, c = spec_c
    if name == "small":
        seam, _ = loci.seam_for(loci.SMALL, c=c)
    elif name == "mixed":
        ld, z, _, _, u2l = synth.mixed_locus(30, 25, 12, seed=7)
        seam = E.seam_from_arrays(ld, z, u2l, (5000, 9000), max_causal=c, sharing_param=0.5)
    else:
        ld, z, _, _, u2l = synth.syn_v1(40)
        seam = E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=c, sharing_param=0.25)
    ref = O.postcal(seam)
    m0 = int(seam.m[0])
    for u in range(seam.n_union):
        g = O.member_sums(seam, u, threads=4)
        l0, l1 = seam.union_to_local[:, u]
        want = [ref["post"][l0] if l0 >= 0 else 0.0, ref["post"][m0 + l1] if l1 >= 0 else 0.0,
                ref["shared"][u], ref["shared_ll"][u], ref["notshared_ll"][u]]
        got = [g["post0"], g["post1"], g["shared"], g["shared_ll"], g["notshared_ll"]]
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=0, err_msg=f"u={u}")


def test_cholesky_seam_equals_eigen_seam():
    """A Cholesky seam (B = L^T, S' = L^-1 z) gives the eigen-route seam's
    accumulators (the path consumes only B^T B, B^T S', ||S'||^2)."""
    from pipsort_amd import synth
    ld, z, _, _, u2l = synth.syn_v1(50)
    a = O.postcal(E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=3, sharing_param=0.25))
    b = O.postcal(O.cholesky_seam(ld, z, u2l, (10000, 8000), max_causal=3, sharing_param=0.25))
    assert a["n_configs"] == b["n_configs"]
    for k in ("post", "no_causal", "shared", "shared_ll", "notshared_ll"):
        np.testing.assert_allclose(a[k], b[k], rtol=1e-11, atol=0, err_msg=k)
    assert abs(a["total"] - b["total"]) <= 1e-11 * abs(a["total"])


def test_construct_configs_matches_reference_script():
    """synth.construct_configs restates utils/construct_configs_all_studies.py;
    tests/golden/configs_gen/expected_* were written by the reference script
    itself (make_fixture.py) on the small important-SNP files beside them,
    including out-of-order groups that exercise its special_sort."""
    from pipsort_amd import synth
    d = os.path.join(loci.GOLDEN, "configs_gen")
    n, g = [int(x) for x in open(os.path.join(d, "expected_dims.txt")).read().split()]
    exp = np.fromfile(os.path.join(d, "expected_configs_int16"), dtype=np.int16).reshape(n, g)
    got = synth.construct_configs([synth.read_imp_snps(os.path.join(d, "imp0.tsv")),
                                   synth.read_imp_snps(os.path.join(d, "imp1.tsv"))], [9, 8])
    assert got.dtype == np.int16 and np.array_equal(got, exp)


def test_all_configs_rows_through_oracle_equal_exhaustive():
    """A -b file listing every configuration of a locus, run through the
    oracle's configs enumerator (postcal.cpp:400-714), gives the oracle's
    exhaustive accumulators (postcal.cpp:716-1092)."""
    from pipsort_amd import synth
    ld, z, _, _, u2l = synth.mixed_locus(9, 8, 5, seed=3)
    seam = E.seam_from_arrays(ld, z, u2l, (5000, 9000), max_causal=3, sharing_param=0.5)
    rows = synth.all_configs_rows(seam.union_to_local, seam.m, 3)
    a = O.postcal(seam)
    b = O.postcal(seam, "configs", rows)
    assert a["n_configs"] == b["n_configs"] == rows.shape[0]
    for k in ("post", "no_causal", "shared", "shared_ll", "notshared_ll"):
        np.testing.assert_allclose(b[k], a[k], rtol=1e-12, atol=0, err_msg=k)


@pytest.mark.parametrize("u", [0, 125, 499])
def test_fullsize_golden_sums_reproduce(u):
    """The committed full-size golden sums (tests/golden/fullsize/, made by
    make_member_sums.py) are the oracle's: recompute three SNPs of SYN-v1 M = 500."""
    import numpy as np
    from pipsort_amd import synth
    rows = np.loadtxt(os.path.join(loci.GOLDEN, "fullsize", "syn500c3_member_sums.txt"), comments="#")
    ld, z, _, _, u2l = synth.syn_v1(500)
    seam = O.cholesky_seam(ld, z, u2l, (10000, 8000), max_causal=3, sharing_param=0.25)
    r = O.member_sums(seam, u)
    got = [r["post0"], r["post1"], r["shared"], r["shared_ll"], r["notshared_ll"], r["n_patterns"]]
    np.testing.assert_allclose(got, rows[u, 1:7], rtol=1e-14, atol=0)
