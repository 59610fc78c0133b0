"""The drop-in CLI's argument handling (pipsort.cpp:68-228 quirks).  These
paths exit before the engine is created, so they run without a GPU."""
import os
import shutil
import subprocess

import pytest

import loci
from pipsort_amd import engine as E


def run(args, cwd):
    return subprocess.run([E.PIPSORT_BIN] + args, cwd=cwd, capture_output=True, text=True, timeout=60)


@pytest.fixture
def ex(tmp_path):
    d = tmp_path / "ex"
    shutil.copytree(os.path.join(loci.GOLDEN, "small_example"), d)
    return d


def test_required_options(ex):
    r = run(["-l", "ldfiles.txt", "-z", "zfiles.txt", "-o", "out"], ex)
    assert r.returncode == 1 and "Error: -l, -z, -o, and -n are required" in r.stdout


def test_flag_without_argument_aborts(ex):
    # pipsort.cpp:92-95: -h/-v/-x take no argument, so optarg is NULL -> exit 1
    r = run(["-h"], ex)
    assert r.returncode == 1 and "optarg is NULL" in r.stdout


def test_m_falls_through_into_n(ex):
    # pipsort.cpp:128-131: '-m' has no break, so -m after -n overwrites the sample sizes
    r = run(["-l", "ldfiles.txt", "-z", "zfiles.txt", "-n", "7000,7000", "-m", "eur_afr_small_test_snp_map",
             "-o", "out"], ex)
    assert r.returncode == 1 and "sample size is not in the right format" in r.stdout


def test_sample_size_format(ex):
    r = run(["-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "eur_afr_small_test_snp_map", "-n", "70a0,7000",
             "-o", "out"], ex)
    assert r.returncode == 1 and "sample size is not in the right format" in r.stdout


def test_study_count_mismatch(ex):
    r = run(["-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "eur_afr_small_test_snp_map", "-n", "7000",
             "-o", "out"], ex)
    assert r.returncode == 1 and "do not match in number" in r.stdout


def test_configs_requires_count(ex):
    r = run(["-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "eur_afr_small_test_snp_map", "-n", "7000,7000",
             "-b", "x", "-o", "out"], ex)
    assert r.returncode == 1 and "Number of configs must be greater than 0" in r.stdout


def test_no_gpu_fails_loudly(ex):
    if E.device_count() > 0:
        pytest.skip("GPU present")
    r = run(["-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "eur_afr_small_test_snp_map", "-n", "7000,7000",
             "-o", "out"], ex)
    assert r.returncode == 1 and "no HIP device" in r.stdout


@pytest.mark.parametrize("stop_at", [None, 1, 250_000, 999_999])
def test_ld_parser_stops_at_first_rejected_token(tmp_path, stop_at):
    """util.cpp:86-96 semantics of the chunk-parallel LD parser: parsing stops at
    the first token `istream >> double` rejects, wherever the parallel chunks
    are cut (a 1000 x 1000 file is ~20 MB, several chunks).  The CLI then
    reports the size it parsed (model.h:98-103) before touching the engine."""
    import numpy as np
    from pipsort_amd import synth
    M = 1000
    ld, z, names, rows, _ = synth.syn_v1(M)
    d = synth.write_locus(str(tmp_path / "loc"), ld, z, names, rows)
    if stop_at is not None:
        p = os.path.join(d, "syn0.ld")
        toks = open(p).read().split()
        toks[stop_at] = "x" + toks[stop_at]
        open(p, "w").write(" ".join(toks) + "\n")
    r = run(["-c", "2", "-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "snp_map", "-n", "10000,8000", "-o", "out"], d)
    if stop_at is None:
        assert "LD matrix is size" not in r.stdout
        assert "pushing back num snps 0 for study %d" % M in r.stdout
    else:
        m = int(np.sqrt(stop_at))
        assert r.returncode == 1
        assert f"LD matrix is size {m} x {m} but zscores has {M} snps" in r.stdout


@pytest.mark.parametrize("tok,parsed", [("-nan", 399), ("-inf", 399), ("nan", 399), ("inf", 399), ("1e400", 399),
                                        ("-1e400", 399), ("1e+", 399), ("+-1", 399), ("-", 399), ("0x10", 400),
                                        ("1e5e3", 400), ("x1", 399)])
def test_ld_parser_matches_istream_extraction(tmp_path, tok, parsed):
    """util.cpp:94 `while (file >> data)`: libstdc++'s num_get collects a sign,
    digits with one '.', and an exponent, and fails on a partial conversion or an
    overflow to inf (checked with a g++ probe: "0x10" yields 0 then stops at 'x';
    "1e5e3" yields 1e5 then stops; nan / inf / 1e400 / "1e+" stop at once)."""
    from pipsort_amd import synth
    M = 30
    ld, z, names, rows, _ = synth.syn_v1(M)
    d = synth.write_locus(str(tmp_path / "loc"), ld, z, names, rows)
    p = os.path.join(d, "syn0.ld")
    toks = open(p).read().split()
    toks[399] = tok
    open(p, "w").write(" ".join(toks) + "\n")
    r = run(["-c", "2", "-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "snp_map", "-n", "10000,8000", "-o", "out"], d)
    m = int(parsed ** 0.5)
    assert r.returncode == 1
    assert f"LD matrix is size {m} x {m} but zscores has {M} snps" in r.stdout
