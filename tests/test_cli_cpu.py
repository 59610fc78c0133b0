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
