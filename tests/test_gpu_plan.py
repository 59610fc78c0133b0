"""The sweep plans' record CSR, built on the device since r05 (psx_plan.hip:
record keys from the unit list, hipcub's stable radix sort, binary-searched
run starts), equals the host restatement entry for entry: pos (record slot ->
position or -1), dptr (per-SNP runs) and gidx (records in (SNP, slot) order,
the merges' fold order).  Marked gpu."""
import numpy as np
import pytest

from pipsort_amd import engine as E

CASES = []
for U in (3, 64, 65, 200, 1000):
    for k, variant in ((2, 0), (3, 0), (3, 1)):
        for rank, world in ((0, 1), (0, 2), (1, 2), (7, 8)):
            CASES.append((U, k, variant, rank, world))


@pytest.mark.gpu
@pytest.mark.parametrize("U,k,variant,rank,world", CASES)
def test_device_csr_matches_host(gpu, U, k, variant, rank, world):
    bad, nrec = E.plan_csr_selftest(U, k, rank, world, variant)
    assert bad == 0, (U, k, variant, rank, world, bad)
    assert nrec > 0 or U < 64


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])
def test_device_csr_mixed_presence(gpu, variant):
    rng = np.random.default_rng(3)
    U = 333
    pres = rng.integers(1, 4, U).astype(np.uint8)  # study 0 only / study 1 only / both
    for rank, world in ((0, 1), (2, 3)):
        bad, _ = E.plan_csr_selftest(U, 3, rank, world, variant, presence=pres)
        assert bad == 0, (variant, rank, world, bad)
