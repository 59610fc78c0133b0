"""Host Model setup (PSD shift + eigen low-rank transform) against the oracle
restatement of model.h:171-264 / util.cpp:195-263.  CPU only."""
import numpy as np

import loci
from oracle import oracle as O
from pipsort_amd import engine as E


def _blocks(Bflat, sp, m):
    out, o, so = [], 0, 0
    for s in range(2):
        M = int(m[s])
        Bs = Bflat[o:o + M * M].reshape(M, M).T  # column-major -> B(r, c)
        out.append((Bs.T @ Bs, Bs.T @ sp[so:so + M]))
        o += M * M
        so += M
    return out


def test_psd_shift_matches_oracle():
    for spec in (loci.EXAMPLE, loci.SMALL):
        L = loci.read_locus(spec["dirname"])
        _, _, _, _, add = O.setup_from_files(*L["files"])
        for s in range(2):
            _, a = E.psd_shift(L["ld"][s])
            assert a == add[s], (spec["dirname"], s, a, add[s])
    # the eur LD of small_example is rank deficient (SNPs 0/1 perfectly correlated)
    L = loci.read_locus("small_example")
    assert E.psd_shift(L["ld"][0])[1] > 0


def test_lowrank_invariants_match_oracle():
    """B^T B, B^T S' and ||S'||^2 are invariant to eigenvector order/sign and are
    all the PostCal path consumes."""
    for spec in (loci.EXAMPLE, loci.SMALL):
        seam, L = loci.seam_for(spec)
        B, sp, u2l, m, _ = O.setup_from_files(*L["files"])
        np.testing.assert_array_equal(u2l, seam.union_to_local)
        for (Sa, ya), (Sb, yb) in zip(_blocks(seam.B, seam.s_prime, seam.m), _blocks(B, sp, m)):
            np.testing.assert_allclose(Sa, Sb, rtol=0, atol=1e-10 * np.abs(Sb).max())
            np.testing.assert_allclose(ya, yb, rtol=0, atol=1e-10 * np.abs(yb).max())
        ka, kb = (seam.s_prime ** 2).sum(), (sp ** 2).sum()
        assert abs(ka - kb) <= 1e-10 * kb


def test_sym_eigen_reconstructs():
    rng = np.random.default_rng(1)
    for n in (1, 2, 7, 64, 129):
        a = rng.standard_normal((n, n))
        a = a + a.T
        w, q = E.sym_eigen(a)
        np.testing.assert_allclose(q @ np.diag(w) @ q.T, a, atol=1e-11 * max(1, np.abs(a).max()))
        np.testing.assert_allclose(q.T @ q, np.eye(n), atol=1e-12)
        np.testing.assert_allclose(np.sort(w), np.linalg.eigvalsh(a), atol=1e-10 * max(1, np.abs(w).max()))


def test_product_setup_reproduces_reference_pips():
    """Product setup -> (oracle) PostCal reproduces tests/example's expected PIPs."""
    seam, L = loci.seam_for(loci.EXAMPLE)
    r = O.postcal(seam)
    pip = np.exp(r["post"] - r["total"])
    pip[r["post"] == 0] = 0
    m0 = int(seam.m[0])
    for s, sl in ((0, slice(0, m0)), (1, slice(m0, None))):
        exp = np.array([float(l.split()[1]) for l in
                        open(f"{L['dir']}/expected_study{s}_post.txt").read().splitlines()[1:]])
        assert np.abs(pip[sl] - exp).max() <= 1e-6
