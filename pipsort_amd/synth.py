"""SYN-v1 synthetic two-study locus.

LD_s[i, j] = rho_s^|i-j| (rho_0 = 0.6, rho_1 = 0.4); every SNP in both studies;
effects lambda_0[M/4] = lambda_1[M/4] = 5 (shared) and lambda_0[3M/4] = 4;
z_s = Sigma_s lambda_s + chol(Sigma_s) eps_s with eps_s from
numpy.random.default_rng(20261015 + s).  numpy's PCG64 stream is platform
stable, so the files regenerate identically on any box.  Also provides
"mixed" loci (some SNPs in one study only) for parity edge cases.
"""
from __future__ import annotations

import os

import numpy as np

RHO = (0.6, 0.4)
SEED = 20261015


def syn_v1(M: int):
    """Return (ld[2], z[2], names[2], snp_map rows, union_to_local[2, U])."""
    ld, z, names = [], [], []
    idx = np.arange(M)
    for s in range(2):
        sig = RHO[s] ** np.abs(idx[:, None] - idx[None, :])
        lam = np.zeros(M)
        lam[M // 4] = 5.0
        if s == 0:
            lam[3 * M // 4] = 4.0
        eps = np.random.default_rng(SEED + s).standard_normal(M)
        zs = sig @ lam + np.linalg.cholesky(sig) @ eps
        ld.append(sig)
        z.append(zs)
        names.append([f"syn{i}" for i in range(M)])
    u2l = np.stack([idx, idx]).astype(np.int32)
    rows = [(f"syn{i}", i, i) for i in range(M)]
    return ld, z, names, rows, u2l


def mixed_locus(M0: int, M1: int, n_shared: int, seed: int = 7):
    """Two studies with partially overlapping SNPs (union ordered, local indices
    increasing in union order as model.h:134-139 assumes)."""
    rng = np.random.default_rng(seed)
    U = M0 + M1 - n_shared
    # decide membership per union SNP: first build a random interleaving
    kinds = np.array([3] * n_shared + [1] * (M0 - n_shared) + [2] * (M1 - n_shared))
    rng.shuffle(kinds)
    u2l = -np.ones((2, U), dtype=np.int32)
    c = [0, 0]
    for u, k in enumerate(kinds):
        for s in range(2):
            if k & (1 << s):
                u2l[s, u] = c[s]
                c[s] += 1
    ld, z, names = [], [], []
    for s, M in enumerate((M0, M1)):
        x = rng.standard_normal((M, 3 * M))
        x = x + 0.8 * np.roll(x, 1, axis=0)
        sig = np.atleast_2d(np.corrcoef(x))
        lam = np.zeros(M)
        lam[rng.integers(0, M)] = 4.0 + s
        zs = sig @ lam + rng.standard_normal(M) * 0.5
        ld.append(sig)
        z.append(zs)
        names.append([f"s{s}_{i}" for i in range(M)])
    rows = []
    for u in range(U):
        rows.append((f"u{u}", int(u2l[0, u]), int(u2l[1, u])))
    return ld, z, names, rows, u2l


def write_locus(dirpath: str, ld, z, names, rows, prefix="syn"):
    """Write the reference input formats (LD rows, `name\\tz`, snp map, path lists)."""
    os.makedirs(dirpath, exist_ok=True)
    ldp, zp = [], []
    for s in range(2):
        lf = os.path.join(dirpath, f"{prefix}{s}.ld")
        zf = os.path.join(dirpath, f"{prefix}{s}.z")
        np.savetxt(lf, ld[s], fmt="%.17g", delimiter=" ")
        with open(zf, "w") as f:
            for n, v in zip(names[s], z[s]):
                f.write(f"{n}\t{v:.17g}\n")
        ldp.append(os.path.basename(lf))
        zp.append(os.path.basename(zf))
    with open(os.path.join(dirpath, "ldfiles.txt"), "w") as f:
        f.write("\n".join(ldp) + "\n")
    with open(os.path.join(dirpath, "zfiles.txt"), "w") as f:
        f.write("\n".join(zp) + "\n")
    with open(os.path.join(dirpath, "snp_map"), "w") as f:
        for r in rows:
            f.write(f"{r[0]},{r[1]},{r[2]}\n")
    # model.h:100-103 needs the z names to be the SNP names of the study
    return dirpath
