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


def construct_configs(groups, num_snps):
    """The -b configs file of utils/construct_configs_all_studies.py:50-158:
    `groups[s]` lists study s's groups (its important-SNP file's rows cut by
    sorted group id, :50-65) as local SNP indices; each group contributes
    either no SNP (-1) or one of its SNPs, offset by the studies before it
    (:70-78); rows are the Cartesian product of the groups in order, the first
    varying slowest (:98-106), with each row's non-negative entries sorted in
    place (special_sort, :131-139).  Returns int16 [n_configs, n_groups]."""
    arrs = []
    off = 0
    for s, gs in enumerate(groups):
        if s > 0:
            off += int(num_snps[s - 1])
        for g in gs:
            arrs.append(np.concatenate([[-1], np.asarray(g, dtype=np.int64) + off]).astype(np.int16))
    if not arrs:
        return np.full((1, 1), -1, dtype=np.int16)
    grid = np.stack(np.meshgrid(*arrs, indexing="ij"), axis=-1).reshape(-1, len(arrs))
    # special_sort: sorted non-negative entries back into the non-negative slots
    pos = grid >= 0
    key = np.where(pos, grid.astype(np.int32), np.iinfo(np.int32).max)
    srt = np.sort(key, axis=1)
    out = np.full(grid.shape, -1, dtype=np.int16)
    rank = np.cumsum(pos, axis=1) - 1
    rows_i = np.nonzero(pos)
    out[rows_i] = srt[rows_i[0], rank[rows_i]].astype(np.int16)
    return out


def read_imp_snps(path):
    """One study's important-SNP file as construct_configs_all_studies.py:20-26,
    50-65 reads it (tab separated, column 2 the local index, column 3 the group
    id; rows taken in file order, cut by the sorted group ids' counts)."""
    if not os.path.exists(path) or os.path.getsize(path) == 0:
        return []
    cols = [l.rstrip("\n").split("\t") for l in open(path) if l.strip()]
    gid = np.array([float(c[3]) for c in cols])
    loc = [int(float(c[2])) for c in cols]
    _, counts = np.unique(gid, return_counts=True)
    out, o = [], 0
    for n in counts:
        out.append(loc[o:o + n])
        o += n
    return out


def all_configs_rows(union_to_local, m, c):
    """Every configuration of an exhaustive sweep up to c union SNPs
    (postcal.cpp:716-1092: union subsets, then the per-study assignments
    passing checkOR) as -b rows of global indices (study 1 offset by M_0),
    ascending, -1 padded to 2c columns; the null configuration is the all -1
    row."""
    import itertools
    u2l = np.asarray(union_to_local)
    U = u2l.shape[1]
    allowed = [[x for x in (1, 2, 3) if all(not (x >> s) & 1 or u2l[s, u] >= 0 for s in range(2))] for u in range(U)]
    rows = [[-1] * (2 * c)]
    for k in range(1, c + 1):
        for S in itertools.combinations(range(U), k):
            for xs in itertools.product(*(allowed[u] for u in S)):
                g = sorted([int(u2l[0, u]) for u, x in zip(S, xs) if x & 1] +
                           [int(m[0]) + int(u2l[1, u]) for u, x in zip(S, xs) if x & 2])
                rows.append(g + [-1] * (2 * c - len(g)))
    return np.array(rows, dtype=np.int16)
