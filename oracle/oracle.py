"""ctypes wrapper of the oracle (TEST INFRASTRUCTURE ONLY — see postcal_oracle.cpp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
CLI = os.path.join(HERE, "_build", "oracle_pipsort")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        P = ctypes.POINTER
        d, i32, i64 = ctypes.c_double, ctypes.c_int, ctypes.c_long
        _lib.oracle_postcal.restype = i32
        _lib.oracle_postcal.argtypes = [i32, P(i32), P(d), P(d), i32, P(i32), i32, P(i32), d, d, d, d, i32,
                                        P(ctypes.c_int16), i64, i32, i32, P(d), P(d), P(d), P(d), P(d), P(d),
                                        P(i64)]
        _lib.oracle_eval_patterns.restype = i32
        _lib.oracle_eval_patterns.argtypes = [i32, P(i32), P(d), P(d), i32, P(i32), P(i32), d, d, d, d, i32, i32,
                                              P(i32), P(i32), i32, P(d), P(d)]
        _lib.oracle_member_sums.restype = i32
        _lib.oracle_member_sums.argtypes = [i32, P(i32), P(d), P(d), i32, P(i32), P(i32), d, d, d, d, i32, i32, i32,
                                            P(d), P(i64)]
        _lib.oracle_setup_dims.restype = i32
        _lib.oracle_setup_dims.argtypes = [ctypes.c_char_p] * 5 + [P(i32), P(i32)]
        _lib.oracle_setup.restype = i32
        _lib.oracle_setup.argtypes = [ctypes.c_char_p] * 5 + [P(d), P(d), P(i32), P(d)]
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def postcal(seam, mode="exhaustive", rows=None, literal=False):
    """Run the restated PostCal on the seam inputs; returns a dict of accumulators."""
    lib = load()
    m = np.ascontiguousarray(seam.m, dtype=np.int32)
    B = np.ascontiguousarray(seam.B, dtype=np.float64)
    sp = np.ascontiguousarray(seam.s_prime, dtype=np.float64)
    u2l = np.ascontiguousarray(seam.union_to_local, dtype=np.int32)
    n = np.ascontiguousarray(seam.sample_sizes, dtype=np.int32)
    N, U = int(m.sum()), u2l.shape[1]
    out = {k: np.zeros(N if k == "post" else (2 if k == "no_causal" else U))
           for k in ("post", "no_causal", "shared", "shared_ll", "notshared_ll")}
    tot = ctypes.c_double(0)
    nev = ctypes.c_long(0)
    md = {"exhaustive": 0, "sss": 1, "configs": 2}[mode]
    if rows is None:
        r = np.zeros((1, 1), dtype=np.int16)
        nr, ng = 0, 1
    else:
        r = np.ascontiguousarray(rows, dtype=np.int16)
        nr, ng = r.shape
    D = ctypes.c_double
    rc = lib.oracle_postcal(2, _p(m, ctypes.c_int), _p(B, D), _p(sp, D), U, _p(u2l, ctypes.c_int),
                            int(seam.max_causal), _p(n, ctypes.c_int), float(seam.sharing_param), float(seam.gamma),
                            float(seam.t_squared), float(seam.s_squared), md, _p(r, ctypes.c_int16), nr, ng,
                            1 if literal else 0, _p(out["post"], D), _p(out["no_causal"], D), _p(out["shared"], D),
                            _p(out["shared_ll"], D), _p(out["notshared_ll"], D), ctypes.byref(tot),
                            ctypes.byref(nev))
    if rc != 0:
        raise RuntimeError(f"oracle_postcal failed: {rc}")
    out["total"] = tot.value
    out["n_configs"] = nev.value
    return out


def eval_patterns(seam, sets, bits, literal=False):
    """(L, ll) for explicit patterns: sets int[n, k] ascending union idx, bits int[n, 2, k]."""
    lib = load()
    m = np.ascontiguousarray(seam.m, dtype=np.int32)
    B = np.ascontiguousarray(seam.B, dtype=np.float64)
    sp = np.ascontiguousarray(seam.s_prime, dtype=np.float64)
    u2l = np.ascontiguousarray(seam.union_to_local, dtype=np.int32)
    n = np.ascontiguousarray(seam.sample_sizes, dtype=np.int32)
    s = np.ascontiguousarray(sets, dtype=np.int32)
    b = np.ascontiguousarray(bits, dtype=np.int32)
    L = np.zeros(s.shape[0])
    ll = np.zeros(s.shape[0])
    D = ctypes.c_double
    rc = lib.oracle_eval_patterns(2, _p(m, ctypes.c_int), _p(B, D), _p(sp, D), u2l.shape[1], _p(u2l, ctypes.c_int),
                                  _p(n, ctypes.c_int), float(seam.sharing_param), float(seam.gamma),
                                  float(seam.t_squared), float(seam.s_squared), s.shape[1], s.shape[0],
                                  _p(s, ctypes.c_int), _p(b, ctypes.c_int), 1 if literal else 0, _p(L, D), _p(ll, D))
    if rc != 0:
        raise RuntimeError("oracle_eval_patterns failed")
    return L, ll


def member_sums(seam, u, threads=None):
    """One union SNP's accumulators over the exhaustive sweep (oracle_member_sums):
    dict post0, post1, shared, shared_ll, notshared_ll (log, 0 = empty) and
    n_patterns.  Exact log-sum-exp over every union set containing u."""
    lib = load()
    m = np.ascontiguousarray(seam.m, dtype=np.int32)
    B = np.ascontiguousarray(seam.B, dtype=np.float64)
    sp = np.ascontiguousarray(seam.s_prime, dtype=np.float64)
    u2l = np.ascontiguousarray(seam.union_to_local, dtype=np.int32)
    n = np.ascontiguousarray(seam.sample_sizes, dtype=np.int32)
    out = np.zeros(5)
    npat = ctypes.c_long(0)
    threads = threads or len(os.sched_getaffinity(0))
    D = ctypes.c_double
    rc = lib.oracle_member_sums(2, _p(m, ctypes.c_int), _p(B, D), _p(sp, D), u2l.shape[1], _p(u2l, ctypes.c_int),
                                _p(n, ctypes.c_int), float(seam.sharing_param), float(seam.gamma),
                                float(seam.t_squared), float(seam.s_squared), int(seam.max_causal), int(u),
                                int(threads), _p(out, D), ctypes.byref(npat))
    if rc != 0:
        raise RuntimeError("oracle_member_sums failed")
    return dict(post0=out[0], post1=out[1], shared=out[2], shared_ll=out[3], notshared_ll=out[4],
                n_patterns=npat.value)


def cholesky_seam(ld, z, union_to_local, sample_sizes, **params):
    """A PostCal seam for a positive-definite LD without the eigen route: B_s =
    L_s^T (Sigma_s = L_s L_s^T), S'_s = L_s^-1 z_s.  The path consumes only
    B^T B = Sigma, B^T S' = z and ||S'||^2 = z^T Sigma^-1 z, which equal the
    reference's eigen-route values (model.h:213-259) in exact arithmetic, so
    this is a fast oracle input for large synthetic loci (no PSD shift: SYN-v1
    needs none up to M = 2000)."""
    import scipy.linalg
    from pipsort_amd.engine import Seam
    Bs, sps = [], []
    for s in range(2):
        L = np.linalg.cholesky(np.asarray(ld[s], dtype=np.float64))
        Bs.append(np.asarray(L.T, order="F").ravel(order="F"))  # column-major B_s = L^T
        sps.append(scipy.linalg.solve_triangular(L, np.asarray(z[s], dtype=np.float64), lower=True))
    m = np.array([ld[0].shape[0], ld[1].shape[0]], dtype=np.int32)
    return Seam(m=m, B=np.concatenate(Bs), s_prime=np.concatenate(sps),
                union_to_local=np.asarray(union_to_local, dtype=np.int32),
                sample_sizes=np.asarray(sample_sizes, dtype=np.int32), **params)


def setup_from_files(ld0, ld1, z0, z1, snp_map):
    """Model setup restated by the oracle: returns (B, s_prime, union_to_local, m, psd_add)."""
    lib = load()
    m = np.zeros(2, dtype=np.int32)
    U = ctypes.c_int(0)
    args = [x.encode() for x in (ld0, ld1, z0, z1, snp_map)]
    if lib.oracle_setup_dims(*args, _p(m, ctypes.c_int), ctypes.byref(U)) != 0:
        raise RuntimeError("oracle_setup_dims failed")
    B = np.zeros(int(m[0]) ** 2 + int(m[1]) ** 2)
    sp = np.zeros(int(m.sum()))
    u2l = np.zeros((2, U.value), dtype=np.int32)
    add = np.zeros(2)
    D = ctypes.c_double
    if lib.oracle_setup(*args, _p(B, D), _p(sp, D), _p(u2l, ctypes.c_int), _p(add, D)) != 0:
        raise RuntimeError("oracle_setup failed")
    return B, sp, u2l, m, add
