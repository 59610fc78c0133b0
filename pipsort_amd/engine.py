"""ctypes binding of the MI355X PostCal engine (include/pipsort_engine.h).

`PostCal` mirrors the reference class's seam (postcal.h:118 constructor inputs,
postcal.cpp:1128 run, postcal.h:62-78 accumulators) so parity tests read like
the reference's own usage.  There is no CPU fallback: constructing a PostCal
without a HIP device raises EngineError (PSX_ENODEV).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PSX_ENGINE_LIB: an alternative build of the same library (A/B experiments).
# It must export every symbol the ABI declares unless PSX_AB=1 (an older build
# under comparison), so a stray variable cannot run the suite on a stale build.
LIB_PATH = os.environ.get("PSX_ENGINE_LIB") or os.path.join(_HERE, "lib", "libpipsort_engine.so")
PIPSORT_BIN = os.path.join(_HERE, "bin", "PIPSORT")

PSX_OK = 0
PSX_EINVAL = -1
PSX_ENODEV = -2
PSX_EHIP = -3
PSX_ESINGULAR = -4
PSX_EORDER = -5
PSX_ERANGE = -6
PSX_EEXCHANGE = -7

# Every symbol declared in include/pipsort_engine.h and include/pipsort_model.h
EXPORTED = [
    "psx_abi_version", "psx_overlap_cus", "psx_last_error", "psx_device_count", "psx_pool_trim", "psx_pool_cached_bytes", "psx_warmup", "psx_warmup_for", "psx_single_queue", "psx_create", "psx_destroy",
    "psx_set_shard", "psx_run_exhaustive", "psx_run_configs", "psx_run_sss",
    "psx_eval_union_batch", "psx_reset", "psx_get_accum", "psx_partials_bytes",
    "psx_export_partials", "psx_partials_device_ptr", "psx_merge_partials", "psx_get_timing", "psx_count_configs",
    "psx_fold_partials_host", "psx_plan_hash", "psx_plan_build_ms", "psx_plan_csr_selftest", "psx_shard_stats", "psx_plan_units_k3", "psx_set_stream",
    "psx_psd_shift", "psx_lowrank_study", "psx_sym_eigen", "psx_lu_det",
    "psx_create_from_ld", "psx_psd_shift_gpu", "psx_lu_det_gpu", "psx_elim_gpu",
    "psx_run_exhaustive_async", "psx_sync", "psx_run_sss_sharded", "psx_run_sss_sharded_dev",
    "psx_multi_create", "psx_multi_create_from_ld", "psx_multi_run_exhaustive", "psx_multi_run_configs",
    "psx_multi_run_sss", "psx_multi_get_accum", "psx_multi_get_timing", "psx_multi_count",
    "psx_multi_last_error", "psx_multi_destroy",
]

# psx_allgather_fn (include/pipsort_engine.h): int (*)(void *ctx, const void *send, void *recv, int64_t bytes)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
# device variant: (ctx, device send, device recv, bytes per rank, hipStream_t)
ALLGATHER_DEV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                    ctypes.c_void_p)


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"psx error {code}: {msg}")
        self.code = code


class _Problem(ctypes.Structure):
    _fields_ = [
        ("n_studies", ctypes.c_int32),
        ("m", ctypes.POINTER(ctypes.c_int32)),
        ("B", ctypes.POINTER(ctypes.c_double)),
        ("s_prime", ctypes.POINTER(ctypes.c_double)),
        ("n_union", ctypes.c_int32),
        ("union_to_local", ctypes.POINTER(ctypes.c_int32)),
        ("max_causal", ctypes.c_int32),
        ("sample_sizes", ctypes.POINTER(ctypes.c_int32)),
        ("sharing_param", ctypes.c_double),
        ("gamma", ctypes.c_double),
        ("t_squared", ctypes.c_double),
        ("s_squared", ctypes.c_double),
    ]


class _LdProblem(ctypes.Structure):
    _fields_ = [
        ("n_studies", ctypes.c_int32),
        ("m", ctypes.POINTER(ctypes.c_int32)),
        ("ld", ctypes.POINTER(ctypes.c_double)),
        ("z", ctypes.POINTER(ctypes.c_double)),
        ("n_union", ctypes.c_int32),
        ("union_to_local", ctypes.POINTER(ctypes.c_int32)),
        ("max_causal", ctypes.c_int32),
        ("sample_sizes", ctypes.POINTER(ctypes.c_int32)),
        ("sharing_param", ctypes.c_double),
        ("gamma", ctypes.c_double),
        ("t_squared", ctypes.c_double),
        ("s_squared", ctypes.c_double),
    ]


class SetupInfo(ctypes.Structure):
    _fields_ = [
        ("psd_added", ctypes.c_double * 2),
        ("psd_iterations", ctypes.c_int32 * 2),
        ("eigen_route", ctypes.c_int32 * 2),
        ("min_pivot_ratio", ctypes.c_double * 2),
        ("setup_ms", ctypes.c_double),
        ("spsq", ctypes.c_double * 2),
        ("alloc_ms", ctypes.c_double),
        ("studies_ms", ctypes.c_double),
        ("tail_ms", ctypes.c_double),
        ("study_upload_ms", ctypes.c_double * 2),
        ("study_psd_ms", ctypes.c_double * 2),
        ("study_finish_ms", ctypes.c_double * 2),
    ]

    def as_dict(self):
        d = {}
        for f, _ in self._fields_:
            v = getattr(self, f)
            d[f] = v if isinstance(v, float) else list(v)
        return d


class _Accum(ctypes.Structure):
    _fields_ = [
        ("post", ctypes.POINTER(ctypes.c_double)),
        ("no_causal", ctypes.POINTER(ctypes.c_double)),
        ("shared", ctypes.POINTER(ctypes.c_double)),
        ("shared_ll", ctypes.POINTER(ctypes.c_double)),
        ("notshared_ll", ctypes.POINTER(ctypes.c_double)),
        ("total", ctypes.c_double),
        ("n_configs", ctypes.c_uint64),
    ]


class Timing(ctypes.Structure):
    _fields_ = [
        ("sweep_ms", ctypes.c_double),
        ("kernel_ms", ctypes.c_double),
        ("kernel_launches", ctypes.c_int32),
        ("merge_ms", ctypes.c_double),
        ("configs", ctypes.c_uint64),
        ("union_sets", ctypes.c_uint64),
        ("alg_bytes", ctypes.c_double),
        ("flops", ctypes.c_double),
        ("exact_rerun", ctypes.c_int32),
        ("robust_units", ctypes.c_int32),
        ("span_ms", ctypes.c_double),
        ("prepare_ms", ctypes.c_double),
        ("run_ms", ctypes.c_double),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_lib = None


def load_library(path: str = LIB_PATH):
    """Load the in-tree engine library (fails loudly if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise EngineError(PSX_ENODEV, f"engine library missing: {path} (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    c_int, c_i32, c_i64, c_u64 = ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    P = ctypes.POINTER
    dbl = ctypes.c_double
    vp = ctypes.c_void_p
    sig = {
        "psx_abi_version": (c_i32, []),
        "psx_overlap_cus": (c_i32, [vp]),
        "psx_last_error": (ctypes.c_char_p, []),
        "psx_device_count": (c_int, [P(c_int)]),
        "psx_pool_trim": (c_int, []),
        "psx_pool_cached_bytes": (ctypes.c_int64, []),
        "psx_warmup": (c_int, [c_int]),
        "psx_warmup_for": (c_int, [c_int, c_i32, c_i32]),
        "psx_single_queue": (c_int, [c_i32]),
        "psx_create": (c_int, [P(_Problem), c_int, P(vp)]),
        "psx_destroy": (None, [vp]),
        "psx_set_shard": (c_int, [vp, c_int, c_int]),
        "psx_run_exhaustive": (c_int, [vp]),
        "psx_run_configs": (c_int, [vp, P(ctypes.c_int16), c_i64, c_i32]),
        "psx_run_sss": (c_int, [vp, P(c_i32)]),
        "psx_eval_union_batch": (c_int, [vp, P(c_i32), c_i32, c_i32, c_int, P(dbl)]),
        "psx_reset": (c_int, [vp]),
        "psx_get_accum": (c_int, [vp, P(_Accum)]),
        "psx_partials_bytes": (c_i64, [vp]),
        "psx_export_partials": (c_int, [vp, vp]),
        "psx_partials_device_ptr": (c_int, [vp, ctypes.POINTER(vp)]),
        "psx_merge_partials": (c_int, [vp, vp, c_i32]),
        "psx_get_timing": (c_int, [vp, P(Timing)]),
        "psx_count_configs": (c_u64, [P(_Problem)]),
        "psx_fold_partials_host": (c_int, [vp, c_i32, c_i64, vp]),
        "psx_plan_hash": (c_int, [vp, P(ctypes.c_uint64)]),
        "psx_plan_build_ms": (c_int, [c_i32, c_i32, c_i32, c_i32, P(dbl), P(c_i32), P(c_i64)]),
        "psx_plan_csr_selftest": (c_int, [c_i32, P(ctypes.c_uint8), c_i32, c_i32, c_i32, c_i32, c_int, P(c_i64),
                                          P(c_i64)]),
        "psx_set_stream": (c_int, [vp, vp]),
        "psx_shard_stats": (c_int, [P(_Problem), c_i32, c_i32, c_i32, P(c_u64), P(dbl)]),
        "psx_plan_units_k3": (c_int, [c_i32, c_i32, c_i32, P(c_i32), c_i32]),
        "psx_psd_shift": (c_int, [P(dbl), c_i32, P(dbl)]),
        "psx_lowrank_study": (c_int, [P(dbl), P(dbl), c_i32, P(dbl), P(dbl)]),
        "psx_sym_eigen": (c_int, [P(dbl), c_i32, P(dbl), P(dbl)]),
        "psx_lu_det": (c_int, [P(dbl), c_i32, P(dbl)]),
        "psx_create_from_ld": (c_int, [P(_LdProblem), c_int, P(vp), P(SetupInfo)]),
        "psx_psd_shift_gpu": (c_int, [P(dbl), c_i32, P(dbl), c_int]),
        "psx_lu_det_gpu": (c_int, [P(dbl), c_i32, c_int, P(dbl)]),
        "psx_elim_gpu": (c_int, [P(dbl), c_i32, P(dbl), c_i32, P(dbl), P(dbl), P(c_i32), c_int]),
        "psx_run_exhaustive_async": (c_int, [vp]),
        "psx_sync": (c_int, [vp, P(c_i32)]),
        "psx_run_sss_sharded": (c_int, [vp, ALLGATHER_FN, vp, P(c_i32)]),
        "psx_run_sss_sharded_dev": (c_int, [vp, ALLGATHER_DEV_FN, vp, P(c_i32)]),
        "psx_multi_create": (c_int, [P(_Problem), P(c_i32), c_i32, P(vp)]),
        "psx_multi_create_from_ld": (c_int, [P(_LdProblem), P(c_i32), c_i32, P(vp), P(SetupInfo)]),
        "psx_multi_run_exhaustive": (c_int, [vp]),
        "psx_multi_run_configs": (c_int, [vp, P(ctypes.c_int16), c_i64, c_i32]),
        "psx_multi_run_sss": (c_int, [vp, P(c_i32)]),
        "psx_multi_get_accum": (c_int, [vp, P(_Accum)]),
        "psx_multi_get_timing": (c_int, [vp, P(Timing)]),
        "psx_multi_count": (c_i32, [vp]),
        "psx_multi_last_error": (ctypes.c_char_p, []),
        "psx_multi_destroy": (None, [vp]),
    }
    ab = os.environ.get("PSX_AB") == "1"
    for name, (res, args) in sig.items():
        if not hasattr(lib, name):
            if ab:
                continue  # an older build under A/B comparison
            raise EngineError(PSX_ENODEV, f"{path} lacks {name}: a stale engine build (PSX_AB=1 to compare anyway)")
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.psx_abi_version() != 4 and os.environ.get("PSX_AB") != "1":
        raise EngineError(PSX_ENODEV, f"{path}: ABI version {lib.psx_abi_version()}, this module needs 4")
    _lib = lib
    return lib


def _ptr(a, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def _check(rc: int):
    if rc != PSX_OK:
        raise EngineError(rc, load_library().psx_last_error().decode())


def device_count() -> int:
    c = ctypes.c_int(0)
    load_library().psx_device_count(ctypes.byref(c))
    return c.value


def pool_trim():
    """Give the engine's cached device / pinned blocks back to the HIP runtime."""
    _check(load_library().psx_pool_trim())


def pool_cached_bytes() -> int:
    return int(load_library().psx_pool_cached_bytes())


# ---------------------------------------------------------------------------
# Model setup (model.h:171-264) through the host C++ in the same library
# ---------------------------------------------------------------------------
def psd_shift(sigma: np.ndarray):
    """util.cpp:195-226: returns (sigma + a I, a)."""
    s = np.ascontiguousarray(sigma, dtype=np.float64).copy()
    add = ctypes.c_double(0.0)
    _check(load_library().psx_psd_shift(_ptr(s, ctypes.c_double), s.shape[0], ctypes.byref(add)))
    return s, add.value


def lu_det(a: np.ndarray, gpu: bool = False, device: int = 0) -> float:
    """The determinant util.cpp:214-215 tests (GSL-order LU, index-order product)."""
    aa = np.ascontiguousarray(a, dtype=np.float64)
    d = ctypes.c_double(0.0)
    lib = load_library()
    if gpu:
        _check(lib.psx_lu_det_gpu(_ptr(aa, ctypes.c_double), aa.shape[0], int(device), ctypes.byref(d)))
    else:
        _check(lib.psx_lu_det(_ptr(aa, ctypes.c_double), aa.shape[0], ctypes.byref(d)))
    return d.value


def elim_gpu(a: np.ndarray, z=None, check: bool = True, device: int = 0):
    """The setup's swap-free elimination on the GPU (psx_elim_gpu): returns
    (pivots U_ii, L^-1 z or None, swap_needed)."""
    aa = np.ascontiguousarray(a, dtype=np.float64)
    n = aa.shape[0]
    piv = np.empty(n)
    zz = None if z is None else np.ascontiguousarray(z, dtype=np.float64)
    zt = None if z is None else np.empty(n)
    sw = ctypes.c_int32(0)
    _check(load_library().psx_elim_gpu(_ptr(aa, ctypes.c_double), n,
                                       None if zz is None else _ptr(zz, ctypes.c_double), int(check),
                                       _ptr(piv, ctypes.c_double), None if zt is None else _ptr(zt, ctypes.c_double),
                                       ctypes.byref(sw), int(device)))
    return piv, zt, bool(sw.value)


def psd_shift_gpu(sigma: np.ndarray, device: int = 0):
    """util.cpp:195-226 with the determinants on the GPU: returns (sigma + a I, a)."""
    s = np.ascontiguousarray(sigma, dtype=np.float64).copy()
    add = ctypes.c_double(0.0)
    _check(load_library().psx_psd_shift_gpu(_ptr(s, ctypes.c_double), s.shape[0], ctypes.byref(add), int(device)))
    return s, add.value


def lowrank_study(sigma: np.ndarray, z: np.ndarray):
    """model.h:213-259: (B column-major flattened, S')."""
    m = sigma.shape[0]
    s = np.ascontiguousarray(sigma, dtype=np.float64)
    zz = np.ascontiguousarray(z, dtype=np.float64)
    B = np.empty(m * m, dtype=np.float64)
    sp = np.empty(m, dtype=np.float64)
    _check(load_library().psx_lowrank_study(_ptr(s, ctypes.c_double), _ptr(zz, ctypes.c_double), m,
                                             _ptr(B, ctypes.c_double), _ptr(sp, ctypes.c_double)))
    return B, sp


def sym_eigen(a: np.ndarray):
    m = a.shape[0]
    aa = np.ascontiguousarray(a, dtype=np.float64)
    w = np.empty(m)
    q = np.empty((m, m))
    _check(load_library().psx_sym_eigen(_ptr(aa, ctypes.c_double), m, _ptr(w, ctypes.c_double),
                                        _ptr(q, ctypes.c_double)))
    return w, q


@dataclass
class Seam:
    """PostCal constructor inputs (postcal.h:118) for two studies."""
    m: np.ndarray            # int32[2]
    B: np.ndarray            # float64, per-study column-major blocks concatenated
    s_prime: np.ndarray      # float64[N]
    union_to_local: np.ndarray  # int32[2, U]
    sample_sizes: np.ndarray    # int32[2]
    max_causal: int = 3
    sharing_param: float = 0.75
    gamma: float = 0.01
    t_squared: float = 0.52
    s_squared: float = 5.2

    @property
    def n_union(self):
        return int(self.union_to_local.shape[1])

    @property
    def N(self):
        return int(self.m.sum())

    def _struct(self):
        self._keep = [np.ascontiguousarray(self.m, dtype=np.int32),
                      np.ascontiguousarray(self.B, dtype=np.float64),
                      np.ascontiguousarray(self.s_prime, dtype=np.float64),
                      np.ascontiguousarray(self.union_to_local, dtype=np.int32),
                      np.ascontiguousarray(self.sample_sizes, dtype=np.int32)]
        m, B, sp, u2l, n = self._keep
        p = _Problem()
        p.n_studies = 2
        p.m = _ptr(m, ctypes.c_int32)
        p.B = _ptr(B, ctypes.c_double)
        p.s_prime = _ptr(sp, ctypes.c_double)
        p.n_union = u2l.shape[1]
        p.union_to_local = _ptr(u2l, ctypes.c_int32)
        p.max_causal = int(self.max_causal)
        p.sample_sizes = _ptr(n, ctypes.c_int32)
        p.sharing_param = float(self.sharing_param)
        p.gamma = float(self.gamma)
        p.t_squared = float(self.t_squared)
        p.s_squared = float(self.s_squared)
        return p

    def count_configs(self) -> int:
        p = self._struct()
        return int(load_library().psx_count_configs(ctypes.byref(p)))

    def shard_stats(self, k: int, rank: int, world: int):
        """(union sets, configurations) of level k evaluated by shard rank/world (host only)."""
        p = self._struct()
        sets = ctypes.c_uint64(0)
        cfg = ctypes.c_double(0)
        _check(load_library().psx_shard_stats(ctypes.byref(p), k, rank, world, ctypes.byref(sets),
                                              ctypes.byref(cfg)))
        return int(sets.value), float(cfg.value)


def seam_from_arrays(ld, z, union_to_local, sample_sizes, **params) -> Seam:
    """Model setup (model.h:171-264): PSD shift + eigen low-rank transform per study."""
    Bs, sps, ms = [], [], []
    for s in range(2):
        sig, _ = psd_shift(np.asarray(ld[s], dtype=np.float64))
        B, sp = lowrank_study(sig, np.asarray(z[s], dtype=np.float64))
        Bs.append(B)
        sps.append(sp)
        ms.append(sig.shape[0])
    return Seam(m=np.array(ms, dtype=np.int32), B=np.concatenate(Bs), s_prime=np.concatenate(sps),
                union_to_local=np.asarray(union_to_local, dtype=np.int32),
                sample_sizes=np.asarray(sample_sizes, dtype=np.int32), **params)


@dataclass
class ModelInputs:
    """What Model reads from the input files (model.h:60-160): per-study LD and z,
    the snp map and the CLI parameters.  PostCal(ModelInputs) runs the Model
    setup on the GPU (psx_create_from_ld) instead of taking B / S'."""
    ld: list
    z: list
    union_to_local: np.ndarray
    sample_sizes: np.ndarray
    max_causal: int = 3
    sharing_param: float = 0.75
    gamma: float = 0.01
    t_squared: float = 0.52
    s_squared: float = 5.2

    def __post_init__(self):
        self.ld = [np.ascontiguousarray(x, dtype=np.float64) for x in self.ld]
        self.z = [np.ascontiguousarray(x, dtype=np.float64) for x in self.z]
        self.m = np.array([x.shape[0] for x in self.ld], dtype=np.int32)

    @property
    def n_union(self):
        return int(np.asarray(self.union_to_local).shape[1])

    @property
    def N(self):
        return int(self.m.sum())

    def _struct(self):
        """psx_problem view (shape and parameters only; B / S' are not formed)."""
        self._keep = [self.m, np.ascontiguousarray(self.union_to_local, dtype=np.int32),
                      np.ascontiguousarray(self.sample_sizes, dtype=np.int32)]
        m, u2l, n = self._keep
        p = _Problem()
        p.n_studies = 2
        p.m = _ptr(m, ctypes.c_int32)
        p.n_union = u2l.shape[1]
        p.union_to_local = _ptr(u2l, ctypes.c_int32)
        p.max_causal = int(self.max_causal)
        p.sample_sizes = _ptr(n, ctypes.c_int32)
        p.sharing_param = float(self.sharing_param)
        p.gamma = float(self.gamma)
        p.t_squared = float(self.t_squared)
        p.s_squared = float(self.s_squared)
        return p

    def _ld_struct(self):
        # the ABI takes the studies' LDs concatenated; built once per ModelInputs
        # (a 2 x 32 MB copy at M = 2000 is ~10 ms of host time per create)
        key = tuple(id(x) for x in self.ld) + tuple(id(x) for x in self.z)
        if getattr(self, "_ld_key", None) != key:
            self._ld_key = key
            self._ld_cat = np.concatenate([np.asarray(x, dtype=np.float64).ravel() for x in self.ld])
            self._z_cat = np.concatenate([np.asarray(x, dtype=np.float64) for x in self.z])
        self._keep_ld = [self.m, self._ld_cat, self._z_cat,
                         np.ascontiguousarray(self.union_to_local, dtype=np.int32),
                         np.ascontiguousarray(self.sample_sizes, dtype=np.int32)]
        m, ld, z, u2l, n = self._keep_ld
        q = _LdProblem()  # (ld / z are read-only to the engine: the cached copies stay valid)
        q.n_studies = 2
        q.m = _ptr(m, ctypes.c_int32)
        q.ld = _ptr(ld, ctypes.c_double)
        q.z = _ptr(z, ctypes.c_double)
        q.n_union = u2l.shape[1]
        q.union_to_local = _ptr(u2l, ctypes.c_int32)
        q.max_causal = int(self.max_causal)
        q.sample_sizes = _ptr(n, ctypes.c_int32)
        q.sharing_param = float(self.sharing_param)
        q.gamma = float(self.gamma)
        q.t_squared = float(self.t_squared)
        q.s_squared = float(self.s_squared)
        return q

    count_configs = Seam.count_configs
    shard_stats = Seam.shard_stats


def model_inputs(ld, z, union_to_local, sample_sizes, **params) -> ModelInputs:
    return ModelInputs(list(ld), list(z), np.asarray(union_to_local, dtype=np.int32),
                       np.asarray(sample_sizes, dtype=np.int32), **params)


def fold_partials_host(images: np.ndarray) -> np.ndarray:
    """Fold partial images (uint8 [count, image_bytes], rank order) on the host."""
    imgs = np.ascontiguousarray(images, dtype=np.uint8)
    out = np.empty(imgs.shape[1], dtype=np.uint8)
    _check(load_library().psx_fold_partials_host(imgs.ctypes.data_as(ctypes.c_void_p), imgs.shape[0],
                                                 imgs.shape[1], out.ctypes.data_as(ctypes.c_void_p)))
    return out


def plan_build_ms(n_union: int, k: int = 3, rank: int = 0, world: int = 1):
    """Host time of building a level's unit plan + record CSR (psx_plan_build_ms):
    (ms, units, records)."""
    ms, nu, nr = ctypes.c_double(0), ctypes.c_int32(0), ctypes.c_int64(0)
    _check(load_library().psx_plan_build_ms(n_union, k, rank, world, ctypes.byref(ms), ctypes.byref(nu),
                                            ctypes.byref(nr)))
    return ms.value, nu.value, nr.value


def plan_csr_selftest(n_union: int, k: int, rank: int, world: int, variant: int, presence=None, device: int = 0):
    """GPU: (mismatches, records) of a plan's device-built record CSR against the
    host restatement (psx_plan_csr_selftest)."""
    bad, nrec = ctypes.c_int64(0), ctypes.c_int64(0)
    pr = None
    if presence is not None:
        pr = np.ascontiguousarray(presence, dtype=np.uint8)
    _check(load_library().psx_plan_csr_selftest(n_union, None if pr is None else _ptr(pr, ctypes.c_uint8), k, rank,
                                                world, variant, int(device), ctypes.byref(bad), ctypes.byref(nrec)))
    return bad.value, nrec.value


def plan_units_k3(n_union: int, rank: int = 0, world: int = 1) -> np.ndarray:
    """The k = 3 fast sweep's work units of one shard (host-only diagnostics):
    int32 [n, 4] rows {a0, a1, K | j0 << 16, C | j1 << 16} in dispatch order."""
    lib = load_library()
    n = lib.psx_plan_units_k3(n_union, rank, world, None, 0)
    _check(min(n, 0))
    out = np.zeros((max(n, 1), 4), dtype=np.int32)
    _check(min(lib.psx_plan_units_k3(n_union, rank, world, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n), 0))
    return out[:n]


# partial image record layout (psx_math.h Acc5 / SetRec)
ACC5_DTYPE = np.dtype([("mP", "<i4"), ("mS", "<i4"), ("mN", "<i4"), ("pad", "<i4"), ("post0", "<f8"),
                       ("post1", "<f8"), ("shared", "<f8"), ("sll", "<f8"), ("nsll", "<f8")])
SETREC_DTYPE = np.dtype([("m", "<i4"), ("m0", "<i4"), ("m1", "<i4"), ("pad", "<i4"), ("tot", "<f8"),
                         ("nc0", "<f8"), ("nc1", "<f8"), ("score", "<f8"), ("npat", "<f8")])
# last slot of an image: which shard of which plan (psx_math.h PlanTag)
PLANTAG_DTYPE = np.dtype([("magic", "<i4"), ("world", "<i4"), ("rank", "<i4"), ("U", "<i4"), ("hash", "<u8"),
                          ("pad", "<u8", (4,))])
PLAN_MAGIC = 0x54585350


def plan_tag(rank: int, world: int, U: int, hash_: int) -> bytes:
    """The PlanTag slot of a partial image (for images built on the host)."""
    t = np.zeros(1, dtype=PLANTAG_DTYPE)
    t["magic"], t["world"], t["rank"], t["U"], t["hash"] = PLAN_MAGIC, world, rank, U, hash_
    return t.tobytes()


@dataclass
class Accumulators:
    """PostCal accumulators in the reference's log-space convention (0 = empty)."""
    post: np.ndarray
    no_causal: np.ndarray
    shared: np.ndarray
    shared_ll: np.ndarray
    notshared_ll: np.ndarray
    total: float
    n_configs: int

    def pips(self):
        """special_exp(post, total) (postcal.h:277-283)."""
        def se(v):
            with np.errstate(over="ignore"):
                out = np.exp(v - self.total)
            out[v == 0] = 0.0
            return out
        return se(self.post), se(self.no_causal), se(self.shared)


class MultiPostCal:
    """PostCal over several devices in one process (psx_multi_*): one shard per
    entry of `devices` (entries may repeat), folded on devices[0]."""

    def __init__(self, seam, devices):
        self.lib = load_library()
        self.seam = seam
        dv = np.ascontiguousarray(devices, dtype=np.int32)
        h = ctypes.c_void_p()
        self.setup_info = None
        if isinstance(seam, ModelInputs):
            self._p = seam._ld_struct()
            info = SetupInfo()
            self._chk(self.lib.psx_multi_create_from_ld(ctypes.byref(self._p), _ptr(dv, ctypes.c_int32), len(dv),
                                                        ctypes.byref(h), ctypes.byref(info)))
            self.setup_info = info.as_dict()
        else:
            self._p = seam._struct()
            self._chk(self.lib.psx_multi_create(ctypes.byref(self._p), _ptr(dv, ctypes.c_int32), len(dv),
                                                ctypes.byref(h)))
        self.h = h

    def _chk(self, rc):
        if rc != PSX_OK:
            raise EngineError(rc, self.lib.psx_multi_last_error().decode())

    def close(self):
        if getattr(self, "h", None):
            self.lib.psx_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run_exhaustive(self):
        self._chk(self.lib.psx_multi_run_exhaustive(self.h))

    def run_configs(self, rows):
        r = np.ascontiguousarray(rows, dtype=np.int16)
        self._chk(self.lib.psx_multi_run_configs(self.h, _ptr(r, ctypes.c_int16), r.shape[0], r.shape[1]))

    def run_sss(self) -> int:
        it = ctypes.c_int32(0)
        self._chk(self.lib.psx_multi_run_sss(self.h, ctypes.byref(it)))
        return it.value

    def accum(self) -> "Accumulators":
        N, U = self.seam.N, self.seam.n_union
        post, noc = np.zeros(N), np.zeros(2)
        sh, sll, nsll = np.zeros(U), np.zeros(U), np.zeros(U)
        a = _Accum()
        a.post, a.no_causal = _ptr(post, ctypes.c_double), _ptr(noc, ctypes.c_double)
        a.shared, a.shared_ll = _ptr(sh, ctypes.c_double), _ptr(sll, ctypes.c_double)
        a.notshared_ll = _ptr(nsll, ctypes.c_double)
        self._chk(self.lib.psx_multi_get_accum(self.h, ctypes.byref(a)))
        return Accumulators(post, noc, sh, sll, nsll, a.total, int(a.n_configs))

    def timing(self) -> dict:
        t = Timing()
        self._chk(self.lib.psx_multi_get_timing(self.h, ctypes.byref(t)))
        return t.as_dict()


class PostCal:
    """The engine handle: one per GPU (postcal.h:118 PostCal::PostCal)."""

    def __init__(self, seam, device: int = 0):
        """seam: a Seam (PostCal's own inputs, B / S') or ModelInputs (LD / z;
        the Model setup then runs on the GPU, psx_create_from_ld)."""
        self.lib = load_library()
        self.seam = seam
        h = ctypes.c_void_p()
        self.setup_info = None
        if isinstance(seam, ModelInputs):
            self._p = seam._ld_struct()
            info = SetupInfo()
            _check(self.lib.psx_create_from_ld(ctypes.byref(self._p), int(device), ctypes.byref(h),
                                               ctypes.byref(info)))
            self.setup_info = info.as_dict()
        else:
            self._p = seam._struct()
            _check(self.lib.psx_create(ctypes.byref(self._p), int(device), ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.psx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle: int | None):
        """Enqueue on a caller HIP stream (e.g. torch.cuda.current_stream().cuda_stream)."""
        _check(self.lib.psx_set_stream(self.h, ctypes.c_void_p(stream_handle or None)))

    def set_shard(self, rank: int, world: int):
        _check(self.lib.psx_set_shard(self.h, rank, world))

    def overlap_cus(self) -> int:
        """CUs reserved beside overlapped asynchronous passes (psx_overlap_cus;
        -1 before the handle's first asynchronous pass)."""
        return int(self.lib.psx_overlap_cus(self.h))

    def plan_hash(self) -> int:
        """The shard plan's hash (psx_plan_hash): equal on every rank of a job."""
        h = ctypes.c_uint64(0)
        _check(self.lib.psx_plan_hash(self.h, ctypes.byref(h)))
        return int(h.value)

    def run_exhaustive(self):
        """postcal.cpp:716 computeTotalLikelihood."""
        _check(self.lib.psx_run_exhaustive(self.h))

    def run_exhaustive_async(self):
        """Enqueue one exhaustive pass without host synchronisation (psx_run_exhaustive_async)."""
        _check(self.lib.psx_run_exhaustive_async(self.h))

    def sync(self) -> bool:
        """Wait for the engine stream; True if some asynchronous pass since the last
        sync needs the exact rerun (its results are then not valid)."""
        f = ctypes.c_int32(0)
        _check(self.lib.psx_sync(self.h, ctypes.byref(f)))
        return bool(f.value)

    def run_configs(self, rows: np.ndarray):
        """postcal.cpp:400 computeTotalLikelihoodGivenConfigs; rows int16 [n, groups]."""
        r = np.ascontiguousarray(rows, dtype=np.int16)
        _check(self.lib.psx_run_configs(self.h, _ptr(r, ctypes.c_int16), r.shape[0], r.shape[1]))

    def run_sss(self) -> int:
        """sss_postcal.cpp:102 sss_computeTotalLikelihood; returns iterations."""
        it = ctypes.c_int32(0)
        _check(self.lib.psx_run_sss(self.h, ctypes.byref(it)))
        return it.value

    def run_sss_sharded(self, allgather) -> int:
        """The SSS walk across the ranks of set_shard (psx_run_sss_sharded).
        allgather(send: bytes) -> bytes gathers every rank's equal-sized `send`
        in rank order (e.g. torch.distributed.all_gather_into_tensor).  Merge
        the accumulators afterwards with export_partials / merge_partials."""
        err = []

        def cb(_ctx, send, recv, nbytes):
            try:
                out = allgather(ctypes.string_at(send, nbytes))
                ctypes.memmove(recv, out, len(out))
                return 0
            except BaseException as ex:  # reported through the engine's error code
                err.append(ex)
                return 1

        fn = ALLGATHER_FN(cb)
        it = ctypes.c_int32(0)
        rc = self.lib.psx_run_sss_sharded(self.h, fn, None, ctypes.byref(it))
        if err:
            raise err[0]
        _check(rc)
        return it.value

    def run_sss_sharded_dev(self, allgather_dev) -> int:
        """The sharded SSS walk with the per-iteration exchange on the device
        (psx_run_sss_sharded_dev): allgather_dev(send, recv, nbytes, stream)
        gets device addresses and the engine's hipStream_t and enqueues the
        all-gather of nbytes per rank on that stream (e.g. torch.distributed's
        all_gather_into_tensor on device_bytes views, with that stream current)."""
        err = []

        def cb(_ctx, send, recv, nbytes, stream):
            try:
                allgather_dev(int(send), int(recv), int(nbytes), int(stream or 0))
                return 0
            except BaseException as ex:  # reported through the engine's error code
                err.append(ex)
                return 1

        fn = ALLGATHER_DEV_FN(cb)
        it = ctypes.c_int32(0)
        rc = self.lib.psx_run_sss_sharded_dev(self.h, fn, None, ctypes.byref(it))
        if err:
            raise err[0]
        _check(rc)
        return it.value

    def eval_union_batch(self, sets: np.ndarray, accumulate: bool = False) -> np.ndarray:
        """sss_postcal.cpp:447 expand_and_compute_lkl over a batch; returns scores."""
        s = np.ascontiguousarray(sets, dtype=np.int32)
        out = np.empty(s.shape[0], dtype=np.float64)
        _check(self.lib.psx_eval_union_batch(self.h, _ptr(s, ctypes.c_int32), s.shape[1], s.shape[0],
                                             1 if accumulate else 0, _ptr(out, ctypes.c_double)))
        return out

    def reset(self):
        _check(self.lib.psx_reset(self.h))

    def accum(self) -> Accumulators:
        N, U = self.seam.N, self.seam.n_union
        post, noc = np.zeros(N), np.zeros(2)
        sh, sll, nsll = np.zeros(U), np.zeros(U), np.zeros(U)
        a = _Accum()
        a.post, a.no_causal = _ptr(post, ctypes.c_double), _ptr(noc, ctypes.c_double)
        a.shared, a.shared_ll = _ptr(sh, ctypes.c_double), _ptr(sll, ctypes.c_double)
        a.notshared_ll = _ptr(nsll, ctypes.c_double)
        _check(self.lib.psx_get_accum(self.h, ctypes.byref(a)))
        return Accumulators(post, noc, sh, sll, nsll, a.total, int(a.n_configs))

    def timing(self) -> dict:
        t = Timing()
        _check(self.lib.psx_get_timing(self.h, ctypes.byref(t)))
        return t.as_dict()

    def partials_bytes(self) -> int:
        return int(self.lib.psx_partials_bytes(self.h))

    def export_partials(self, device_ptr: int):
        _check(self.lib.psx_export_partials(self.h, ctypes.c_void_p(device_ptr)))

    def partials_device_ptr(self) -> int:
        """Device address of the handle's own partial image (read in place by a
        collective instead of an exported copy; valid until the next pass /
        merge / reset on this handle)."""
        p = ctypes.c_void_p()
        _check(self.lib.psx_partials_device_ptr(self.h, ctypes.byref(p)))
        return int(p.value)

    def partials_tensor(self):
        """The handle's own partial image as a uint8 torch tensor on its device
        (no copy: a view of psx_partials_device_ptr, for the collective to read
        in place)."""
        return device_bytes(self.partials_device_ptr(), self.partials_bytes())

    def merge_partials(self, device_ptr: int, count: int):
        _check(self.lib.psx_merge_partials(self.h, ctypes.c_void_p(device_ptr), int(count)))


class _DeviceSpan:
    """__cuda_array_interface__ of nbytes of device memory at ptr (uint8)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1", "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def device_bytes(ptr: int, nbytes: int):
    """A uint8 torch tensor viewing nbytes of device memory at ptr (no copy; the
    memory stays owned by the engine)."""
    import torch
    return torch.as_tensor(_DeviceSpan(ptr, nbytes), device="cuda")
