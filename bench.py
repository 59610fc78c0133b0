#!/usr/bin/env python3
"""bench.py — PostCal exhaustive sweep on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload syn1000c3]

A step is one full exhaustive sweep of the locus (every causal configuration,
postcal.cpp:716-1092) plus, for N > 1, the single RCCL all-gather + merge of
the per-GPU accumulators.  The locus is sharded across ranks (one process per
GPU under torch.distributed.run); the total work per step is fixed, so the
scaling is "strong".  Inputs are resident in HBM before the timed region.

Prints ONE JSON line on rank 0 (contract in the task statement), including
`roofline` for the dominant kernel (k_sweep<3>) and `cpu_baseline` (the
oracle's literal N x N restatement of the reference algorithm timed on the host
cores on a bounded sample of the same workload, rank 0 at N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

# torch first: its bundled HIP runtime then also serves the engine library
# (same SONAME), so device pointers from torch and from the engine are one space.
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from pipsort_amd import engine as E  # noqa: E402
from pipsort_amd import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (spec)
SIMDS = 256 * 4
CLOCK_HZ = 2.4e9          # peak engine clock (spec)
# SIMD cycles per wave64 VALU instruction on gfx950, measured by tools/valu_lat.hip
# with 4 waves per SIMD, 8 independent chains each (profiles/archive/r03a_valu_issue.txt):
# FP64 FMA / MUL / ADD and v_ldexp_f64 4.2 (the 16-lane FP64 pipe), v_rsq_f64
# 16.15, 32-bit integer / f32 ops 2.28 (the 32-lane pipe: half the FP64 cost)
VALU_CYCLES = {"fp64": 4.20, "fp64_trans": 16.15, "int32": 2.28, "other": 4.20}


def valu_issue_roof(pmc, kernel_s, world):
    """VALU issue roof of the dominant kernel with measured cycle weights per
    instruction class (PMC counts of the same build): FP64 FMA / MUL / ADD and
    FP64 transcendentals from their own counters, 32-bit integer ops from
    SQ_INSTS_VALU_INT32, the rest of SQ_INSTS_VALU (v_ldexp_f64, 64-bit moves /
    shifts / compares, DPP moves) at the FP64 rate (v_ldexp_f64 measured 4.2).
    Achieved = SIMD cycles the launch's instructions need / (1024 SIMDs x launch
    time); frac against the 2.4 GHz peak clock, and at the clock the chip held
    during the PMC run (GRBM_GUI_ACTIVE / 8 per launch time)."""
    c = pmc["counters_per_dispatch"]
    fp64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64"))
    trans = c.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
    int32 = c.get("SQ_INSTS_VALU_INT32", 0.0)
    other = max(0.0, c["SQ_INSTS_VALU"] - fp64 - trans - int32)
    cyc = (VALU_CYCLES["fp64"] * fp64 + VALU_CYCLES["fp64_trans"] * trans + VALU_CYCLES["int32"] * int32
           + VALU_CYCLES["other"] * other) / world
    need_s = cyc / SIMDS / CLOCK_HZ  # launch time at full issue, peak clock
    out = {"achieved": need_s / kernel_s * CLOCK_HZ / 1e9, "peak": CLOCK_HZ / 1e9, "unit": "G SIMD-cycles/s per SIMD",
           "frac": need_s / kernel_s,
           "simd_cycles_per_launch": cyc, "cycle_weights": VALU_CYCLES,
           "mix_per_launch": {"fp64": fp64 / world, "fp64_trans": trans / world, "int32": int32 / world,
                              "other": other / world},
           "source": "PMC instruction classes (profiles/pmc_latest.json) x cycles per instruction measured by "
                     "tools/valu_lat.hip (profiles/archive/r03a_valu_issue.txt) / (1024 SIMDs x kernel_ms)"}
    if pmc.get("gpu_cycles_per_launch") and world == 1:
        out["frac_at_measured_clock"] = cyc / SIMDS / pmc["gpu_cycles_per_launch"]
    return out

WORKLOADS = {
    # name: (M, c, p, n, description)
    "syn1000c3": (1000, 3, 0.25, (10000, 8000), "SYN-v1 2-study locus, M=1000 SNPs, -c 3 -p 0.25 -n 10000,8000"),
    "syn500c3": (500, 3, 0.25, (10000, 8000), "SYN-v1 2-study locus, M=500 SNPs, -c 3 -p 0.25 -n 10000,8000"),
    "syn200c2": (200, 2, 0.25, (10000, 8000), "SYN-v1 2-study locus, M=200 SNPs, -c 2 -p 0.25 -n 10000,8000"),
    "example": (None, 2, 0.25, (334324, 6771), "reference tests/example locus, -c 2 -p 0.25 -n 334324,6771"),
}


def _locus(name):
    M, c, p, n, _ = WORKLOADS[name]
    if M is None:
        import loci
        L = loci.read_locus("example")
        return (L["ld"], L["z"], L["u2l"], n), dict(max_causal=c, sharing_param=p)
    ld, z, _, _, u2l = synth.syn_v1(M)
    return (ld, z, u2l, n), dict(max_causal=c, sharing_param=p)


def build_seam(name):
    """PostCal's own inputs (B, S') through the host restatement of the reference
    Model setup (eigen route): what the CPU baseline's N x N likelihood needs."""
    args, kw = _locus(name)
    return E.seam_from_arrays(*args, **kw)


def build_inputs(name):
    """Model inputs (LD, z) for the engine: the setup runs on the GPU."""
    args, kw = _locus(name)
    return E.model_inputs(*args, **kw)


def host_cores():
    """Host cores this process may use: its CPU affinity set (what
    sched_getaffinity reports), and the cgroup CPU quota if one is set
    (/sys/fs/cgroup/cpu.max, in CPUs; None when unlimited)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return n, quota


def usable_cores():
    """Threads the CPU baselines run: min(affinity set, cgroup CPU quota), so
    `cores` counts CPUs the process can actually run on at once (256 threads on
    a 16-CPU quota would time 16 CPUs, oversubscribed)."""
    n, quota = host_cores()
    return max(1, min(n, int(quota))) if quota is not None else n


def cores_note(threads):
    n, quota = host_cores()
    return (f"{threads} host threads = min(the {n} CPUs of this process's affinity set, "
            + (f"cgroup CPU quota {quota:g})" if quota is not None else "no cgroup CPU quota)"))


def cores_fields(threads):
    n, quota = host_cores()
    return {"cores": threads, "affinity_cpus": n, "cgroup_cpu_quota": quota}


def cpu_baseline(seam, budget_s=15.0, threads=None):
    """Oracle literal (N x N, postcal.cpp:214-304) per-configuration cost on the
    host cores (usable_cores()), on a random sample of this workload's
    configurations."""
    from oracle import oracle as O
    threads = threads or usable_cores()
    U = seam.n_union
    k = int(seam.max_causal)
    rng = np.random.default_rng(0)
    both = (seam.union_to_local[0] >= 0) & (seam.union_to_local[1] >= 0)

    def sample(n):
        sets = np.sort(np.stack([rng.choice(U, k, replace=False) for _ in range(n)]), axis=1).astype(np.int32)
        bits = np.zeros((n, 2, k), dtype=np.int32)
        for i in range(n):
            for j in range(k):
                u = sets[i, j]
                if both[u]:
                    x = rng.integers(1, 4)
                else:
                    x = 1 if seam.union_to_local[0, u] >= 0 else 2
                bits[i, 0, j] = x & 1
                bits[i, 1, j] = (x >> 1) & 1
        return sets, bits

    O.load()
    done = [0] * threads
    stop = time.time() + budget_s
    work = [sample(4) for _ in range(threads)]

    def run(t):
        s, b = work[t]
        while time.time() < stop:
            O.eval_patterns(seam, s, b, literal=True)
            done[t] += s.shape[0]

    t0 = time.time()
    th = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.time() - t0
    n = sum(done)
    # The reference's own per-configuration cost (measured on
    # the reference built with OpenBLAS: -b path, 64 configurations, 1 thread):
    # 23.1 ms at N = 1000, 117.5 ms at N = 2000; it grows ~N^2 (N x N temporaries
    # and pinv per configuration), so other N scale from the N = 2000 point.
    N = int(seam.N)
    ref_ms = {1000: 23.1, 2000: 117.5}.get(N, 117.5 * (N / 2000.0) ** 2)
    per_thread = n / dt / threads
    return {"value": n / dt, "unit": "configs/s", **cores_fields(threads), "kind": "port",
            "kind_note": f"port: the oracle's literal N x N restatement without Armadillo's temporaries and pinv "
                         f"SVD, {per_thread * ref_ms / 1e3:.0f}x cheaper per configuration per thread than the "
                         f"reference's measured cost at N = {N}; a conservative stand-in, not the reference's "
                         f"OpenBLAS path",
            "reference_measured": {"ms_per_config_per_core": ref_ms, "configs_per_s_per_core": 1e3 / ref_ms,
                                   "N": N, "measured_at": "N = 1000 / 2000" if N in (1000, 2000) else
                                   "scaled as N^2 from N = 2000",
                                   "source": "SURVEY.md section 6 (reference built with OpenBLAS, -b path, "
                                             "64 configurations, 1 thread; 8-core Xeon)",
                                   "configs_per_s_64_cores_linear": 64e3 / ref_ms},
            "port_vs_reference_per_config": per_thread * ref_ms / 1e3,
            "sample": f"{n} random {k}-SNP configurations of this workload, oracle literal N x N "
                      f"restatement of lowrank_likelihood (postcal.cpp:214-304), {cores_note(threads)}, "
                      f"{dt:.1f} s"}


def example_patterns(seam):
    """Every configuration of an exhaustive sweep except the null one
    (postcal.cpp:716-1092: union subsets of size 1..c, then the per-study
    assignments passing checkOR), as (sets, bits) per level for
    oracle.eval_patterns."""
    import itertools
    u2l = seam.union_to_local
    allowed = []
    for u in range(seam.n_union):
        a0, a1 = u2l[0, u] >= 0, u2l[1, u] >= 0
        allowed.append([x for x in (1, 2, 3) if (x & 1 and a0 or not x & 1) and (x & 2 and a1 or not x & 2)])
    out = []
    for k in range(1, int(seam.max_causal) + 1):
        sets, bits = [], []
        for S in itertools.combinations(range(seam.n_union), k):
            for xs in itertools.product(*(allowed[u] for u in S)):
                sets.append(S)
                bits.append([[x & 1 for x in xs], [(x >> 1) & 1 for x in xs]])
        out.append((np.array(sets, dtype=np.int32), np.array(bits, dtype=np.int32)))
    return out


def cpu_baseline_example(threads=None):
    """BASELINE configs[0] (tests/example, -c 2 -p 0.25) on this box's host
    cores, in full: the oracle's literal N x N restatement of the reference
    likelihood (lowrank_likelihood, postcal.cpp:214-304) for all 216,817
    configurations, split over `threads` host threads.  The PIPs folded from its
    L values are checked against the reference's expected_study*_post.txt."""
    from oracle import oracle as O
    import loci
    threads = threads or usable_cores()
    seam = build_seam("example")
    levels = example_patterns(seam)
    O.load()
    work = []
    for sets, bits in levels:
        for ch in np.array_split(np.arange(sets.shape[0]), threads * 4):
            if ch.size:
                work.append((sets[ch], bits[ch], ch))
    res = [None] * len(work)
    nxt = [0]
    lock = threading.Lock()

    def run():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= len(work):
                return
            res[i] = O.eval_patterns(seam, work[i][0], work[i][1], literal=True)[0]

    t0 = time.time()
    th = [threading.Thread(target=run) for _ in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.time() - t0
    n = sum(s.shape[0] for s, _ in levels) + 1
    # fold: total and per-SNP post (log-sum-exp), null configuration L0 (postcal.cpp:802-803)
    L0 = -0.5 * float(np.dot(seam.s_prime, seam.s_prime)) - 1.0 + seam.n_union * np.log(1 - seam.gamma)
    m0 = int(seam.m[0])
    Ls, members = [np.array([L0])], []
    wi = 0
    for sets, bits in levels:
        Lk = np.empty(sets.shape[0])
        while wi < len(work) and work[wi][0].shape[1] == sets.shape[1]:
            Lk[work[wi][2]] = res[wi]
            wi += 1
        Ls.append(Lk)
        members.append((sets, bits, Lk))
    allL = np.concatenate(Ls)
    mx = allL.max()
    total = mx + np.log(np.exp(allL - mx).sum())
    acc = np.zeros(seam.N)
    for sets, bits, Lk in members:
        w = np.exp(Lk - total)
        for s in range(2):
            for j in range(sets.shape[1]):
                sel = bits[:, s, j] == 1
                loc = seam.union_to_local[s, sets[sel, j]] + s * m0
                np.add.at(acc, loc, w[sel])
    ok = True
    for s in range(2):
        exp = [float(l.split()[1]) for l in open(os.path.join(loci.GOLDEN, "example", f"expected_study{s}_post.txt"))
               .read().splitlines()[1:]]
        got = acc[s * m0: s * m0 + len(exp)]
        ok = ok and bool(np.all(np.abs(got - np.array(exp)) <= 5e-6 * np.maximum(np.abs(exp), 1e-300) + 1e-12))
    return {"value": n / dt, "unit": "configs/s", **cores_fields(threads), "kind": "port", "wall_s": dt, "configs": n,
            "pips_match_reference_expected": ok,
            "reference_measured": {"wall_s_8_cores": 117.4, "wall_s_1_core": 870.7, "wall_64_cores_readme": "< 2 min",
                                   "configs_per_s_8_cores": 1847,
                                   "source": "SURVEY.md section 6 (reference -O3, OpenBLAS; README.md:85 for 64 "
                                             "processors)"},
            "sample": f"full tests/example c=2 sweep ({n} configurations), oracle literal N x N restatement of "
                      f"lowrank_likelihood (postcal.cpp:214-304), {cores_note(threads)}; PIPs checked against "
                      f"expected_study*_post.txt (6 digits)"}


def sss_batch(M):
    """The SSS neighbourhood of the 4-SNP configuration {M/4 - 1, M/4, 3M/4,
    3M/4 + 1} (sss_postcal.cpp:20-99): 4 x (M - 4) swaps, 4 removals, M - 4
    additions, -1 padded to 5; and its pattern count."""
    cur = [M // 4 - 1, M // 4, 3 * M // 4, 3 * M // 4 + 1]
    rest = [u for u in range(M) if u not in cur]
    sets = []
    for i in range(4):  # swaps (nbdzero)
        keep = [c for j, c in enumerate(cur) if j != i]
        sets += [sorted(keep + [u]) + [-1] for u in rest]
    sets += [sorted([c for j, c in enumerate(cur) if j != i]) + [-1, -1] for i in range(4)]  # nbdminus
    sets += [sorted(cur + [u]) for u in rest]  # nbdplus
    arr = np.array(sets, dtype=np.int32)
    return arr, int(sum(3 ** int((r >= 0).sum()) for r in arr))


def sss_probe(reps=20):
    """BASELINE configs[4]: the SSS path (sss_postcal.cpp:102-380) on SYN-v1
    M = 2000, -c 5 — the walk itself, and the throughput of one SSS proposal
    batch (the neighbourhood of a 4-SNP configuration, sss_postcal.cpp:20-99:
    4 x 1996 swaps, 4 removals, 1996 additions) through psx_eval_union_batch
    with accumulation, inputs resident on the device."""
    M = 2000
    ld, z, _, _, u2l = synth.syn_v1(M)
    mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=5, sharing_param=0.25)
    pc = E.PostCal(mi)
    setup_ms = pc.setup_info["setup_ms"]
    t0 = time.perf_counter()
    iters = pc.run_sss()
    walk_ms = (time.perf_counter() - t0) * 1e3
    walk_configs = pc.accum().n_configs
    arr, npat = sss_batch(M)
    sets = arr
    pc.eval_union_batch(arr, accumulate=True)
    torch.cuda.synchronize()
    # the timed calls alone (each call returns after the batch is folded and its
    # scores are on the host); the kernel time is read on separate calls after
    t0 = time.perf_counter()
    for _ in range(reps):
        pc.eval_union_batch(arr, accumulate=True)
    batch_ms = (time.perf_counter() - t0) * 1e3 / reps
    kms = []
    for _ in range(5):
        pc.eval_union_batch(arr, accumulate=True)
        kms.append(pc.timing()["kernel_ms"])  # the batch's k_eval_batch launch (HIP events)
    pc.close()
    roof = sss_roofline(len(sets), npat, sum(kms) / len(kms))
    return {"workload": "SYN-v1 2-study locus, M=2000 SNPs, -c 5 -p 0.25 -n 10000,8000 (BASELINE configs[4])",
            "gpu_model_setup_and_create_ms": setup_ms, "walk_iterations": iters, "walk_configs": walk_configs,
            "walk_ms": walk_ms, "batch_sets": len(sets), "batch_configs": npat, "batch_ms": batch_ms,
            "batch_configs_per_s": npat / (batch_ms / 1e3), "roofline": roof, "long_walks": sss_long_walks(),
            "multi_gpu": "sharded under --gpus N (psx_run_sss_sharded: every iteration's batch split over the "
                         "ranks, one all-gather of scores per iteration); this N = 1 line times one GPU"}


def sss_roofline(n_sets, npat, kernel_ms):
    """The batch's dominant kernel, k_eval_batch5 (k_eval_batch for rows of 6
    members; a wave per union set: 2^k
    subset LDL^T per study, then the 3^k assignments), is FP64 VALU work:
    achieved = FP64 operations of one launch (PMC SQ_INSTS_VALU_FLOPS_FP64 x 64
    of this very build and batch shape, profiles/pmc_latest.json "sss_eval") /
    its launch duration measured here (HIP events around the launch)."""
    out = {"bound": "valu_fp64", "kernel": "k_eval_batch5", "kernel_ms": kernel_ms, "peak": FP64_PEAK_TFLOPS,
           "unit": "TFLOP/s", "kernel_configs_per_s": npat / (kernel_ms / 1e3) if kernel_ms > 0 else None,
           "duration_source": "HIP events around the launch on the engine stream (psx_get_timing), mean of reps",
           "achieved": None, "frac": None, "eval_src_sha": eval_src_sha()}
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        ev = json.load(open(p)).get("sss_eval") or {}
    except Exception:
        ev = {}
    if (ev.get("eval_src_sha") == out["eval_src_sha"] and ev.get("grid_size") == 64 * n_sets
            and ev.get("fp64_flop_insts_per_launch") and kernel_ms > 0):
        flops = ev["fp64_flop_insts_per_launch"] * 64.0
        out.update(achieved=flops / (kernel_ms / 1e3) / 1e12, flops_per_launch=flops,
                   flops_source="PMC SQ_INSTS_VALU_FLOPS_FP64 x 64 (profiles/pmc_latest.json sss_eval, same build)")
        out["frac"] = out["achieved"] / FP64_PEAK_TFLOPS
        c = ev.get("counters_per_dispatch", {})
        if c.get("SQ_INSTS_VALU"):
            out["fp64_valu_share"] = sum(c.get(k, 0.0) for k in (
                "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                "SQ_INSTS_VALU_TRANS_F64")) / c["SQ_INSTS_VALU"]
    else:
        out["flops_source"] = "no PMC counters of this build / batch shape (profiles/pmc_latest.json sss_eval)"
    return out


def sss_long_walks(reps=3):
    """The seeded walk at configs[4] stops after 2 iterations, so the host side
    of the walk (neighbourhoods, set map, sampling, one GPU round trip per
    iteration) is timed on SYN-v1 loci whose walks run long: M = 100 (22
    iterations, climbing to 5-SNP sets) and M = 200 (100 iterations, the
    convergence stop of sss_postcal.cpp:265-270), -c 5.  The M = 100 walk is
    also timed through the oracle's restated walk on one host core (the
    cpu_baseline leg's port; M = 200 takes it ~70 s)."""
    from oracle import oracle as O
    out = []
    for M in (100, 200):
        ld, z, _, _, u2l = synth.syn_v1(M)
        mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=5, sharing_param=0.25)
        pc = E.PostCal(mi)
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            it = pc.run_sss()
            dt = (time.perf_counter() - t0) * 1e3
            if best is None or dt < best[0]:
                best = (dt, it, pc.timing()["kernel_ms"])
        n = pc.accum().n_configs
        pc.close()
        dt, it, kms = best
        row = {"locus": f"SYN-v1 M={M} -c 5", "iterations": it, "configs": n, "walk_ms": dt,
               "kernel_ms": kms, "ms_per_iteration": dt / max(it, 1), "configs_per_s": n / (dt / 1e3)}
        if M == 100:
            seam = E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=5, sharing_param=0.25)
            # the restated walk prints the reference's stop message on stdout,
            # which carries only the bench line: send fd 1 to stderr meanwhile
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                t0 = time.perf_counter()
                ref = O.postcal(seam, "sss")
                row["cpu_port_walk_ms"] = (time.perf_counter() - t0) * 1e3
            finally:
                import ctypes
                ctypes.CDLL(None).fflush(None)  # C stdio's buffered copy of the message
                os.dup2(saved, 1)
                os.close(saved)
            row["cpu_port_cores"] = 1
            row["cpu_port_configs_match"] = int(ref["n_configs"]) == int(n)
        out.append(row)
    return out


def configs_probe(reps=3):
    """The -b configs-file enumerator (postcal.cpp:400-714) at scale: a file
    made by the restated generator (synth.construct_configs =
    utils/construct_configs_all_studies.py:50-158) for SYN-v1 M = 1000 with
    three 12-SNP groups per study around the planted signals: 13^6 = 4,826,809
    rows of 6 int16 global indices.  Timed: psx_run_configs from the host rows
    (parallel host row preprocessing, one upload, the GPU evaluation and
    merges), inputs already set up on the GPU; best of `reps`."""
    M = 1000
    ld, z, _, _, u2l = synth.syn_v1(M)
    mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=3, sharing_param=0.25)
    grp = [list(range(c - 6, c + 6)) for c in (M // 4, M // 2, 3 * M // 4)]
    rows = synth.construct_configs([grp, grp], [M, M])
    pc = E.PostCal(mi)
    pc.run_configs(rows)  # warm-up (buffers)
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pc.run_configs(rows)
        dt = time.perf_counter() - t0
        if best is None or dt < best[0]:
            best = (dt, pc.timing())
    n = pc.accum().n_configs
    pc.close()
    dt, tm = best
    return {"workload": "SYN-v1 M=1000 -c 3, -b file of 3 x 12-SNP groups per study (construct_configs_all_studies)",
            "rows": int(rows.shape[0]), "n_groups": int(rows.shape[1]), "configs_checked": int(n),
            "wall_ms": dt * 1e3, "configs_per_s": rows.shape[0] / dt, "kernel_ms": tm["kernel_ms"],
            "note": "rows -> one upload -> the device row walk (validation, index maps, evaluation: psx_configs.hip) "
                    "+ merges; best of %d" % reps}


def torch_allgather(backend):
    """psx_allgather_fn over torch.distributed (RCCL for nccl, host for gloo)."""
    world = dist.get_world_size()

    def ag(b: bytes) -> bytes:
        dev = "cuda" if backend == "nccl" else "cpu"
        x = torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
        out = torch.empty(len(b) * world, dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(out, x)
        return out.cpu().numpy().tobytes()
    return ag


def sss_probe_sharded(rank, world, backend):
    """BASELINE configs[4] on `world` GPUs: the walk with every iteration's
    batch split across the ranks (psx_run_sss_sharded, one all-gather of the
    slices' scores per iteration), then the accumulator exchange."""
    M = 2000
    ld, z, _, _, u2l = synth.syn_v1(M)
    mi = E.model_inputs(ld, z, u2l, (10000, 8000), max_causal=5, sharing_param=0.25)
    pc = E.PostCal(mi)
    pc.set_shard(rank, world)
    dev = backend == "nccl"
    if dev:
        # the per-iteration exchange stays on the device: RCCL all-gather of the
        # engine's device send block, ordered on the engine stream (torch's current)
        stream = torch.cuda.current_stream()
        pc.set_stream(stream.cuda_stream)

        def agd(send, recv, nbytes, _stream):
            dist.all_gather_into_tensor(E.device_bytes(recv, nbytes * world), E.device_bytes(send, nbytes))

        run = lambda: pc.run_sss_sharded_dev(agd)  # noqa: E731
    else:
        ag = torch_allgather(backend)
        run = lambda: pc.run_sss_sharded(ag)  # noqa: E731
    run()  # warm-up (allocations, collective setup)
    dist.barrier()
    t0 = time.perf_counter()
    iters = run()
    nb = pc.partials_bytes()
    gathered = torch.empty(nb * world, dtype=torch.uint8, device="cuda")
    if dev:
        dist.all_gather_into_tensor(gathered, pc.partials_tensor())
    else:
        mine = torch.empty(nb, dtype=torch.uint8, device="cuda")
        pc.export_partials(mine.data_ptr())
        torch.cuda.synchronize()
        gathered.copy_(torch.frombuffer(bytearray(ag(mine.cpu().numpy().tobytes())), dtype=torch.uint8))
    pc.merge_partials(gathered.data_ptr(), world)
    pc.sync()
    torch.cuda.synchronize()
    walk_ms = (time.perf_counter() - t0) * 1e3
    x = torch.tensor([walk_ms], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    dist.all_reduce(x, op=dist.ReduceOp.MAX)
    n = pc.accum().n_configs
    pc.close()
    return {"workload": "SYN-v1 2-study locus, M=2000 SNPs, -c 5 -p 0.25 -n 10000,8000 (BASELINE configs[4])",
            "walk_iterations": iters, "walk_configs": n, "walk_ms_incl_exchange": float(x.item()),
            "multi_gpu": f"batch split over {world} ranks, one all-gather of scores per iteration "
                         + ("on the device (psx_run_sss_sharded_dev, RCCL on the engine stream)" if dev else
                            "(psx_run_sss_sharded, host-staged)") + " + one accumulator exchange"}


def pcie_inclusive(mi, configs, device, reps=3):
    """Whole-locus rate from host buffers to host results: the GPU Model setup
    from the host LD / z arrays (H2D included), one synchronous exhaustive
    pass, and the accumulators read back to the host (psx_get_accum, D2H).
    Not the bench value (inputs are not resident): reported beside it, split
    into phases (best repetition)."""
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pc = E.PostCal(mi, device=device)
        t1 = time.perf_counter()
        pc.run_exhaustive()
        t2 = time.perf_counter()
        pc.accum()
        t3 = time.perf_counter()
        dt = t3 - t0
        si = pc.setup_info
        tm = pc.timing()
        ph = {"create_ms": (t1 - t0) * 1e3,
              "setup_ms": si["setup_ms"],
              "setup_alloc_ms": si.get("alloc_ms"), "setup_studies_ms": si.get("studies_ms"),
              "setup_tail_ms": si.get("tail_ms"),
              "study_upload_ms": si.get("study_upload_ms"), "study_psd_lu_ms": si.get("study_psd_ms"),
              "study_finish_ms": si.get("study_finish_ms"),
              "first_pass_ms": (t2 - t1) * 1e3,
              "pass_prepare_ms": tm.get("prepare_ms"),
              "pass_kernel_ms": tm.get("kernel_ms"),
              "readback_ms": (t3 - t2) * 1e3}
        pc.close()
        if best is None or dt < best[0]:
            best = (dt, ph)
    return {"value": configs / best[0], "unit": "configs/s", "s": best[0], "setup_ms": best[1]["setup_ms"],
            "phases": best[1],
            "note": "host LD/z -> GPU Model setup (H2D) -> one synchronous pass -> accumulators on the host "
                    "(D2H); best of %d" % reps}


def example_wall():
    """Wall-clock of the drop-in PIPSORT CLI on tests/example (-c 2 -p 0.25)."""
    import loci
    src = os.path.join(loci.GOLDEN, "example")
    with tempfile.TemporaryDirectory() as d:
        for f in os.listdir(src):
            if not f.startswith("expected_"):
                os.symlink(os.path.join(src, f), os.path.join(d, f))
        t0 = time.time_ns()
        env = dict(os.environ, PSX_TIMING="1", PSX_T0=str(t0))
        r = subprocess.run([E.PIPSORT_BIN, "-c", "2", "-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "snp_map",
                            "-n", "334324,6771", "-p", "0.25", "-o", "out"], cwd=d, capture_output=True, text=True,
                           env=env)
        t1 = time.time_ns()
        wall = (t1 - t0) / 1e9
        same = all(open(os.path.join(d, f"out_{f}.txt")).read() ==
                   open(os.path.join(src, f"expected_{f}.txt")).read()
                   for f in ("study0_post", "study1_post", "study0_set", "study1_set", "nocausal"))
    phases, warm, setup_split = None, None, None
    for line in r.stderr.splitlines():
        if line.startswith("psx-timing "):
            phases = json.loads(line[len("psx-timing "):])
        elif line.startswith("psx-warm "):  # psx_warmup_for's split of context_and_code_load
            warm = json.loads(line[len("psx-warm "):])
        elif line.startswith("psx-setup "):  # psx_create_from_ld's phases (gpu_setup_ms)
            setup_split = json.loads(line[len("psx-setup "):])
    if phases:
        # process exit (teardown of the HIP runtime, unmapping) until the parent sees it
        phases["exit_ms"] = t1 / 1e6 - phases.pop("end_epoch_ms")
        phases["sum_ms"] = sum(v for k, v in phases.items() if k.endswith("_ms"))
        phases["note"] = ("to_main = exec + dynamic loading; the HIP runtime and context come up on a second "
                          "thread during parsing (hip_runtime, context_and_code_load), wait_for_gpu is what the "
                          "main thread still waits for them after parsing; sum_ms adds the main-thread phases")
        # the concurrent warm-up phases are not on the main thread's path
        phases["sum_ms"] -= phases["hip_runtime_ms"] + phases["context_and_code_load_ms"]
        if warm:
            phases["context_and_code_load_split"] = warm
        if setup_split:
            phases["gpu_setup_split"] = setup_split
    return (wall if r.returncode == 0 else None), same, phases


KERNEL_SOURCES = ("psx_sweep3.hip", "psx_wave.h", "psx_sweep_dev.h", "psx_sweep_unit.h", "psx_math.h", "psx_sweep.h")


def kernel_src_sha():
    """Hash of the sources k_sweep3 is compiled from: a PMC summary describes
    this build only if it carries the same hash (tools/pmc_summary.py)."""
    import hashlib
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        with open(os.path.join(ROOT, "pipsort_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


EVAL_SOURCES = ("psx_engine.hip", "psx_wave.h", "psx_math.h", "psx_sweep_dev.h")


def eval_src_sha():
    """Hash of the sources k_eval_batch (the SSS batch evaluator) is built from."""
    import hashlib
    h = hashlib.sha256()
    for f in EVAL_SOURCES:
        with open(os.path.join(ROOT, "pipsort_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def load_pmc(workload):
    """profiles/pmc_latest.json (rocprofv3 --pmc passes, tools/gpu_pmc.sh +
    tools/pmc_summary.py) if it was collected on this workload AND this build
    of the kernel; else None."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        if d.get("workload") == workload and d.get("kernel_src_sha") == kernel_src_sha():
            return d
    except Exception:
        pass
    return None


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): start N ranks,
    one process per GPU, as a torch.distributed.run child — before this process
    touches the GPU (device_count() does not create a context) — and exit with
    its status.  Rank 0 prints the bench line on the inherited stdout.  The
    whole-node analogue of the reference's 64 OpenMP threads
    (postcal.cpp:747-769)."""
    import socket
    backend = os.environ.get("PSX_DIST_BACKEND", "nccl")
    have = torch.cuda.device_count()
    if backend == "nccl" and have < n:
        print(f"bench: --gpus {n} but only {have} HIP device(s) visible", file=sys.stderr)
        return 2
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="syn1000c3", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    args = ap.parse_args()
    # integrity: a timing-ablation switch (results wrong) never produces a line
    ablate = sorted(k for k in os.environ if k.startswith("PSX_ABLATE"))
    if ablate:
        print(f"bench: refusing to run with timing-ablation variables set: {ablate}", file=sys.stderr)
        sys.exit(3)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    # the bench line must be the only thing on stdout: native libraries print
    # banners there (RCCL prints its version block at communicator init), so
    # fd 1 is pointed at stderr for the whole run and the line is written to a
    # saved copy of the original stdout
    sys.stdout.flush()
    line_fd = os.dup(1)
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
    # PSX_DIST_BACKEND=gloo lets a multi-rank run share one GPU for validation
    # (host-staged exchange); the real path is nccl = RCCL over xGMI, one GPU per rank.
    backend = os.environ.get("PSX_DIST_BACKEND", "nccl")
    if backend == "nccl" and world > 1 and torch.cuda.device_count() < world:
        print(f"bench: {world} ranks but only {torch.cuda.device_count()} HIP device(s)", file=sys.stderr)
        sys.exit(2)
    # PSX_FORCE_DIST=1 takes the multi-rank code path even at world 1 (under
    # torch.distributed.run): the RCCL calls of the exchange then run on a
    # one-GPU box, as a check of the N > 1 path (not a bench line)
    use_dist = world > 1 or bool(os.environ.get("PSX_FORCE_DIST"))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    t_setup = time.time()
    seam = build_inputs(args.workload)
    t_synth = time.time() - t_setup
    configs_per_step = seam.count_configs()
    pc = E.PostCal(seam, device=local)  # Model setup + PostCal construction on the GPU
    pc.set_shard(rank, world)
    plan_hash = pc.plan_hash()
    if use_dist:
        # every rank must cut the same shard plan (PSX_K3_* knobs are read per
        # process); the merge refuses mismatched images too, this fails early
        hs = [None] * world
        dist.all_gather_object(hs, plan_hash)
        if len(set(hs)) != 1:
            print(f"bench: ranks cut different shard plans: {hs}", file=sys.stderr)
            sys.exit(4)
    # one stream for torch (collectives, copies) and the engine: the exchange is
    # ordered by the stream, no host synchronisation between export and merge
    stream = torch.cuda.Stream(priority=-1)  # high: merges + exchange ahead of the sweeps
    torch.cuda.set_stream(stream)
    pc.set_stream(stream.cuda_stream)
    nbytes = pc.partials_bytes()
    mine = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    gathered = torch.empty(nbytes * world, dtype=torch.uint8, device="cuda")
    setup_s = time.time() - t_setup

    use_async = not os.environ.get("PSX_BENCH_SYNC")
    step_sync = bool(os.environ.get("PSX_BENCH_STEPSYNC"))  # A/B: psx_sync after every asynchronous pass

    def step():
        # the pass is enqueued without a host sync; the exchange is ordered after
        # it on the same stream, so consecutive steps pipeline on the device
        if use_async:
            pc.run_exhaustive_async()
        else:
            pc.run_exhaustive()
        if use_dist:
            pc.export_partials(mine.data_ptr())  # enqueued on torch's current stream
            if backend == "nccl":
                dist.all_gather_into_tensor(gathered, mine)  # the one exchange step (RCCL over xGMI)
            else:
                parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
                dist.all_gather(parts, mine.cpu())
                gathered.copy_(torch.cat(parts))
            pc.merge_partials(gathered.data_ptr(), world)  # ordered after the collective
        if use_async and step_sync:
            step_exact[0] |= bool(pc.sync())
            step_t.append(pc.timing())

    step_exact = [False]
    step_t = []

    def timed():
        kms, launches = 0.0, 0
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        pc.sync()
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
            if not use_async:
                t = pc.timing()
                kms += t["kernel_ms"]
                launches += t["kernel_launches"]
        torch.cuda.synchronize()
        if use_dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        exact = pc.sync()  # EXACT flag of any pass (OR-ed over ranks by the merge)
        if use_async and step_sync:  # the passes were synced (and timed) one by one
            ts = step_t[-args.steps:]
            exact = exact or step_exact[0]
            kms, launches = sum(t["kernel_ms"] for t in ts), sum(t["kernel_launches"] for t in ts)
        elif use_async:
            t = pc.timing()
            kms, launches = t["kernel_ms"], t["kernel_launches"]
        return elapsed, kms, launches, exact

    elapsed, kms, launches, exact = timed()

    def single_passes(n=15):
        """One locus swept once (what a real per-locus run and the CLI see): each
        pass = psx_run_exhaustive_async + (N > 1) the exchange + psx_sync, with
        nothing overlapping the next pass; median host wall per pass (all ranks
        start together: barrier before each)."""
        ws = []
        for i in range(n + 2):
            if use_dist:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pc.run_exhaustive_async()
            if use_dist:
                if backend == "nccl":
                    dist.all_gather_into_tensor(gathered, mine_view)  # the image read in place
                else:
                    parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
                    dist.all_gather(parts, mine_view.cpu())
                    gathered.copy_(torch.cat(parts))
                pc.merge_partials(gathered.data_ptr(), world)
            pc.sync()
            dt = (time.perf_counter() - t0) * 1e3
            if i >= 2:
                ws.append(dt)
        if use_dist:
            x = torch.tensor(ws, dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
            dist.all_reduce(x, op=dist.ReduceOp.MAX)
            ws = x.tolist()
        ws.sort()
        return ws[len(ws) // 2]

    if exact and use_async:
        # some pass needs the exact notSharedLL variant: the asynchronous results
        # are not valid, time the validated synchronous path instead
        print("bench: EXACT rerun needed, timing the synchronous path", file=sys.stderr)
        use_async = False
        elapsed, kms, launches, _ = timed()
    if use_dist:
        x = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        elapsed = float(x.item())
    tm = pc.timing()
    torch.cuda.synchronize()
    mine_view = pc.partials_tensor() if use_dist else None
    single_pass_ms = single_passes() if use_async else None  # after the timed region (and its timing)
    acc = pc.accum() if (world == 1 or rank == 0) else None

    sss_line = None
    if use_dist:  # after the timed region; a failure here must not lose the bench line
        try:
            sss_line = sss_probe_sharded(rank, world, backend)
        except Exception as ex:  # noqa: BLE001
            sss_line = {"error": f"{type(ex).__name__}: {ex}"}
    if rank == 0 and (acc is None or int(acc.n_configs) != configs_per_step):
        # integrity: the merged accumulators must hold every configuration once
        print(f"bench: configurations checked {None if acc is None else acc.n_configs} != "
              f"{configs_per_step} per step; no line", file=sys.stderr)
        sys.exit(5)
    if rank == 0:
        value = configs_per_step * args.steps / elapsed
        avg_kernel_s = (kms / max(launches, 1)) / 1e3
        dur_src = ("average launch duration (in-kernel wall clocks: the sweep's first block's start to the "
                   "merge's first block's start; serial passes on one stream, no dispatch events)" if world == 1
                   and not os.environ.get("PSX_SERIAL") else
                   "average launch duration (start / stop events in the sweep's own dispatch packet)")
        span_s = (tm.get("span_ms") or 0.0) / 1e3 if use_async else 0.0
        if 0 < span_s < avg_kernel_s:
            # overlapped passes (worlds >= 4): launches overlap, so a launch's own
            # duration counts its neighbour's; the per-pass device span is the cost
            avg_kernel_s = span_s
            dur_src = "per-pass device span (first sweep start to last sweep end / passes; launches overlap)"
        alg_bytes = tm["alg_bytes"]  # per launch of the dominant kernel (this rank's shard)
        pmc = load_pmc(args.workload)
        # The binding roof of k_sweep3 is FP64 VALU issue, not HBM:
        # achieved = FP64 operations of one launch (PMC SQ_INSTS_VALU_FLOPS_FP64,
        # FMA = 2, per wave instruction x 64 lanes, collected on this build) / the
        # launch's average duration measured here (HIP events of its own dispatch).
        if pmc and pmc.get("fp64_flop_insts_per_launch"):
            # counters of the world-1 launch; a shard of `world` equal-work slices does 1/world of it
            flops = pmc["fp64_flop_insts_per_launch"] * 64.0 / world
            flops_src = ("PMC SQ_INSTS_VALU_FLOPS_FP64 x 64 (profiles/pmc_latest.json, same kernel build)"
                         + (f" / {world} (this rank's shard)" if world > 1 else ""))
        else:
            flops = tm["flops"]
            flops_src = ("model: 131 FP64 operations per 3-SNP union set (fitted to the PMC count of the last "
                         "collected build, a lower bound for later ones) - NOT counters of this build")
        achieved = flops / avg_kernel_s / 1e12 if avg_kernel_s > 0 else 0.0
        # the roofline fraction is reported only from counters of this very build;
        # without them the model's figure goes to a separately named field
        have_pmc = bool(pmc and pmc.get("fp64_flop_insts_per_launch"))
        roofline = {"bound": "valu_fp64", "achieved": achieved if have_pmc else None, "peak": FP64_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS if have_pmc else None,
                    "traffic": (pmc or {}).get("hbm_bytes_per_launch") if world == 1 else None,
                    "kernel": "k_sweep3" if seam.max_causal >= 3 else "k_sweep<2>",
                    "kernel_ms": avg_kernel_s * 1e3, "duration_source": dur_src,
                    "flops_per_launch": flops, "flops_source": flops_src,
                    "pmc_kernel_src_sha": (pmc or {}).get("kernel_src_sha"), "kernel_src_sha": kernel_src_sha()}
        if not have_pmc:
            roofline["model_achieved"] = achieved
            roofline["model_frac"] = achieved / FP64_PEAK_TFLOPS
        if pmc and pmc.get("valu_insts_per_launch") and avg_kernel_s > 0:
            roofline["valu_issue"] = valu_issue_roof(pmc, avg_kernel_s, world)
        if pmc and world == 1:
            roofline["valu_busy"] = pmc.get("valu_busy")
            roofline["fp64_valu_share"] = pmc.get("fp64_valu_share")
            if pmc.get("hbm_bytes_per_launch") and avg_kernel_s > 0:
                gbs = pmc["hbm_bytes_per_launch"] / avg_kernel_s / 1e9
                roofline["hbm"] = {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                                   "source": "PMC 2 x FETCH_SIZE + WRITE_SIZE per launch / kernel_ms"}
        # SURVEY 8(d)'s per-configuration byte count, kept as a labelled
        # diagnostic only: the kernel reuses each gathered operand from
        # registers / LDS across 3^k assignments and 64 lanes, so these bytes
        # never cross HBM and their "rate" is not bounded by any roof
        alg_diag = {"bytes_per_launch": alg_bytes,
                    "rate_GBs": alg_bytes / avg_kernel_s / 1e9 if avg_kernel_s > 0 else 0.0,
                    "note": "SURVEY 8(d) 8*sum_s(|C_s|^2+|C_s|) per configuration; register/LDS-reused, not HBM traffic"}
        out = {
            "metric": "causal configurations evaluated/sec (whole node)",
            "value": value,
            "unit": "configs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic" if args.workload != "example" else "reference fixture",
            "config": {"workload": WORKLOADS[args.workload][4], "union_snps": seam.n_union,
                       "max_causal": int(seam.max_causal), "configs_per_step": configs_per_step,
                       "parallelism": (f"config-shard x{world} + 1 {'RCCL' if backend == 'nccl' else backend} all-gather"
                            if use_dist else "single GPU")},
            "roofline": roofline,
            "algorithmic_bytes_diagnostic": alg_diag,
            "rccl_world": dist.get_world_size() if use_dist else 1,
            "setup_s": setup_s,
            "setup": {"synthetic_locus_s": t_synth, "gpu_model_setup_and_create_ms": pc.setup_info["setup_ms"],
                      "psd_added": pc.setup_info["psd_added"], "eigen_route": pc.setup_info["eigen_route"]},
            "pass_mode": "async (no host sync per step)" if use_async else "synchronous",
            "single_pass_ms": single_pass_ms,
            "single_pass_note": "one pass of this rank's shard from the host call to merged accumulators "
                                "(psx_run_exhaustive_async + exchange + psx_sync, nothing overlapping), median of "
                                "15, max over ranks; setup excluded — the latency of sweeping one locus once",
            # CUs kept for the merges / exchange beside overlapped passes (one XCD
            # at world >= 8 by default, PSX_OVERLAP overrides; 0: not overlapped)
            "overlap_reserved_cus": pc.overlap_cus(),
            "span_ms_per_pass": tm.get("span_ms") if use_async else None,
            "configs_checked": int(acc.n_configs) if acc is not None else None,
            "plan_hash": f"{plan_hash:016x}",
            # every engine environment knob in force (plan shape, overlap, sync mode)
            "env_knobs": {k: v for k, v in sorted(os.environ.items()) if k.startswith("PSX_")},
        }
        if use_dist:
            out["sss"] = sss_line
        else:
            out["pcie_inclusive"] = pcie_inclusive(seam, configs_per_step, local)
            out["sss"] = sss_probe()
            try:
                out["configs_file"] = configs_probe()
            except Exception as ex:  # noqa: BLE001  (a side measurement must not lose the line)
                out["configs_file"] = {"error": f"{type(ex).__name__}: {ex}"}
            w, same, phases = example_wall()
            out["example_wall_s"] = w
            out["example_outputs_match_reference"] = same
            out["example_wall_phases"] = phases
            if not args.no_cpu_baseline:
                # BASELINE configs[0] on the same box: the north star's >= 100x is
                # cpu_baseline_example.wall_s / example_wall_s
                out["cpu_baseline_example"] = cpu_baseline_example()
                if w:
                    out["cpu_baseline_example"]["speedup_vs_example_wall"] = out["cpu_baseline_example"]["wall_s"] / w
                # the reference's N x N likelihood needs B and S': host eigen route
                out["cpu_baseline"] = cpu_baseline(build_seam(args.workload), budget_s=args.cpu_budget)
        sys.stdout.flush()
        os.write(line_fd, (json.dumps(out) + "\n").encode())
    pc.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
