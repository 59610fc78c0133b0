#!/usr/bin/env python3
"""Golden per-SNP accumulators of the full-size SYN-v1 loci (BASELINE configs[2]
and configs[3]: M = 500 and M = 1000, c = 3, p = 0.25, n = 10000,8000).

For EVERY union SNP u this writes the oracle's exact sums over all union sets
containing u (oracle.member_sums: long-double log-sum-exp over the 3^k study
assignments, the checker pinned to the whole-sweep oracle by
tests/test_oracle_golden.py::test_member_sums_checker_matches_whole_oracle):
post (study 0, study 1), sharedPips, sharedLL and notSharedLL as the reference
holds them (postcal.cpp:981-1030, log values, 0 = empty), one line per SNP,
%.17g.  The GPU tests compare every line with no oracle call on the GPU box.

The oracle input is the Cholesky seam (oracle.cholesky_seam), equal to the
eigen route's in exact arithmetic.  Run in this container (hours of CPU at
M = 1000); resumable: SNPs already in the output file are skipped.

usage: python tests/golden/fullsize/make_member_sums.py M [threads]
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", "..", ".."))
sys.path.insert(0, ROOT)

from pipsort_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

M = int(sys.argv[1])
threads = int(sys.argv[2]) if len(sys.argv) > 2 else len(os.sched_getaffinity(0))
out = os.path.join(HERE, f"syn{M}c3_member_sums.txt")
ld, z, _, _, u2l = synth.syn_v1(M)
seam = O.cholesky_seam(ld, z, u2l, (10000, 8000), max_causal=3, sharing_param=0.25)
done = set()
if os.path.exists(out):
    for line in open(out):
        if line.strip() and not line.startswith("#"):
            done.add(int(line.split()[0]))
else:
    with open(out, "w") as f:
        f.write(f"# SYN-v1 M={M} c=3 p=0.25 n=10000,8000: u post0 post1 shared shared_ll notshared_ll n_patterns\n")
t0 = time.time()
with open(out, "a") as f:
    for u in range(seam.union_to_local.shape[1]):
        if u in done:
            continue
        r = O.member_sums(seam, u, threads=threads)
        f.write(f"{u} {r['post0']:.17g} {r['post1']:.17g} {r['shared']:.17g} {r['shared_ll']:.17g} "
                f"{r['notshared_ll']:.17g} {r['n_patterns']}\n")
        f.flush()
        if u % 50 == 0:
            print(f"M={M} u={u} {time.time() - t0:.0f}s", flush=True)
