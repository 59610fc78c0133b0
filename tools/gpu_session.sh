#!/bin/bash
# One GPU-box session: GPU test suite on the in-tree library, alternating
# shard-rehearsal A/B against other builds, the bench line and a rocprofv3
# kernel-trace summary of the bench.  Each GPU step has its own time limit and
# the script stops at the first failure (fault / abort / time limit).
#   TAG=r03c AB="- _ab/base" WORLDS=1,8 REPS=3 [NOTEST=1] [NOBENCH=1] [TESTS="tests/x.py ..."] \
#       [PRE="python tools/setup_time.py"] [POST="python tools/shard_rehearsal.py ..."] [PROF=1] [PMC=1] \
#       bash tools/gpu_session.sh
# PRE runs before the tests, POST after the bench (each under its own time
# limit, output in $OUT/pre.txt / post.txt); PROF=1 adds the rocprofv3
# kernel-trace summary of the bench, PMC=1 the counter passes (tools/gpu_pmc.sh).
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-s}
mkdir -p "$OUT"
if [ -n "${PRE:-}" ]; then
    timeout -k 10 ${PRE_LIMIT:-300} $PRE > "$OUT/pre.txt" 2>&1 || { echo "PRE failed rc=$?"; tail -20 "$OUT/pre.txt"; exit 1; }
fi
if [ -z "${NOTEST:-}" ]; then
    timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
    rc=$?
    echo "pytest rc=$rc" >> "$OUT/pytest_gpu.log"
    [ $rc -ne 0 ] && exit $rc
fi
if [ -n "${AB:-}" ]; then
    rm -f gpurun_out/ab/abn.txt
    bash tools/abn.sh "${WORLDS:-1,8}" "${REPS:-3}" $AB || exit $?
    cp gpurun_out/ab/abn.txt "$OUT/abn.txt"
fi
if [ -z "${NOBENCH:-}" ]; then
    timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
fi
if [ -n "${PROF:-}" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?
fi
if [ -n "${PMC:-}" ]; then TAG=${TAG:-s} bash tools/gpu_pmc.sh || exit $?; fi
if [ -n "${POST:-}" ]; then
    timeout -k 10 ${POST_LIMIT:-300} $POST > "$OUT/post.txt" 2>&1 || { echo "POST failed rc=$?"; tail -20 "$OUT/post.txt"; exit 1; }
fi
[ -f "$OUT/pytest_gpu.log" ] && tail -3 "$OUT/pytest_gpu.log"
[ -f "$OUT/pre.txt" ] && tail -5 "$OUT/pre.txt"
[ -f "$OUT/post.txt" ] && tail -5 "$OUT/post.txt"
exit 0
