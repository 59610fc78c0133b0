#!/bin/bash
# One GPU-box session: GPU test suite on the in-tree library, alternating
# shard-rehearsal A/B against other builds, the bench line and a rocprofv3
# kernel-trace summary of the bench.  Each GPU step has its own time limit and
# the script stops at the first failure (fault / abort / time limit).
#   TAG=r03c AB="- _ab/base" WORLDS=1,8 REPS=3 [NOTEST=1] [NOBENCH=1] bash tools/gpu_session.sh
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-s}
mkdir -p "$OUT"
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
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?
fi
exit 0
