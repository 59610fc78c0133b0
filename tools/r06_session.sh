#!/bin/bash
# one GPU-box session of round 6: [GPU tests] + single-pass latency + kernel traces + [bench]
#   TAG=r06e [NOTEST=1] [TESTS=...] [SP=1] [TRACE=1] [BENCH=1] [POST="cmd"] bash tools/r06_session.sh
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-s}; mkdir -p $OUT
if [ -z "${NOTEST:-}" ]; then
    timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc" >> $OUT/pytest_gpu.log; tail -3 $OUT/pytest_gpu.log
    [ $rc -ne 0 ] && exit $rc
fi
if [ -n "${SP:-}" ]; then
    timeout -k 10 240 python tools/single_pass.py --passes 20 > $OUT/single.txt 2>&1 || { echo single rc=$?; tail $OUT/single.txt; exit 1; }
    grep -v '^{' $OUT/single.txt
fi
if [ -n "${TRACE:-}" ]; then
    for w in 1 8; do
        timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr$w -o run -- python3 tools/single_pass.py --passes 10 --rounds 1 --worlds $w > $OUT/tr$w.log 2>&1 || { echo trace rc=$?; exit 1; }
    done
fi
if [ -n "${BENCH:-}" ]; then
    timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench rc=$?; tail $OUT/bench.err; exit 1; }
fi
if [ -n "${POST:-}" ]; then
    timeout -k 10 ${POST_LIMIT:-300} $POST > $OUT/post.txt 2>&1 || { echo post rc=$?; tail -20 $OUT/post.txt; exit 1; }
    tail -${POST_TAIL:-20} $OUT/post.txt
fi
exit 0
