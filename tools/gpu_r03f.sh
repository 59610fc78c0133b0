#!/bin/bash
# r03f: GPU suite on the in-tree build, SSS / configs timelines, bench + rocprof
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03f}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/cfg -o run -- python3 tools/configs_time.py > $OUT/cfg.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sss -o run -- python3 tools/sss_time.py --M 200 --c 5 --reps 2 > $OUT/sss.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline > $OUT/prof.log 2>&1 || exit $?
