#!/bin/bash
# Round record on one box: GPU suite, smoke(), bench line, rocprofv3 kernel
# stats of the bench, PMC passes of k_sweep3 (tools/gpu_pmc.sh).  Stops at the
# first failure.
#   TAG=r03n bash tools/gpu_final.sh
export TMPDIR=/tmp
TAG=${TAG:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline > $OUT/prof.log 2>&1 || exit $?
TAG=$TAG bash tools/gpu_pmc.sh || exit $?
