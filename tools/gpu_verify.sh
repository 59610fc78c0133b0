#!/bin/bash
# Full GPU suite, smoke() and the bench line on the tree (no PMC passes: for a
# tree whose k_sweep3 sources match profiles/pmc_latest.json).
#   TAG=r04ao bash tools/gpu_verify.sh
export TMPDIR=/tmp
TAG=${TAG:-verify}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -2 $OUT/pytest_gpu.log
tail -1 $OUT/smoke.log
