#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel-trace summary,
# PMC counter passes.  Stops at the first GPU fault / abort / timeout.
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r01}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline > $OUT/prof.log 2>&1 || exit $?
if [ -n "${PMC:-}" ]; then TAG=${TAG:-r01} bash tools/gpu_pmc.sh || exit $?; fi
exit 0
