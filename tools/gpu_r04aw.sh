#!/bin/bash
# r04aw: SSS first walk on a handle (workspace allocation, 8-pair event ring):
# M = 200 and M = 2000 (configs[4]) -c 5, 3 walks each, host phases.
export TMPDIR=/tmp
OUT=gpurun_out/r04aw
mkdir -p $OUT
for M in 200 2000; do
  PSX_SSS_PROFILE=1 timeout -k 10 200 python -u tools/sss_time.py --M $M --c 5 --reps 3 > $OUT/sss_M$M.txt 2>&1 || exit $?
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sss_shard.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k sss > $OUT/pytest_sss.log 2>&1 || exit $?
tail -1 $OUT/pytest_sss.log
grep -h "psx sss\|wall_s" $OUT/sss_M*.txt | cut -c1-160
