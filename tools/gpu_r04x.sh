#!/bin/bash
# r04x: FP64 matrix pipe vs FP64 VALU on one SIMD (tools/mfma_overlap.hip);
# SSS workspace kept across walks + eval event ring: SSS parity tests and
# walk timing (M = 100 / 200, -c 5, 5 walks on one handle).
export TMPDIR=/tmp
OUT=gpurun_out/r04x
mkdir -p $OUT
timeout -k 10 60 ./tools/mfma_overlap.bin > $OUT/mfma_overlap.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sss_shard.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "sss" > $OUT/pytest_sss.log 2>&1 || exit $?
for M in 100 200; do
  PSX_SSS_PROFILE=1 timeout -k 10 120 python -u tools/sss_time.py --M $M --c 5 --reps 5 > $OUT/sss_M$M.txt 2>&1 || exit $?
done
tail -3 $OUT/pytest_sss.log
cat $OUT/mfma_overlap.txt
grep -h "psx sss\|wall_s" $OUT/sss_M*.txt | cut -c1-200
