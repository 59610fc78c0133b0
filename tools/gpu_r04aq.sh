#!/bin/bash
# r04aq: the fast walk's per-step n_abc - n_ac maximum dropped — a unit whose
# sums overflow (non-finite accumulators) goes to the robust variant instead
# (SEP 180 -> 178 VALU per step pair, diagonal 217 -> 214): parity + multi +
# async files, same-box A/B vs the previous commit at worlds 1 and 8.
export TMPDIR=/tmp
OUT=gpurun_out/r04aq
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_async.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 _ab/base - || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; kernel ms per rank.*//'
