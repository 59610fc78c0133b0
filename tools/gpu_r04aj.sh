#!/bin/bash
# r04aj: pass merge with eight records in flight per lane and its gather
# indices loaded a round ahead (k_merge_pass_l1) vs the previous commit
# (_ab/base), worlds 1 and 8, 3 reps; parity + multi + async files.
export TMPDIR=/tmp
OUT=gpurun_out/r04aj
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_async.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 _ab/base - || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; step ms per rank.*//'
