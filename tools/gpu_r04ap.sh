#!/bin/bash
# r04ap: pass-merge record loads non-temporal (PSX_MERGE_NT=1, _ab/nt: no L2
# allocation for the ~100 MB of records a pass streams beside the next sweep)
# vs the tree, worlds 1 and 8, 3 reps alternating; multi + async on _ab/nt.
export TMPDIR=/tmp
OUT=gpurun_out/r04ap
mkdir -p $OUT
PSX_AB=1 PSX_ENGINE_LIB=$PWD/_ab/nt/libpipsort_engine.so timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_multi.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 - _ab/nt || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; kernel ms per rank.*//'
