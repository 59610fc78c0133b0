#!/bin/bash
# r04am: stream priorities swapped (PSX_PRIO_SWAP=1: sweeps on the highest-
# priority queue, merges / exchange lowest, so a pass's merge takes the slots
# the next sweep's drain frees) vs the default (merges first), worlds 1, 8;
# async + multi tests under the swap.
export TMPDIR=/tmp
OUT=gpurun_out/r04am
mkdir -p $OUT
PSX_PRIO_SWAP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_multi.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 - -@PSX_PRIO_SWAP=1 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; kernel ms per rank.*//'
