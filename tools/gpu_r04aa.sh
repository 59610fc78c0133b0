#!/bin/bash
# r04aa: per-a cost of masked diagonal walks in the unit work model
# (PSX_K3_MASKW: 1.0 tried as default; 0.59 = the old model, kept; 1.3), worlds 1, 2, 8,
# 3 reps alternating (per-rank kernel spread at world 8 was 0.125-0.139 ms);
# parity subset with the default.
export TMPDIR=/tmp
OUT=gpurun_out/r04aa
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "syn or headline or mixed or strong or multi" > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2,8" 3 - -@PSX_K3_MASKW=0.59 -@PSX_K3_MASKW=1.3 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
tail -2 $OUT/pytest_gpu.log
grep "world 8\|==" $OUT/abn.txt | sed 's/; step ms.*//'
grep "world 1\|world 2" $OUT/abn.txt | sed 's/; kernel ms.*//'
