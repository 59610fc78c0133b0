#!/bin/bash
# r04af: diagonal walk weight 0.65 (pipelined and masked) as the default plan
# vs the previous 0.59 / 0.59, worlds 1, 2, 4, 8, 3 reps alternating; parity
# subset + multi (the plan cuts different units).
export TMPDIR=/tmp
OUT=gpurun_out/r04af
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "syn or headline or mixed or strong or multi or extreme" > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2,4,8" 3 - -@PSX_K3_DIAGW=0.59,PSX_K3_MASKW=0.59 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; kernel ms per rank.*//'
