#!/bin/bash
# r04ab: walk b-weights relative to the wave's largest R_s (slot {b} / {a, b}
# weights scaled once per a in LDS, lane factors folded into the lane vectors
# and the walk sums; SEP loop 195 -> 180 VALU, diagonal 231 -> 217, no scratch):
# full parity file + multi/async files, same-box A/B vs the previous commit
# (_ab/base) at worlds 1 and 8.
export TMPDIR=/tmp
OUT=gpurun_out/r04ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_async.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 _ab/base - || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; step ms.*//'
