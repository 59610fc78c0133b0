#!/bin/bash
# r04w: a-chunk cap (PSX_K3_CAMAX) 4 (default) / 6 / 8 with the tail split,
# worlds 1, 2 (where the cap binds), 3 reps alternating; parity subset.
export TMPDIR=/tmp
OUT=gpurun_out/r04w
mkdir -p $OUT
PSX_K3_CAMAX=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "syn or headline or mixed or strong or extreme" > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2" 3 - -@PSX_K3_CAMAX=6 -@PSX_K3_CAMAX=8 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
