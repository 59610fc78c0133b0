#!/bin/bash
# r04s: dispatch rounds the k = 3 a-chunk is sized for (PSX_K3_ROUNDS; the
# default 2.0) with the tail split (now default 0.05): worlds 1 (unaffected:
# a-chunk capped at 4), 2, 4, 8; and overlap at 4 / 8; tree = first-a loads
# issued with the unit prologue (off-diagonal units).
export TMPDIR=/tmp
OUT=gpurun_out/r04s
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread --deselect tests/test_gpu_parity.py::test_headline_full_vector > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2,4,8" 3 - -@PSX_K3_ROUNDS=1.0 -@PSX_K3_ROUNDS=1.4 -@PSX_OVERLAP=8,PSX_K3_ROUNDS=1.0 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
