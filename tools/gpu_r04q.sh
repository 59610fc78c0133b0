#!/bin/bash
# r04q: CU-mask mapping probe; overlapped sweeps (PSX_OVERLAP = reserved CUs)
# against the default, worlds 1, 2, 4, 8, same box alternating; async tests.
export TMPDIR=/tmp
OUT=gpurun_out/r04q
mkdir -p $OUT
timeout -k 10 60 ./tools/cumask_probe.bin > $OUT/cumask_probe.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2,4,8" 2 - -@PSX_OVERLAP=8 -@PSX_OVERLAP=8,PSX_RESERVE_STRIDE=32 -@PSX_OVERLAP=16,PSX_RESERVE_STRIDE=16 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
