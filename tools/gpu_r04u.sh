#!/bin/bash
# r04u: multi-rank / async GPU tests with overlap on by default at worlds >= 4;
# rehearsal: default vs overlap off vs half-walk tail pieces (PSX_K3_TAIL2).
export TMPDIR=/tmp
OUT=gpurun_out/r04u
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_multi.py tests/test_gpu_dist.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2,4,8" 3 - -@PSX_OVERLAP=0 -@PSX_K3_TAIL2=0.02 -@PSX_K3_TAIL2=0.02,PSX_K3_TAIL=0.08 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
