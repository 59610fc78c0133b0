#!/bin/bash
# r04al: records at their CSR positions (PSX_REC_CSR=1: each SNP's run
# contiguous, merge reads coalesced; sweep writes scattered) vs unit-major
# records gathered by the merge (default), with the 8-deep merge; worlds 1, 8.
export TMPDIR=/tmp
OUT=gpurun_out/r04al
mkdir -p $OUT
PSX_REC_CSR=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_async.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "syn or headline or mixed or strong or multi or async or extreme" > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 - -@PSX_REC_CSR=1 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; kernel ms per rank.*//'
