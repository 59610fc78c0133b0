#!/bin/bash
# r04an: pass-merge blocks of 4 / 16 waves (one SNP per wave; a block needs
# that many free slots on one CU, so the merge waits for the next sweep's
# drain) vs one-wave blocks (tree), worlds 1 and 8; async + multi + parity
# subset on the 16-wave build.
export TMPDIR=/tmp
OUT=gpurun_out/r04an
mkdir -p $OUT
PSX_AB=1 PSX_ENGINE_LIB=$PWD/_ab/mw16/libpipsort_engine.so timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_multi.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "async or multi or syn or headline or mixed" > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 - _ab/mw4 _ab/mw16 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; kernel ms per rank.*//'
