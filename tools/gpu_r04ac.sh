#!/bin/bash
# r04ac: transposed wave reductions (v_permlane32/16_swap, psx_wave.h) for the
# a prologue / a record / unit record batches: semantics probe, parity +
# multi + async files, same-box A/B vs the previous commit at worlds 1 and 8.
export TMPDIR=/tmp
OUT=gpurun_out/r04ac
mkdir -p $OUT
timeout -k 10 60 ./tools/wave_red_probe.bin > $OUT/wave_red_probe.txt 2>&1 || { cat $OUT/wave_red_probe.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_async.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 _ab/base - || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
cat $OUT/wave_red_probe.txt
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; step ms.*//'
