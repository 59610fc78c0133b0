#!/bin/bash
# r04y: k_sweep3<true> without scratch (robust path's lane constants and the
# diagonal units' A_bb / y_b / A_cc / y_c parked in LDS): parity file, same-box
# A/B against the previous build (_ab/base) at worlds 1 and 8, unit traces at
# world 8 of both builds.
export TMPDIR=/tmp
OUT=gpurun_out/r04y
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 _ab/base - || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
timeout -k 10 120 env PSX_AB=1 PSX_ENGINE_LIB=$PWD/_ab/base/libpipsort_engine.so python -u tools/unit_trace.py --world 8 --rank 0 > $OUT/trace_w8_base.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/unit_trace.py --world 8 --rank 0 > $OUT/trace_w8_new.txt 2>&1 || exit $?
tail -2 $OUT/pytest_gpu.log
cat $OUT/abn.txt
