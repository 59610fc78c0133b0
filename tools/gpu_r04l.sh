#!/bin/bash
# r04l: GPU parity on the in-tree build (a records reduced with the next a's
# prologue batch), unit trace, same-box A/B vs round 3 (_ab/base) and r04j.
export TMPDIR=/tmp
OUT=gpurun_out/r04l
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py tests/test_gpu_multi.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread --deselect tests/test_gpu_parity.py::test_headline_full_vector > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/unit_trace.py --world 1 --rank 0 > $OUT/trace_w1.txt 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 _ab/base _ab/r04j - || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
