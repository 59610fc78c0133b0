#!/bin/bash
# r04m: GPU parity on the in-tree build (row_bcast wave reductions + a records
# in the next batch), unit trace; A/B: r04j, K (= r04j + row_bcast reductions),
# tree.
export TMPDIR=/tmp
OUT=gpurun_out/r04m
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py tests/test_gpu_multi.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread --deselect tests/test_gpu_parity.py::test_headline_full_vector > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/unit_trace.py --world 1 --rank 0 > $OUT/trace_w1.txt 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 _ab/r04j _ab/K - || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
