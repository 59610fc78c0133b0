#!/bin/bash
# r04j: GPU suite on the in-tree build (batched wave reductions, one-wave LDS
# ordering instead of __syncthreads in the fast k = 3 variant), unit traces,
# same-box A/B: round-3 kernel (_ab/base), batched reductions only (_ab/C1), tree.
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread --deselect tests/test_gpu_parity.py::test_headline_full_vector > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/unit_trace.py --world 1 --rank 0 > $OUT/trace_w1.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/unit_trace.py --world 8 --rank 0 > $OUT/trace_w8.txt 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 _ab/base _ab/C1 - || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
