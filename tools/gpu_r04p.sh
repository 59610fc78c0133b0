#!/bin/bash
# r04p: tail split fraction (PSX_K3_TAIL) on the tree (+ slot scale folded into
# the SEP notSharedLL vector), worlds 1, 2, 4, 8; unit trace with the last-a
# prologue.
export TMPDIR=/tmp
OUT=gpurun_out/r04p
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread --deselect tests/test_gpu_parity.py::test_headline_full_vector > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2,4,8" 2 - -@PSX_K3_TAIL=0.03 -@PSX_K3_TAIL=0.05 -@PSX_K3_TAIL=0.08 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
timeout -k 10 120 env PSX_K3_TAIL=0.05 python -u tools/unit_trace.py --world 1 --rank 0 > $OUT/trace_w1_tail05.txt 2>&1 || exit $?
timeout -k 10 120 env PSX_K3_TAIL=0.05 python -u tools/unit_trace.py --world 8 --rank 0 > $OUT/trace_w8_tail05.txt 2>&1 || exit $?
