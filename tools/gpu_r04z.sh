#!/bin/bash
# r04z: half-walk tail pieces (PSX_K3_TAIL2) without overlapped passes (r04u
# measured them with overlap on), worlds 1 and 8, 3 reps alternating; parity
# subset with the largest setting.
export TMPDIR=/tmp
OUT=gpurun_out/r04z
mkdir -p $OUT
PSX_K3_TAIL2=0.03 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "syn or headline or mixed or strong" > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 - -@PSX_K3_TAIL2=0.01 -@PSX_K3_TAIL2=0.02 -@PSX_K3_TAIL2=0.03 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
timeout -k 10 120 env PSX_K3_TAIL2=0.02 python -u tools/unit_trace.py --world 8 --rank 0 > $OUT/trace_w8_tail2_02.txt 2>&1 || exit $?
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; kernel ms.*//'
