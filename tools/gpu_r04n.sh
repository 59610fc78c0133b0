#!/bin/bash
# r04n: tail split of the k = 3 plan (PSX_K3_TAIL: share of a shard's work cut
# into single-a units at the end), same box, alternating; worlds 1, 2, 4, 8.
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2,4,8" 2 - -@PSX_K3_TAIL=0.05 -@PSX_K3_TAIL=0.1 -@PSX_K3_TAIL=0.2 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
timeout -k 10 120 env PSX_K3_TAIL=0.1 python -u tools/unit_trace.py --world 1 --rank 0 > $OUT/trace_w1_tail10.txt 2>&1 || exit $?
