#!/bin/bash
# r04r: CU-mask semantics probe; tail split 0.05 and overlap (8 CUs) alone and
# together, worlds 1, 2, 4, 8, 3 reps alternating.
export TMPDIR=/tmp
OUT=gpurun_out/r04r
mkdir -p $OUT
timeout -k 10 60 ./tools/cumask_probe2.bin > $OUT/cumask_probe2.txt 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2,4,8" 3 - -@PSX_K3_TAIL=0.05 -@PSX_OVERLAP=8 -@PSX_OVERLAP=8,PSX_K3_TAIL=0.05 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
