#!/bin/bash
# r04av: shard balance at world 8 — diagonal weights 0.62 / 0.68 vs 0.65
# (default), 3 reps alternating.
export TMPDIR=/tmp
OUT=gpurun_out/r04av
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "8" 3 - -@PSX_K3_DIAGW=0.62,PSX_K3_MASKW=0.62 -@PSX_K3_DIAGW=0.68,PSX_K3_MASKW=0.68 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
grep "world\|==" $OUT/abn.txt | sed 's/; step ms per rank.*//'
