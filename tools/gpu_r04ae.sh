#!/bin/bash
# r04ae: shard balance at world 8 — per-a weight of pipelined diagonal walks
# (PSX_K3_DIAGW), masked ones (PSX_K3_MASKW) and the per-unit fixed cost
# (PSX_K3_UNITW); rank 0 (diagonal-heavy band) slowest, rank 7 (off-diagonal
# band) fastest so far.
export TMPDIR=/tmp
OUT=gpurun_out/r04ae
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "8" 3 - -@PSX_K3_MASKW=0.7 -@PSX_K3_DIAGW=0.65,PSX_K3_MASKW=0.7 -@PSX_K3_DIAGW=0.65,PSX_K3_MASKW=0.65 -@PSX_K3_UNITW=0.2,PSX_K3_MASKW=0.7 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
grep "world\|==" $OUT/abn.txt | sed 's/; step ms per rank.*//'
