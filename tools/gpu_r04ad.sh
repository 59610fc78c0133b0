#!/bin/bash
# r04ad: shard balance at world 8 — per-a weight of masked diagonal walks
# (PSX_K3_MASKW 0.59 default / 0.7 / 0.8 / 0.9); rank 0 (tile (0, 0) with
# padding, every walk masked) was the slowest rank in r04y / r04ab / r04ac.
export TMPDIR=/tmp
OUT=gpurun_out/r04ad
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "8" 3 - -@PSX_K3_MASKW=0.7 -@PSX_K3_MASKW=0.8 -@PSX_K3_MASKW=0.9 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
grep "world\|==" $OUT/abn.txt | sed 's/; step ms per rank.*//'
