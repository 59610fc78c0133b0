#!/bin/bash
# r04ak: pass-merge depth (records in flight per lane, indices a round ahead):
# 8 (tree) / 6 / 4 (_ab/mdN) vs the four-deep gather without index prefetch
# (_ab/base), worlds 1 and 8, 3 reps alternating.
export TMPDIR=/tmp
OUT=gpurun_out/r04ak
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 _ab/base - _ab/md6 _ab/md4 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
grep "world\|==" $OUT/abn.txt | sed 's/; kernel ms per rank.*//'
