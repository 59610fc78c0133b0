#!/bin/bash
# r04ar: r04aq's change (overflow-based redo check) vs the previous commit,
# world 1 only, 6 reps alternating.
export TMPDIR=/tmp
OUT=gpurun_out/r04ar
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1" 6 _ab/base - || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
grep "world\|==" $OUT/abn.txt | sed 's/; step ms per rank.*//'
