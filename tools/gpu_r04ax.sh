#!/bin/bash
# r04ax: k_sweep3 built with other LLVM scheduler strategies (max-ilp, the
# AMDGPU register-pressure trackers, max-memory-clause) vs the default, world 1
# (3 reps) and world 8 (3 reps), alternating.
export TMPDIR=/tmp
OUT=gpurun_out/r04ax
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 - _ab/maxilp _ab/trackers _ab/maxmem || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
grep "world\|==" $OUT/abn.txt | sed 's/; kernel ms per rank.*//'
