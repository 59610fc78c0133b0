#!/bin/bash
# r04ah: wave priority for the latency-bound a prologues (s_setprio 1 / 3 at the
# unit and a prologue, 0 for the walk; -DPSX_K3_PRIO builds in _ab/prioN) vs
# the tree (no priority changes), worlds 1 and 8, 3 reps alternating.
export TMPDIR=/tmp
OUT=gpurun_out/r04ah
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 - _ab/prio1 _ab/prio3 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
grep "world\|==" $OUT/abn.txt | sed 's/; kernel ms per rank.*//'
