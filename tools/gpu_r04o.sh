#!/bin/bash
# r04o: what binds the k = 3 walk: E1 = +8 independent FMAs per step (issue),
# E2 = +4 dependent FMAs per study on the chain's critical path (latency);
# same box, alternating, against the tree.  Results of E1 / E2 are not used.
export TMPDIR=/tmp
OUT=gpurun_out/r04o
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 - _ab/E1 _ab/E2 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
