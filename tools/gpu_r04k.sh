#!/bin/bash
# r04k: k = 3 plan granularity on the current kernel (env knobs, same box,
# alternating): default (2.0 rounds), diagonal a-chunk halved, 3.5 rounds,
# 3.5 rounds + halved diagonal chunk; worlds 1, 2, 4, 8.  Then one bench line
# (no CPU baseline) for the tests/example wall split.
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2,4,8" 2 - -@PSX_K3_DIAG_DIV=2 -@PSX_K3_ROUNDS=3.5 -@PSX_K3_ROUNDS=3.5,PSX_K3_DIAG_DIV=2 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
