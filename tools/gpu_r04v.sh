#!/bin/bash
# r04v: the overlap default decided once per handle: rehearsals in processes
# that start at their world (worlds 4 and 8 separately), default vs off;
# HIP start-up environment probe.
export TMPDIR=/tmp
OUT=gpurun_out/r04v
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "8" 3 - -@PSX_OVERLAP=0 || exit $?
bash tools/abn.sh "4" 3 - -@PSX_OVERLAP=0 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
timeout -k 10 200 python -u tools/init_env_probe.py > $OUT/init_env.txt 2>&1 || exit $?
