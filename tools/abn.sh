#!/bin/bash
# A/B/n the shard rehearsal across engine libraries / env settings on one box
# (alternating):  bash tools/abn.sh "worlds" reps entry1 entry2 ...
# entry = dir[@VAR=v,VAR2=w]; dir "-" = the in-tree library; each dir holds a
# libpipsort_engine.so.  Results in gpurun_out/ab/abn.txt
W=$1; R=$2; shift 2
export PSX_AB=1  # variants may predate a symbol
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for e in "$@"; do
    d=${e%%@*}; envs=""
    [ "$d" != "$e" ] && envs=${e#*@}
    if [ "$d" = "-" ]; then lib=""; else lib=$PWD/$d/libpipsort_engine.so; fi
    echo "== $e rep $i" >> gpurun_out/ab/abn.txt
    env PSX_ENGINE_LIB=$lib ${envs//,/ } timeout -k 10 300 python -u tools/shard_rehearsal.py --worlds $W --steps 20 2>&1 | grep "^world" >> gpurun_out/ab/abn.txt || exit 1
  done
done
