#!/bin/bash
# A/B the shard rehearsal between the in-tree library and _ab/old (same box,
# alternating runs).  Usage (GPU box): bash tools/ab.sh [worlds] [reps]
W=${1:-1,8}
R=${2:-2}
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for v in new old; do
    if [ $v = old ]; then export PSX_ENGINE_LIB=$PWD/_ab/old/libpipsort_engine.so; else unset PSX_ENGINE_LIB; fi
    echo "== $v rep $i" >> gpurun_out/ab/ab.txt
    timeout -k 10 100 python -u tools/shard_rehearsal.py --worlds $W --steps 20 2>&1 | grep "^world" | sed 's/; sweep ms.*//' >> gpurun_out/ab/ab.txt || exit 1
  done
done
