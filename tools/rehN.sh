#!/bin/bash
# alternate world-8 rehearsals of two libraries N times; step lines to gpurun_out/$1/reh.txt
OUT=gpurun_out/$1; N=$2; shift 2
mkdir -p $OUT
for i in $(seq 1 $N); do for d in "$@"; do
  echo "== $d rep $i" >> $OUT/reh.txt
  PSX_ENGINE_LIB=$PWD/$d/libpipsort_engine.so timeout -k 10 100 python -u tools/shard_rehearsal.py --worlds 8 --steps 20 2>&1 | grep "^world" | sed 's/; sweep ms.*//' >> $OUT/reh.txt || exit 1
done; done
