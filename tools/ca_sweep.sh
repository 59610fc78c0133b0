#!/bin/bash
# a-chunk sweep of the shard rehearsal (GPU box): bash tools/ca_sweep.sh "1 2 3 4" 1,2,4,8
mkdir -p gpurun_out/ca
for ca in $1; do
  echo "== ca $ca" >> gpurun_out/ca/ca.txt
  PSX_K3_CA=$ca timeout -k 10 100 python -u tools/shard_rehearsal.py --worlds $2 --steps 20 2>&1 | grep "^world" | sed 's/; sweep ms.*//' >> gpurun_out/ca/ca.txt || exit 1
done
