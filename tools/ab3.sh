#!/bin/bash
# three-way: old lib, new lib with XCD binning auto, new lib with binning off
mkdir -p gpurun_out/ab
for i in 1 2; do
  echo "== new(auto) $i" >> gpurun_out/ab/ab3.txt
  timeout -k 10 100 python -u tools/shard_rehearsal.py --worlds ${1:-1,2,8} --steps 20 2>&1 | grep "^world" | sed 's/; sweep ms.*//' >> gpurun_out/ab/ab3.txt || exit 1
  echo "== new(nobin) $i" >> gpurun_out/ab/ab3.txt
  PSX_XCD_BIN=0 timeout -k 10 100 python -u tools/shard_rehearsal.py --worlds ${1:-1,2,8} --steps 20 2>&1 | grep "^world" | sed 's/; sweep ms.*//' >> gpurun_out/ab/ab3.txt || exit 1
  echo "== new(bin) $i" >> gpurun_out/ab/ab3.txt
  PSX_XCD_BIN=1 timeout -k 10 100 python -u tools/shard_rehearsal.py --worlds ${1:-1,2,8} --steps 20 2>&1 | grep "^world" | sed 's/; sweep ms.*//' >> gpurun_out/ab/ab3.txt || exit 1
  echo "== old $i" >> gpurun_out/ab/ab3.txt
  PSX_ENGINE_LIB=$PWD/_ab/old/libpipsort_engine.so timeout -k 10 100 python -u tools/shard_rehearsal.py --worlds ${1:-1,2,8} --steps 20 2>&1 | grep "^world" | sed 's/; sweep ms.*//' >> gpurun_out/ab/ab3.txt || exit 1
done
