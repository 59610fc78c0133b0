#!/bin/bash
# A/B the shard rehearsal between env settings on the same box:
#   bash tools/ab_env.sh "worlds" "ENV_A=.." "ENV_B=.." ...   (use "-" for no env)
W=$1; shift
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for e in "$@"; do
    echo "== [$e] rep $rep" >> gpurun_out/ab/abenv.txt
    if [ "$e" = "-" ]; then
      timeout -k 10 100 python -u tools/shard_rehearsal.py --worlds $W --steps 20 2>&1 | grep "^world" | sed 's/; sweep ms.*//' >> gpurun_out/ab/abenv.txt || exit 1
    else
      env $e timeout -k 10 100 python -u tools/shard_rehearsal.py --worlds $W --steps 20 2>&1 | grep "^world" | sed 's/; sweep ms.*//' >> gpurun_out/ab/abenv.txt || exit 1
    fi
  done
done
