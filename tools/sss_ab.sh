#!/bin/bash
# SSS walk timing A/B over PSX_SSS_THREADS values (alternating): bash tools/sss_ab.sh "1 4" reps
# (r03v; the knob and the exp thread pool it sized were removed after this A/B)
mkdir -p gpurun_out/sss_ab
for r in $(seq 1 ${2:-3}); do
  for n in $1; do
    echo "threads=$n rep=$r" >> gpurun_out/sss_ab/sss.txt
    PSX_SSS_THREADS=$n PSX_SSS_PROFILE=1 timeout -k 10 120 python tools/sss_time.py --M 200 --c 5 --reps 3 2>&1 | grep -E "psx sss|wall_s" | sed 's/"configs".*//' >> gpurun_out/sss_ab/sss.txt || exit 1
  done
done
