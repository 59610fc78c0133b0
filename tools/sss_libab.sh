#!/bin/bash
# SSS walk timing, alternating engine builds: bash tools/sss_libab.sh "- _ab/prev" reps
# ('-' = the in-tree library); kernel time from rocprofv3 stats of the last rep
mkdir -p gpurun_out/sss_libab
for r in $(seq 1 ${2:-2}); do
  for e in $1; do
    L=""; [ "$e" != "-" ] && L=$PWD/$e/libpipsort_engine.so
    echo "lib=$e rep=$r" >> gpurun_out/sss_libab/sss.txt
    PSX_ENGINE_LIB=$L PSX_SSS_PROFILE=1 timeout -k 10 120 python tools/sss_time.py --M 200 --c 5 --reps 3 2>&1 | grep -E "psx sss|wall_s" | sed 's/"configs".*//' >> gpurun_out/sss_libab/sss.txt || exit 1
  done
done
