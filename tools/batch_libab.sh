#!/bin/bash
# SSS proposal-batch timing (bench.sss_probe), alternating engine builds:
#   bash tools/batch_libab.sh "- _ab/x _ab/y" ROUNDS    ('-' = the in-tree library)
mkdir -p gpurun_out/batch_libab
out=gpurun_out/batch_libab/ab.txt
rm -f $out
for r in $(seq 1 ${2:-3}); do
  for e in $1; do
    L=""; [ "$e" != "-" ] && L=$PWD/$e/libpipsort_engine.so
    PSX_AB=1 PSX_ENGINE_LIB=$L timeout -k 10 120 python tools/sss_probe.py 30 > gpurun_out/batch_libab/p.json 2>/dev/null || exit 1
    python -c "
import json,sys; d=json.load(open('gpurun_out/batch_libab/p.json'))
print('lib=$e round=$r batch_ms=%.4f kernel_ms=%.4f walk200_ms=%.3f' % (d['batch_ms'], d['roofline']['kernel_ms'], d['long_walks'][1]['walk_ms']))" >> $out || exit 1
  done
done
cat $out
