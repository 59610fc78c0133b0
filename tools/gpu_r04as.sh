#!/bin/bash
# r04as: unit traces of the current build (r04ag kernel) at worlds 1 and 8.
export TMPDIR=/tmp
OUT=gpurun_out/r04as
mkdir -p $OUT
timeout -k 10 120 python -u tools/unit_trace.py --world 8 --rank 0 > $OUT/trace_w8.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/unit_trace.py --world 1 --rank 0 > $OUT/trace_w1.txt 2>&1 || exit $?
head -16 $OUT/trace_w8.txt
