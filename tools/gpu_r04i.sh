#!/bin/bash
# r04i: GPU suite on the in-tree build (closed-form notSharedLL slot terms, lazy
# k = 3 layouts, psx_warmup_for, multi-shard fixes), unit traces, same-box A/B
# against the round-3 kernel (_ab/base), process-exit probe.
export TMPDIR=/tmp
OUT=gpurun_out/r04i
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/unit_trace.py --world 1 --rank 0 > $OUT/trace_w1.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/unit_trace.py --world 8 --rank 0 > $OUT/trace_w8.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/exit_probe.py > $OUT/exit_probe.txt 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 _ab/base - || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
