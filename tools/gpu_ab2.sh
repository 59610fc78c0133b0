#!/bin/bash
# GPU suite on the in-tree library, then alternating shard rehearsal A/B vs $AB
#   TAG=r03j AB="- _ab/head" TESTS="tests/test_gpu_parity.py" bash tools/gpu_ab2.sh
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "${WORLDS:-1,8}" "${REPS:-3}" $AB || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
