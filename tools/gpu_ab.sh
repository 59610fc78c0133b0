#!/bin/bash
# One GPU-box session for a kernel change: the GPU test suite on the in-tree
# library, then an alternating A/B of the shard rehearsal against _ab/<old>.
#   TAG=r02b AB="- _ab/old" WORLDS=1,8 REPS=3 TESTS="tests" bash tools/gpu_ab.sh
# Stops at the first GPU fault / abort / time limit.
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "${WORLDS:-1,8}" "${REPS:-3}" ${AB:-- _ab/old} || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
exit $rc
