#!/bin/bash
# r04au: final-tree record — GPU suite, smoke, bench, rocprof stats, PMC passes
# (tools/gpu_final.sh), then the shard rehearsal at worlds 1, 2, 4, 8 (3 reps).
export TMPDIR=/tmp
TAG=r04au bash tools/gpu_final.sh || exit $?
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,2,4,8" 3 - || exit $?
cp gpurun_out/ab/abn.txt gpurun_out/r04au/rehearsal.txt
tail -2 gpurun_out/r04au/pytest_gpu.log
grep "world\|==" gpurun_out/r04au/rehearsal.txt | sed 's/; kernel ms per rank.*//'
