#!/bin/bash
# r04at: fused merges (PSX_FUSE_MERGE=1: an asynchronous pass's merge rides in
# the next pass's sweep launch — scalar fold as the first block, per-SNP folds
# as the last blocks, in the sweep's drain).  Full GPU suite with it on, then
# same-box A/B vs off at worlds 1 and 8, and the bench line with it on.
export TMPDIR=/tmp
OUT=gpurun_out/r04at
mkdir -p $OUT
PSX_FUSE_MERGE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 - -@PSX_FUSE_MERGE=1 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
PSX_FUSE_MERGE=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_fused.json 2> $OUT/bench_fused.err || exit $?
tail -2 $OUT/pytest_gpu.log
grep "world\|==" $OUT/abn.txt | sed 's/; step ms per rank.*//'
python -c "import json;d=json.loads(open('$OUT/bench_fused.json').read().strip().split(chr(10))[-1]);print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
