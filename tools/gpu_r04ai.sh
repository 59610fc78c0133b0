#!/bin/bash
# r04ai: what the pass merge (k_merge_pass_l1, beside the next sweep) costs:
# timing ablation PSX_ABLATE_MERGE=1 (merge skipped, results wrong) vs the
# tree, worlds 1 and 8, 3 reps alternating.
export TMPDIR=/tmp
OUT=gpurun_out/r04ai
mkdir -p $OUT
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "1,8" 3 - -@PSX_ABLATE_MERGE=1 || exit $?
cp gpurun_out/ab/abn.txt $OUT/abn.txt
grep "world\|==" $OUT/abn.txt | sed 's/; step ms per rank.*//'
