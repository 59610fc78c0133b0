#!/bin/bash
# Diagnostics of k_sweep3 builds: alternating shard-rehearsal A/B of the builds
# in $AB, unit traces (world 1) of each, and one SQ counter pass of each.
#   TAG=r03d AB="- _ab/w2k _ab/base" bash tools/gpu_diag.sh
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-diag}
mkdir -p "$OUT"
rm -f gpurun_out/ab/abn.txt
bash tools/abn.sh "${WORLDS:-1,8}" "${REPS:-2}" $AB || exit $?
cp gpurun_out/ab/abn.txt "$OUT/abn.txt"
G="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS"
for e in $AB; do
  n=$(echo "$e" | tr '/' '_'); L=""
  [ "$e" != "-" ] && L=$PWD/$e/libpipsort_engine.so
  timeout -k 10 120 env PSX_ENGINE_LIB=$L python -u tools/unit_trace.py --world 1 --rank 0 > "$OUT/trace_${n}_w1.txt" 2>&1 || exit $?
  PSX_ENGINE_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex 'k_sweep3' --output-format csv -d "$OUT/pmc_$n" -o run -- python3 tools/shard_rehearsal.py --worlds 1 --steps 3 > "$OUT/pmc_$n.log" 2>&1 || exit $?
done
exit 0
