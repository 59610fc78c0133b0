#!/bin/bash
# PMC counter passes for the sweep kernel (run on the GPU box via gpurun).
#   TAG=r01g WL=syn1000c3 bash tools/gpu_pmc.sh
# One counter group per rocprofv3 pass (SQ: 8 slots; FETCH_SIZE and WRITE_SIZE
# each need their own pass).  No trace domains are combined with --pmc.
# Stops at the first GPU fault / abort / time limit (exit 124/134/137/139).
set -u
TAG=${TAG:-pmc}
WL=${WL:-syn1000c3}
OUT=gpurun_out/$TAG/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --workload $WL"

timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1
echo "list rc=$?" >> "$OUT/status.txt"

i=0
while read -r GROUP; do
    [ -z "$GROUP" ] && continue
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $GROUP --kernel-include-regex 'k_sweep' --output-format csv \
        -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "pass $i [$GROUP] rc=$rc" >> "$OUT/status.txt"
    case $rc in
        124|134|137|139) echo "stopping after rc=$rc" >> "$OUT/status.txt"; exit $rc ;;
    esac
done <<'EOF'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES
TCC_HIT_sum TCC_MISS_sum
EOF
exit 0
