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


i=0
while read -r GROUP; do
    [ -z "$GROUP" ] && continue
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $GROUP --kernel-include-regex 'k_sweep|k_merge|k_eval_batch' --output-format csv \
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
SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
EOF
exit 0
