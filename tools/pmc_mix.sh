#!/bin/bash
# Instruction-mix / stall PMC passes of the bench (one rocprofv3 --pmc run per counter group, each under its
# own time limit).  usage (GPU box): bash tools/pmc_mix.sh <outdir> [bench args...]
set -u
OUT=${1:-gpurun_out/pmc_mix}; shift || true
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p "$OUT"
ARGS="${@:---steps 5 --warmup 2 --reps 1 --no-cpu-baseline}"
i=0
for G in "SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_FLAT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "PASS $i FAILED"; exit 1; }
done
echo PMC_MIX_OK
