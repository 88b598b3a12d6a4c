#!/bin/bash
# Bench every non-headline task at its BASELINE.json config size (per GPU), with the CPU restatement beside it.
# usage (GPU box): bash tools/task_sweep.sh [outdir]
set -u
cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r6_tasks}
mkdir -p "$OUT"
for te in "1 4096" "2 8192" "3 8192" "4 4096" "5 8192" "6 4096" "7 4096"; do
  set -- $te
  timeout -k 10 240 python bench.py --task $1 --envs $2 --steps 50 --warmup 5 --reps 3 > "$OUT/task$1.json" 2> "$OUT/task$1.err" || { echo "TASK $1 FAILED"; exit 1; }
  echo "task $1 done"
done
