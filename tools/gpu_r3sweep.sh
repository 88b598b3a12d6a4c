#!/bin/bash
# round-3 sweep: Golf phase cycles (default geometry), then every task at its BASELINE size incl. Box-v0, with the CPU
# restatement beside each
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r3sweep; mkdir -p $OUT
timeout -k 10 300 python tools/phase_prof.py --steps 3 --task 3 --envs 2048 > $OUT/phase_golf.txt 2>&1 || exit 1
echo phase_ok
for te in "1 4096" "2 8192" "3 8192" "4 4096" "5 8192" "6 4096" "7 4096"; do
  set -- $te
  timeout -k 10 300 python bench.py --task $1 --envs $2 --steps 20 --warmup 3 --reps 3 --cpu-seconds 5 > "$OUT/task$1.json" 2> "$OUT/task$1.err" || { echo "TASK $1 FAILED"; exit 1; }
  echo "task $1 done: $(cut -c1-160 $OUT/task$1.json | sed 's/.*"value": \([0-9.]*\).*/\1/')"
done
