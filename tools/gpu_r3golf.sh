#!/bin/bash
# Golf / Box iteration: the GPU suites that cover the cylinder pairs, Golf phase cycles, Golf and Box bench lines
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${1:-r3golf}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_features.py tests/test_gpu_geometry.py tests/test_gpu_box.py tests/test_gpu_failures.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1; rc=$?; echo "gputest rc=$rc"; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/phase_prof.py --steps 3 --task 3 --envs 2048 > $OUT/phase_golf.txt 2>&1 || exit 1
grep -E "cyl_pa|cyl_surv|hull_narrow|collide_cycles" $OUT/phase_golf.txt
for te in "3 8192" "7 4096" "0 4096"; do
  set -- $te
  timeout -k 10 300 python bench.py --task $1 --envs $2 --steps 20 --warmup 3 --reps 3 --no-cpu-baseline > "$OUT/task$1.json" 2> "$OUT/task$1.err" || { echo "TASK $1 FAILED"; exit 1; }
  echo "task $1: $(cut -c1-160 $OUT/task$1.json | sed 's/.*"value": \([0-9.]*\).*/\1/')"
done
