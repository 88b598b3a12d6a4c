#!/bin/bash
# full-geometry mode: GPU parity on every task, then the bench beside the default (BallBalance x 4096, other tasks)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullgeom.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3b/full.log 2>&1; rc=$?; echo "full rc=$rc"; tail -3 gpurun_out/r3b/full.log; [ $rc -eq 0 ] || exit $rc
for g in lod full; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --geometry $g --steps 50 --warmup 5 --reps 3 > gpurun_out/r3b/bench_bb_$g.json 2> gpurun_out/r3b/bench_bb_$g.err || exit 1
  cut -c1-160 gpurun_out/r3b/bench_bb_$g.json
done
for t in 1 2 3; do
  e=4096; [ $t -ge 2 ] && e=8192
  timeout -k 10 300 python bench.py --no-cpu-baseline --geometry full --task $t --envs $e --steps 10 --warmup 2 --reps 3 > gpurun_out/r3b/bench_t${t}_full.json 2> gpurun_out/r3b/bench_t${t}_full.err || exit 1
  cut -c1-160 gpurun_out/r3b/bench_t${t}_full.json
done
