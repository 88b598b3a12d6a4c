#!/bin/bash
# the whole -m gpu suite with the full geometry as the default, then benches of both geometries
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3e
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=15 > gpurun_out/r3e/gputest.log 2>&1; rc=$?; echo "gputest rc=$rc"; tail -22 gpurun_out/r3e/gputest.log; [ $rc -eq 0 ] || exit $rc
for g in full lod; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --geometry $g > gpurun_out/r3e/bench_bb_$g.json 2> gpurun_out/r3e/bench_bb_$g.err || exit 1
  cut -c1-150 gpurun_out/r3e/bench_bb_$g.json
  timeout -k 10 300 python bench.py --no-cpu-baseline --geometry $g --task 3 --envs 8192 --steps 10 --warmup 2 --reps 3 > gpurun_out/r3e/bench_golf_$g.json 2> gpurun_out/r3e/bench_golf_$g.err || exit 1
  cut -c1-150 gpurun_out/r3e/bench_golf_$g.json
done
