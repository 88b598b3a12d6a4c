#!/bin/bash
# full-geometry parity after the chunk cull, phase cycles of both modes (BallBalance), benches of both modes
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3d
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullgeom.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3d/full.log 2>&1; rc=$?; echo "full rc=$rc"; tail -2 gpurun_out/r3d/full.log; [ $rc -eq 0 ] || exit $rc
for g in lod full; do
  timeout -k 10 200 python tools/phase_prof.py --steps 5 --geometry $g > gpurun_out/r3d/phase_bb_$g.txt 2>&1 || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --geometry $g > gpurun_out/r3d/bench_bb_$g.json 2> gpurun_out/r3d/bench_bb_$g.err || exit 1
  cut -c1-150 gpurun_out/r3d/bench_bb_$g.json
done
timeout -k 10 300 python tools/phase_prof.py --steps 3 --task 3 --envs 2048 --geometry full > gpurun_out/r3d/phase_golf_full.txt 2>&1 || exit 1
for t in 1 2 3; do
  e=4096; [ $t -ge 2 ] && e=8192
  timeout -k 10 300 python bench.py --no-cpu-baseline --geometry full --task $t --envs $e --steps 10 --warmup 2 --reps 3 > gpurun_out/r3d/bench_t${t}_full.json 2> gpurun_out/r3d/bench_t${t}_full.err || exit 1
  cut -c1-150 gpurun_out/r3d/bench_t${t}_full.json
done
timeout -k 10 300 python tools/phase_prof.py --steps 3 --task 3 --envs 2048 --geometry lod > gpurun_out/r3d/phase_golf_lod.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "golf or Golf or 3 or sharded" > gpurun_out/r3d/golf_parity.log 2>&1; rc=$?; echo "golf parity rc=$rc"; tail -1 gpurun_out/r3d/golf_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --task 3 --envs 8192 --steps 10 --warmup 2 --reps 3 > gpurun_out/r3d/bench_t3_lod.json 2> gpurun_out/r3d/bench_t3_lod.err || exit 1
cut -c1-150 gpurun_out/r3d/bench_t3_lod.json
