#!/bin/bash
# round-3 check: the new GPU tests first (config E at size, gloo ranks with the real sim, full episodes,
# failure branches, SB3 vs oracle, stream ordering), then the rest of the -m gpu suite, then the world-8 gloo
# rehearsal of config E on this one GPU
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3a
(cd tools/micro && timeout -k 5 60 ./bbidx) > gpurun_out/r3a/bbidx.txt 2>&1; echo "bbidx rc=$?"; tail -1 gpurun_out/r3a/bbidx.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_failures.py tests/test_vec_sb3.py tests/test_gpu_scale.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3a/new.log 2>&1; rc=$?; echo "new rc=$rc"; tail -3 gpurun_out/r3a/new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_features.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3a/old.log 2>&1; rc=$?; echo "old rc=$rc"; tail -3 gpurun_out/r3a/old.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --backend gloo --gpus 8 --task 3 --envs 8192 --steps 20 --warmup 3 --reps 3 > gpurun_out/r3a/world8_gloo_golf.json 2> gpurun_out/r3a/world8.err; rc=$?; echo "world8 rc=$rc"; cut -c1-400 gpurun_out/r3a/world8_gloo_golf.json; exit $rc
