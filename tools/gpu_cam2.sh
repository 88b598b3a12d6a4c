#!/bin/bash
# camera tests + camera throughput + the Robotiq-140 bench lines (each step under its own limit)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py tests/test_gpu_r140.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpucam.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpucam.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/camera_bench.py 5 > gpurun_out/cambench.json 2> gpurun_out/cambench.err; rc=$?; cat gpurun_out/cambench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --robot ur5_robotiq_140 --cpu-seconds 5 > gpurun_out/r140_bench0.json 2> gpurun_out/r140_b0.err || exit 1
timeout -k 10 300 python bench.py --robot ur5_robotiq_140 --task 2 --envs 8192 --steps 50 --warmup 5 --reps 3 --cpu-seconds 5 > gpurun_out/r140_bench2.json 2> gpurun_out/r140_b2.err; rc=$?
cut -c1-200 gpurun_out/r140_bench0.json gpurun_out/r140_bench2.json; exit $rc
