#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpucam.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpucam.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/camera_bench.py 5 > gpurun_out/cambench.json 2> gpurun_out/cambench.err; rc=$?; cat gpurun_out/cambench.json; exit $rc
