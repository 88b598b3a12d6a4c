#!/bin/bash
# camera GPU tests, then the whole GPU suite and the headline bench line (each step under its own limit)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpucam.log 2>&1; rc=$?; echo "camera rc=$rc"; tail -15 gpurun_out/gpucam.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpusuite.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -4 gpurun_out/gpusuite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/bench.json; exit $rc
