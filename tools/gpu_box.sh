#!/bin/bash
# Box-v0 GPU parity, then the parity / features suites (regressions of the shared kernel paths)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/box
timeout -k 10 600 python -u -m pytest tests/test_gpu_box.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/box/box.log 2>&1; rc=$?; echo "box rc=$rc"; tail -3 gpurun_out/box/box.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_features.py tests/test_gpu_geometry.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/box/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/box/parity.log; exit $rc
