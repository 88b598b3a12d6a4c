#!/bin/bash
# quick GPU iteration: parity tests, reset-chain / step-chain timings, default bench line
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_features.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?; echo "gputest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/chain_bench.py 0 4096 > gpurun_out/chain.txt 2>&1 || exit 1
cat gpurun_out/chain.txt
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench.json; exit $rc
