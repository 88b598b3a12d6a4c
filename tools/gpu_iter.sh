#!/bin/bash
# one iteration on the GPU box: parity suite, phase profile (profiling build), chain timings, bench line
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_features.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?; echo "gputest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/phase_prof.py --steps 5 > gpurun_out/phase.txt 2>&1 || exit 1
timeout -k 10 200 python tools/chain_bench.py 0 4096 > gpurun_out/chain.txt 2>&1 || exit 1
cat gpurun_out/chain.txt
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/bench.json; exit $rc
