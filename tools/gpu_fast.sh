#!/bin/bash
# certified-chunk fast path: phase profile before / after (profiling builds), parity suites, bench line
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
URGYM_LIB=$PWD/urgym_amd/_lib/var/prof_base.so timeout -k 10 200 python tools/phase_prof.py --steps 5 > gpurun_out/phase_base.txt 2>&1 || { echo PROF0 FAIL; tail -3 gpurun_out/phase_base.txt; exit 1; }
timeout -k 10 200 python tools/phase_prof.py --steps 5 > gpurun_out/phase_fast.txt 2>&1 || { echo PROF1 FAIL; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_features.py tests/test_gpu_failures.py tests/test_gpu_box.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/chain_bench.py 0 4096 > gpurun_out/chain.txt 2>&1 || exit 1
cat gpurun_out/chain.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cut -c1-200 gpurun_out/bench.json; exit $rc
