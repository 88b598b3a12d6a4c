#!/bin/bash
# round-3 iteration: parity suites (incl. geometry, Box), phase cycles of the default geometry, chain timings, bench
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${1:-r3i}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_features.py tests/test_gpu_geometry.py tests/test_gpu_box.py tests/test_gpu_failures.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1; rc=$?; echo "gputest rc=$rc"; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/phase_prof.py --steps 5 > $OUT/phase.txt 2>&1 || exit 1
timeout -k 10 200 python tools/chain_bench.py 0 4096 > $OUT/chain.txt 2>&1 || exit 1
cat $OUT/chain.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-200 $OUT/bench.json; exit $rc
