#!/bin/bash
# end-of-session GPU check: the whole -m gpu suite, smoke(), phase cycles and chain timings (profiling build),
# and the default bench line with its CPU baseline
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/gputest.log 2>&1; rc=$?; echo "gputest rc=$rc"; tail -2 gpurun_out/final/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/phase_prof.py --steps 5 > gpurun_out/final/phase.txt 2>&1 || exit 1
timeout -k 10 200 python tools/chain_bench.py 0 4096 > gpurun_out/final/chain.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-250 gpurun_out/final/bench.json; exit $rc
