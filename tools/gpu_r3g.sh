#!/bin/bash
# round-3 re-entry check: the whole -m gpu suite, smoke(), bench lines of the default (full) and LOD geometry
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3g
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3g/gputest.log 2>&1; rc=$?; echo "gputest rc=$rc"; tail -2 gpurun_out/r3g/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3g/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r3g/bench_full.json 2> gpurun_out/r3g/bench_full.err; rc=$?; echo "bench full rc=$rc"; cut -c1-200 gpurun_out/r3g/bench_full.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --geometry lod > gpurun_out/r3g/bench_lod.json 2> gpurun_out/r3g/bench_lod.err; rc=$?; echo "bench lod rc=$rc"; cut -c1-200 gpurun_out/r3g/bench_lod.json; exit $rc
