#!/bin/bash
# Round profiling on the GPU box: bench (with CPU baseline), rocprofv3 kernel trace + stats,
# and separate PMC passes for HBM traffic (MI355X_MICROARCH.md: one counter group per pass).
# usage: bash tools/profile_round.sh <tag> [bench args...]
set -u
TAG=${1:-r1}; shift || true
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
# the libraries are built beforehand on the CPU side (__graft_entry__.build()) and travel with the tree
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline "$@" > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
echo TRACE_OK
# PMC passes on a short run of the same workload (traffic per launch does not depend on the step count)
PMCARGS="--steps 20 --warmup 3 --reps 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline "$@" $PMCARGS > $OUT/pmc_fetch.log 2>&1 || { echo PMC1_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --no-cpu-baseline "$@" $PMCARGS > $OUT/pmc_write.log 2>&1 || { echo PMC2_FAIL; exit 1; }
echo PMC_OK
python3 tools/pmc_traffic.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv $OUT/traffic_k_step.json "$@" > /dev/null && echo TRAFFIC_OK
timeout -k 10 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; exit 1; }
echo BENCH_OK

