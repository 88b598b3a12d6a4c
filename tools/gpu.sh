#!/bin/bash
# One launcher for every GPU-box job (run through gpurun; each step under its own time limit, the first failure ends
# the call).  Libraries are built beforehand on the CPU side (__graft_entry__.build(), tools/build_prof.sh) and travel
# with the tree.  Output goes under gpurun_out/<tag>/.
#
#   bash tools/gpu.sh tests <tag> [pytest targets...]   GPU tests (default: the whole -m gpu suite)
#   bash tools/gpu.sh smoke <tag>                       __graft_entry__.smoke()
#   bash tools/gpu.sh bench <tag> [bench.py args...]    one bench line -> <tag>/bench.json
#   bash tools/gpu.sh sweep <tag> [bench.py args...]    every task at its BASELINE size -> <tag>/task<N>.json
#   bash tools/gpu.sh phase <tag> [phase_prof args...]  phase cycles of the profiling build -> <tag>/phase.txt
#   bash tools/gpu.sh chain <tag> [task envs]           reset-chain / step-chain timings -> <tag>/chain.txt
#   bash tools/gpu.sh contend <tag> [bench.py args...]  co-runner contention: PMC at default slots vs one wave per CU
#   bash tools/gpu.sh timeline <tag> [timeline args]    k_step block timeline + schedule predictions -> <tag>/timeline.txt, .json
#   bash tools/gpu.sh profile <tag> [bench.py args...]  rocprofv3 kernel trace + stats, FETCH_SIZE / WRITE_SIZE PMC
#                                                       passes (one counter group per run), traffic json, bench line
#   bash tools/gpu.sh pmcmix <tag> [bench.py args...]   instruction-mix / stall PMC passes
#   bash tools/gpu.sh world8 <tag> [bench.py args...]   the 8-rank path rehearsed on this one GPU: 8 gloo ranks
#                                                       (torch.distributed.run, 127.0.0.1) -> <tag>/world8.json
#   bash tools/gpu.sh icache <tag> [bench.py args...]   instruction-cache PMC pass (SQC_ICACHE_*, SQ_IFETCH) after
#                                                       listing the box's counters -> <tag>/counters.txt, <tag>/ic/
#   bash tools/gpu.sh final <tag>                       round-end check: whole suite, smoke, headline bench
# Several jobs in one call: gpurun -- 'bash tools/gpu.sh tests t1 tests/test_gpu_gjk.py && bash tools/gpu.sh bench t1'
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
JOB=${1:?job}; TAG=${2:-run}; shift 2 || shift $#
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() { # step <seconds> <log> <cmd...>: run under a limit, show the tail, stop on failure
    local lim=$1 log=$2; shift 2
    timeout -k 10 "$lim" "$@" > "$log" 2>&1; local rc=$?
    echo "[$JOB] $(basename "$log") rc=$rc"; tail -4 "$log"
    return $rc
}
case "$JOB" in
tests)
    if [ $# -eq 0 ]; then set -- tests -m gpu; fi
    # page the image in first (a fresh box's first `import torch` can take minutes), printing as it goes
    step 300 "$OUT/warm.log" python -u -c "print('importing torch', flush=True); import torch; print('cuda', torch.cuda.is_available(), flush=True)" &&
    step 1500 "$OUT/tests.log" python -u -m pytest -x -v --timeout 400 --timeout-method thread "$@" ;;
smoke)
    step 300 "$OUT/smoke.log" python -c "import __graft_entry__ as g; g.smoke()" ;;
bench)
    timeout -k 10 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
    echo "[bench] rc=$rc"; cut -c1-400 "$OUT/bench.json"; exit $rc ;;
sweep)
    for te in "1 4096" "2 8192" "3 8192" "4 4096" "5 8192" "6 4096" "7 4096"; do
        set -- $te
        timeout -k 10 300 python bench.py --task $1 --envs $2 --steps 50 --warmup 5 --reps 3 > "$OUT/task$1.json" \
            2> "$OUT/task$1.err" || { echo "TASK $1 FAILED"; exit 1; }
        echo "task $1: $(cut -c1-160 "$OUT/task$1.json")"
    done ;;
phase)
    step 300 "$OUT/phase.txt" python tools/phase_prof.py "$@" ;;
chain)
    step 300 "$OUT/chain.txt" python tools/chain_bench.py "${1:-0}" "${2:-4096}" ;;
timeline)
    step 300 "$OUT/timeline.txt" python tools/timeline.py --json "$OUT/timeline.json" "$@" ;;
profile)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
        python3 bench.py --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1 || { echo TRACE_FAIL; exit 1; }
    echo TRACE_OK
    PMCARGS="--steps 20 --warmup 3 --reps 1"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
        python3 bench.py --no-cpu-baseline "$@" $PMCARGS > "$OUT/pmc_fetch.log" 2>&1 || { echo PMC1_FAIL; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
        python3 bench.py --no-cpu-baseline "$@" $PMCARGS > "$OUT/pmc_write.log" 2>&1 || { echo PMC2_FAIL; exit 1; }
    echo PMC_OK
    python3 tools/pmc_traffic.py "$OUT/pmc_fetch/run_counter_collection.csv" "$OUT/pmc_write/run_counter_collection.csv" \
        "$OUT/traffic_k_step.json" "$@" > /dev/null && echo TRAFFIC_OK
    timeout -k 10 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; exit 1; }
    echo BENCH_OK; cut -c1-400 "$OUT/bench.json" ;;
pmcmix)
    ARGS="${*:---steps 5 --warmup 2 --reps 1 --no-cpu-baseline}"
    i=0
    for G in "SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_FLAT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT"; do
        i=$((i+1))
        timeout -s KILL 180 rocprofv3 --pmc $G --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py $ARGS \
            > "$OUT/p$i.log" 2>&1 || { echo "PASS $i FAILED"; exit 1; }
    done
    echo PMC_MIX_OK ;;
icache)
    ARGS="${*:---steps 5 --warmup 2 --reps 1 --no-cpu-baseline}"
    timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
    G=""
    for c in SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE; do
        grep -qw "$c" "$OUT/counters.txt" && G="$G $c"
    done
    echo "icache counters:$G"
    [ -n "$G" ] || exit 0
    timeout -s KILL 180 rocprofv3 --pmc $G --output-format csv -d "$OUT/ic" -o run -- python3 bench.py $ARGS \
        > "$OUT/ic.log" 2>&1 || { echo "ICACHE PASS FAILED"; exit 1; }
    G2=""
    for c in SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES; do
        grep -qw "$c" "$OUT/counters.txt" && G2="$G2 $c"
    done
    [ -n "$G2" ] || exit 0
    timeout -s KILL 180 rocprofv3 --pmc $G2 --output-format csv -d "$OUT/if" -o run -- python3 bench.py $ARGS \
        > "$OUT/if.log" 2>&1 || { echo "IFETCH PASS FAILED"; exit 1; }
    echo ICACHE_OK ;;
contend)
    # co-runner contention: the same k_step work at the default wave slots and at URGYM_SLOTS=256
    # (one wave per CU), two counter passes each; tools/contend_pmc.py compares them per env-step
    ARGS="${*:---steps 5 --warmup 2 --reps 1 --no-cpu-baseline}"
    for SL in 0 256; do
        i=0
        mkdir -p "$OUT/s$SL"
        for G in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_REQ SQ_BUSY_CYCLES" \
                 "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES"; do
            i=$((i+1))
            URGYM_SLOTS=$SL timeout -s KILL 180 rocprofv3 --pmc $G --output-format csv -d "$OUT/s$SL/p$i" -o run -- \
                python3 bench.py $ARGS > "$OUT/s$SL/p$i.log" 2>&1 || { echo "CONTEND $SL PASS $i FAILED"; exit 1; }
        done
    done
    python3 tools/contend_pmc.py "$OUT" > "$OUT/contend.txt" && cat "$OUT/contend.txt" ;;
world8)
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 8 --backend gloo --no-cpu-baseline "$@" > "$OUT/world8.json" \
        2> "$OUT/world8.err"; rc=$?
    echo "[world8] rc=$rc"; cut -c1-400 "$OUT/world8.json"; exit $rc ;;
final)
    bash tools/gpu.sh tests "$TAG" && bash tools/gpu.sh smoke "$TAG" && bash tools/gpu.sh bench "$TAG" ;;
*)
    echo "unknown job $JOB"; exit 2 ;;
esac
