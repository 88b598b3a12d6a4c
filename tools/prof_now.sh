cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python tools/phase_prof.py --steps 5 > gpurun_out/phase.txt 2>&1 || exit 1
timeout -k 10 200 python tools/chain_bench.py 0 4096 > gpurun_out/chain.txt 2>&1 || exit 1
timeout -k 10 200 python tools/timeline.py 4096 20 > gpurun_out/timeline.txt 2>&1 || exit 1
