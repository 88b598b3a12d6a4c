#!/bin/bash
# round-3 profile set of the default (full) geometry: phase cycles (full and LOD), reset / step chain timings,
# rocprofv3 kernel trace + stats, PMC traffic passes, bench line with the CPU baseline
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3p
timeout -k 10 200 python tools/phase_prof.py --steps 5 > gpurun_out/r3p/phase_bb_full.txt 2>&1 || exit 1
timeout -k 10 200 python tools/phase_prof.py --steps 5 --geometry lod > gpurun_out/r3p/phase_bb_lod.txt 2>&1 || exit 1
timeout -k 10 200 python tools/chain_bench.py 0 4096 > gpurun_out/r3p/chain_full.txt 2>&1 || exit 1
bash tools/profile_round.sh round3_full
