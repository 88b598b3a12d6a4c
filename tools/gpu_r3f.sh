#!/bin/bash
# phase cycles of the default (full) geometry: Golf and BallBalance
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3f
timeout -k 10 300 python tools/phase_prof.py --steps 3 --task 3 --envs 2048 > gpurun_out/r3f/phase_golf_full.txt 2>&1 || exit 1
timeout -k 10 300 python tools/phase_prof.py --steps 5 > gpurun_out/r3f/phase_bb_full.txt 2>&1 || exit 1
