#!/bin/bash
# Golf phase cycles (default geometry) with the cylinder-pass counters
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/golfprof; mkdir -p $OUT
timeout -k 10 300 python tools/phase_prof.py --steps 3 --task 3 --envs 2048 > $OUT/phase_golf.txt 2>&1 || exit 1
grep -E "cyl|hull_narrow|collide_cycles" $OUT/phase_golf.txt
