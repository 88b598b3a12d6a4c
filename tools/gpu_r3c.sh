#!/bin/bash
# phase cycles of the LOD vs full geometry (profiling build), and the default bench protocol for the LOD baseline
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3c
for g in lod full; do
  timeout -k 10 200 python tools/phase_prof.py --steps 5 --geometry $g > gpurun_out/r3c/phase_bb_$g.txt 2>&1 || exit 1
  timeout -k 10 300 python tools/phase_prof.py --steps 3 --task 3 --envs 2048 --geometry $g > gpurun_out/r3c/phase_golf_$g.txt 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r3c/bench_default.json 2> gpurun_out/r3c/bench_default.err || exit 1
cut -c1-200 gpurun_out/r3c/bench_default.json
