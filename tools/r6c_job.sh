set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
bash tools/gpu.sh tests r6c || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_bb.json 2> $O/bench_bb.err || { echo BENCH_FAIL; exit 1; }
echo "BB $(cut -c1-200 $O/bench_bb.json)"
timeout -k 10 300 python bench.py --no-cpu-baseline --task 2 --envs 8192 --steps 40 --warmup 5 --reps 3 > $O/bench_cg.json 2> $O/bench_cg.err || { echo CG_FAIL; exit 1; }
echo "CG $(cut -c1-200 $O/bench_cg.json)"
URGYM_NO_PRIO_MODEL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --task 2 --envs 8192 --steps 40 --warmup 5 --reps 3 > $O/bench_cg_noprio.json 2> $O/bench_cg_noprio.err || { echo CGN_FAIL; exit 1; }
echo "CGN $(cut -c1-200 $O/bench_cg_noprio.json)"
timeout -k 10 300 python tools/phase_prof.py --task 0 --envs 4096 --steps 5 > $O/phase_bb.txt 2>&1 || { echo PHASE_FAIL; exit 1; }
echo PHASE_OK
