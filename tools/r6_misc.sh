# round-6 end extras: Golf / GolfJoints on round 5's short protocol (50 x 3 after 5), timelines of the other tasks,
# CubesPush phase cycles, smoke
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r6misc; mkdir -p $O
for t in 3 5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --task $t --envs 8192 --steps 50 --warmup 5 --reps 3 > $O/short_task$t.json 2> $O/short_task$t.err || { echo "SHORT $t FAIL"; exit 1; }
  echo "short $t: $(cut -c1-120 $O/short_task$t.json)"
done
bash tools/r6_timelines.sh r6tl2 "4 4096" "5 8192" "6 4096" "7 4096" || exit 1
bash tools/r6_phase.sh r6ph2 "1 4096" || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
