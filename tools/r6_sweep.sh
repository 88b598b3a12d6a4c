# round-6 per-task table at the SURVEY 8(d) protocol (bench.py defaults: 10 warm-up, 5 reps x 200 steps, median,
# rep spread in rep_values): bash tools/r6_sweep.sh <tag> "<task> <envs>"...   -> gpurun_out/<tag>/task<N>.json
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
for te in "$@"; do
  set -- $te
  timeout -k 10 420 python bench.py --no-cpu-baseline --task $1 --envs $2 > $O/task$1.json 2> $O/task$1.err || { echo "TASK $1 FAIL"; tail -3 $O/task$1.err; exit 1; }
  echo "task $1: $(python -c "import json; d=json.load(open('$O/task$1.json')); print(round(d['value']), round(d['ms_per_step'],2), [round(v) for v in d['rep_values']], d.get('library',''))")"
done
