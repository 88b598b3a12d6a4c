# GPU suite on the in-tree build, then A/B against the libraries kept in urgym_amd/_lib/base (the previous build):
# bash tools/r6ab.sh <tag> "<task> <envs>"...   (60 steps x 3 reps after 10 warm-up, same seeds)
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
[ -f $O/tests.log ] && tail -1 $O/tests.log
for te in "$@"; do
  set -- $te
  BL=urgym_amd/_lib/base/liburgym.so; [ "$1" = 3 ] || [ "$1" = 5 ] && BL=urgym_amd/_lib/base/liburgym_g8.so
  for v in new base; do
    if [ $v = base ]; then export URGYM_LIB=$PWD/$BL; else unset URGYM_LIB; fi
    timeout -k 10 400 python bench.py --no-cpu-baseline --task $1 --envs $2 --steps 60 --warmup 10 --reps 3 ${BENCH_ARGS:-} > $O/t$1_$v.json 2> $O/t$1_$v.err || { echo "T$1 $v FAIL"; tail -3 $O/t$1_$v.err; exit 1; }
  done
  unset URGYM_LIB
  echo "task $1: new $(python -c "import json; d=json.load(open('$O/t$1_new.json')); print(round(d['value']), [round(v) for v in d['rep_values']])") base $(python -c "import json; d=json.load(open('$O/t$1_base.json')); print(round(d['value']), [round(v) for v in d['rep_values']])")"
done
