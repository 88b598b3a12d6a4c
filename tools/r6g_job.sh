set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
b() { # b <tag> <task> <envs> [env assignments...]
  local tag=$1 t=$2 e=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --task $t --envs $e --steps 30 --warmup 5 --reps 3 > $O/$tag.json 2> $O/$tag.err || { echo "$tag FAIL"; tail -3 $O/$tag.err; return 1; }
  echo "$tag $(python -c "import json; d=json.load(open('$O/$tag.json')); print(round(d['value']), round(d['ms_per_step'],2))")"
}
b g_nohelp 3 8192 URGYM_NO_HELPERS=1 && b g_h64 3 8192 URGYM_HELPERS=64 && b g_h16 3 8192 URGYM_HELPERS=16 && \
b g_h256 3 8192 URGYM_HELPERS=256 && b bb_nohelp 0 4096 URGYM_NO_HELPERS=1 && b bb_h64 0 4096 URGYM_HELPERS=64 && \
b bb_h16 0 4096 URGYM_HELPERS=16 && b cp_nohelp 1 4096 URGYM_NO_HELPERS=1 && b cp_h64 1 4096 URGYM_HELPERS=64
