# phase cycles of the profiling build: bash tools/r6_phase.sh <tag> "<task> <envs>"...
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
for te in "$@"; do
  set -- $te
  LIB=urgym_amd/_lib/liburgym_prof.so; [ "$1" = 3 ] || [ "$1" = 5 ] && LIB=urgym_amd/_lib/liburgym_prof_g8.so
  URGYM_LIB=$PWD/$LIB timeout -k 10 300 python tools/phase_prof.py --task $1 --envs $2 --steps 5 > $O/phase_task$1.txt 2>&1 || { echo "PH $1 FAIL"; tail -3 $O/phase_task$1.txt; exit 1; }
  echo "phase $1 done"
done
