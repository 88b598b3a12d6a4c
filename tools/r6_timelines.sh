# block timelines (profiling builds) of each task at its BASELINE size: longest env vs balanced work
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
for te in "$@"; do
  set -- $te
  LIB=urgym_amd/_lib/liburgym_prof.so; [ "$1" = 3 ] || [ "$1" = 5 ] && LIB=urgym_amd/_lib/liburgym_prof_g8.so
  URGYM_LIB=$PWD/$LIB timeout -k 10 300 python tools/timeline.py --task $1 --envs $2 --steps 12 --skip 4 --json $O/timeline_task$1.json > $O/timeline_task$1.txt 2>&1 || { echo "TL $1 FAIL"; tail -3 $O/timeline_task$1.txt; exit 1; }
  echo "timeline $1: $(grep -i -m3 'launch\|balanced\|longest' $O/timeline_task$1.txt | tr '\n' ' ' | cut -c1-300)"
done
