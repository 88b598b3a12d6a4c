set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r6d; mkdir -p $O
for te in "0 4096" "1 4096" "3 8192"; do
    set -- $te
    timeout -k 10 300 python tools/timeline.py --task $1 --envs $2 --steps 12 --skip 4 --json $O/timeline_task$1.json > $O/timeline_task$1.txt 2>&1 || { echo "TL $1 FAIL"; tail -3 $O/timeline_task$1.txt; exit 1; }
    echo "timeline task $1 OK"; tail -4 $O/timeline_task$1.txt | cut -c1-400
done
bash tools/gpu.sh sweep r6d || exit 1
