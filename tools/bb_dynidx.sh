#!/bin/bash
# team_box_box with run-time-indexed column / element picks (-DUG_BB_DYNIDX) next to the
# serial dBoxBox2 restatement (-DUG_BB_CHECK prints mismatches), driven by the crafted box-box cases.
# Build here (CPU): hipcc ... -DUG_BB_DYNIDX -DUG_BB_CHECK -o urgym_amd/_lib/liburgym_bbdyn.so; run on the box.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/bbdyn
URGYM_LIB=$PWD/urgym_amd/_lib/liburgym_bbdyn.so timeout -k 10 300 python -u -m pytest tests/test_gpu_features.py -m gpu -v --timeout 200 --timeout-method thread -k box_box > gpurun_out/bbdyn/test.log 2>&1; echo "rc=$?"
grep -c BBCHK gpurun_out/bbdyn/test.log; grep -c BBIDX gpurun_out/bbdyn/test.log; grep -m5 "BBCHK\|BBIDX" gpurun_out/bbdyn/test.log; tail -3 gpurun_out/bbdyn/test.log
