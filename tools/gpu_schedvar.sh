#!/bin/bash
# compiler-scheduling variants of liburgym.so (urgym_amd/_lib/var/*.so): parity suite + bench line each
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sched
for v in base v1 v4 v5; do
  if [ $v = base ]; then L=urgym_amd/_lib/liburgym.so; else L=urgym_amd/_lib/var/$v.so; fi
  URGYM_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/sched/$v.test.log 2>&1 || { echo "$v PARITY FAIL"; tail -5 gpurun_out/sched/$v.test.log; exit 1; }
  URGYM_LIB=$PWD/$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --reps 3 > gpurun_out/sched/$v.bench.json 2> gpurun_out/sched/$v.bench.err || { echo "$v BENCH FAIL"; exit 1; }
  python -c "import json,sys; b=json.loads(open('gpurun_out/sched/$v.bench.json').read().strip().splitlines()[-1]); print('$v', round(b['value']), round(b['roofline']['avg_kernel_ms'],3))"
done
