#!/bin/bash
# Launch-order models off their training distribution: every task with a k_prio model, each action
# stream (uniform, Ornstein-Uhlenbeck, x0.3), with the model and with the fallback order (URGYM_NO_PRIO_MODEL=1: the
# last substep count), same seeds -> gpurun_out/<tag>/ab_task<T>_<actions>_<model|fallback>.json
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${1:-prio_ab}; O=gpurun_out/$TAG; mkdir -p $O
for te in "0 4096" "6 4096" "1 4096" "4 4096" "2 8192"; do
    set -- $te
    for A in uniform ou scaled; do
        for M in model fallback; do
            NP=0; [ $M = fallback ] && NP=1
            URGYM_NO_PRIO_MODEL=$NP timeout -k 10 240 python bench.py --no-cpu-baseline --task $1 --envs $2 --steps 60 \
                --warmup 10 --reps 3 --actions $A > $O/ab_task$1_${A}_$M.json 2> $O/ab_task$1_${A}_$M.err \
                || { echo "AB $1 $A $M FAILED"; exit 1; }
            echo "task $1 $A $M $(python -c "import json; d=json.load(open('$O/ab_task$1_${A}_$M.json')); print(round(d['value']), [round(x) for x in d['rep_values']])")"
        done
    done
done
