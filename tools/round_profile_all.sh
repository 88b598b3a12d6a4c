#!/bin/bash
# Round profile set on the GPU box: bench + rocprofv3 kernel stats + PMC traffic (tools/profile_round.sh), the
# instruction-mix PMC passes (tools/pmc_mix.sh) and the per-task sweep (tools/task_sweep.sh).
# usage (GPU box): bash tools/round_profile_all.sh <tag>
set -u
TAG=${1:-round2}
cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh $TAG || exit 1
bash tools/pmc_mix.sh gpurun_out/$TAG/pmc_mix || exit 1
bash tools/task_sweep.sh gpurun_out/$TAG/tasks || exit 1
echo ALL_OK
