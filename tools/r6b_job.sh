set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/r6b
timeout -k 10 300 python tools/predict_steps_cg.py 8192 45 > gpurun_out/r6b/cg.log 2>&1 || { echo CG_FAIL; tail -5 gpurun_out/r6b/cg.log; exit 1; }
echo CG_OK; tail -2 gpurun_out/r6b/cg.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6b/fc_fetch -o run -- ./tools/micro/fetchcal > gpurun_out/r6b/fc_fetch.log 2>&1 || { echo FC1_FAIL; tail -5 gpurun_out/r6b/fc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6b/fc_write -o run -- ./tools/micro/fetchcal > gpurun_out/r6b/fc_write.log 2>&1 || { echo FC2_FAIL; tail -5 gpurun_out/r6b/fc_write.log; exit 1; }
python tools/fetchcal.py gpurun_out/r6b/fc_fetch/run_counter_collection.csv gpurun_out/r6b/fc_write/run_counter_collection.csv gpurun_out/r6b/fetchcal.json || echo FCRED_FAIL
timeout -k 10 300 python tools/phase_prof.py --task 0 --envs 4096 --steps 5 > gpurun_out/r6b/phase_bb.txt 2>&1 || { echo PHASE_FAIL; tail -5 gpurun_out/r6b/phase_bb.txt; exit 1; }
echo PHASE_OK
timeout -k 10 300 python tools/phase_prof.py --task 1 --envs 4096 --steps 5 > gpurun_out/r6b/phase_cp.txt 2>&1 || { echo PHASE1_FAIL; exit 1; }
echo PHASE1_OK
bash tools/gpu.sh tests r6b tests/test_gpu_queue.py
