cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/pcs
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pcs/avail.txt 2>&1
grep -i "pc.sampl\|pc_sampl\|host_trap\|stochastic" gpurun_out/pcs/avail.txt | head -20 > gpurun_out/pcs/pcs_lines.txt
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1000 --output-format csv -d gpurun_out/pcs/out -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --reps 1 > gpurun_out/pcs/run.log 2>&1
echo "rc=$?"; tail -5 gpurun_out/pcs/run.log; ls -R gpurun_out/pcs/out | head
