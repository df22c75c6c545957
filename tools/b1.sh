cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b_cfg2.log 2>&1; echo "cfg2 rc=$?"; tail -n 2 gpurun_out/b_cfg2.log
timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu --workload cfg4 > gpurun_out/b_cfg4.log 2>&1; echo "cfg4 rc=$?"; tail -n 2 gpurun_out/b_cfg4.log
bash tools/prof_kt.sh r02a
cat gpurun_out/prof_r02a/r02a_kernel_stats.csv
