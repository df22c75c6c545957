cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --workload cfg3 --cpu-seconds 8 > gpurun_out/bench_cfg3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --workload cfg4 --batch 16 --ring 48 --cpu-seconds 8 > gpurun_out/bench_cfg4.log 2>&1
rc=$?
tail -n 3 gpurun_out/bench_cfg3.log gpurun_out/bench_cfg4.log
exit $rc
