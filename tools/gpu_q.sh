cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_quality.py tests/test_gpu_configs.py > gpurun_out/t_q.log 2>&1; rc=$?; tail -n 2 gpurun_out/t_q.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab7.sh full:: prev:prev: full2:: prev2:prev:
AB_WORKLOADS="cfg5 cfg4" bash tools/ab_libs.sh "" prev
