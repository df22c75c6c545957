#!/bin/bash
# v6 bring-up: the ladder parity tests on the v6 kernel, then a short cfg2 bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ladder.py -k "v6" \
    > gpurun_out/t_v6.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -n 4 gpurun_out/t_v6.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b_v6.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -n 2 gpurun_out/b_v6.log | cut -c1-600
exit $rc
