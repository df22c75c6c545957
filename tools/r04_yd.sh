#!/bin/bash
# round 4: k_yadif_t after the packed / branch-free rewrite: its parity tests, then the yadif line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_yadif.py > gpurun_out/yd_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/yd_tests.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/yd_tests.log; exit $rc; }
timeout -k 10 200 python -u bench.py --workload yadif --steps 20 --warmup 3 --no-cpu > gpurun_out/yd_line.log 2>&1
rc=$?; echo "line rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/yd_line.log) $(grep -o '"frac": [0-9.]*' gpurun_out/yd_line.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/yd_line.log)"
exit $rc
