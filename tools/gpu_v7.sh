#!/bin/bash
# v7 bring-up: the ladder parity tests on the default (v7) kernel, then cfg2 bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ladder.py -k "v7" \
    > gpurun_out/t_v7.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAIL|Error" gpurun_out/t_v7.log | tail -n 8
[ $rc -ne 0 ] && exit $rc
for w in ${L7_WS:-8}; do
  DTS_L7_W=$w timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b_v7_w$w.log 2>&1
  rc=$?
  echo "W=$w rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/b_v7_w$w.log) $(grep -o '"frac": [0-9.]*' gpurun_out/b_v7_w$w.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/b_v7_w$w.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
