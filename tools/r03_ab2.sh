#!/bin/bash
# k_ladder7 HS=128 epilogue + SIMD-balanced unit order: v7 parity tests, then cfg2 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ladder.py tests/test_gpu_configs.py tests/test_golden.py tests/test_gpu_cfg5.py tests/test_gpu_quality.py tests/test_node.py -m gpu -x -q --timeout 300 --timeout-method thread -k "v7 or configs or golden or cfg5 or rendition or worker" > gpurun_out/t_v7.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/t_v7.log
[ $rc -ne 0 ] && exit $rc
./tools/ab7.sh new:: hs256::DTS_L7_HSPLIT=256 nobal::DTS_L7_BAL=0 old::DTS_L7_HSPLIT=256,DTS_L7_BAL=0 new2::
for t in 1 16; do
  DTS_HOST_THREADS=$t timeout -k 10 300 python -u bench.py --e2e --steps 6 --warmup 2 > gpurun_out/e2e_t$t.log 2>&1; rc=$?
  echo "== e2e threads $t rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/e2e_t$t.log) $(grep -o '"host_io_GBps": [0-9.]*' gpurun_out/e2e_t$t.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/e2e_t$t.log)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
