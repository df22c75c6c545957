#!/bin/bash
# every -m gpu test, then the e2e line at 1 / 16 host threads, the DMA-position A/B and the nv12 line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/t_all.log
[ $rc -ge 124 ] && exit $rc
for t in 1 16; do
  DTS_HOST_THREADS=$t timeout -k 10 300 python -u bench.py --e2e --steps 6 --warmup 2 > gpurun_out/e2e_t$t.log 2>&1; rc=$?
  echo "== e2e threads $t rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/e2e_t$t.log) $(grep -o '"host_io_GBps": [0-9.]*' gpurun_out/e2e_t$t.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/e2e_t$t.log)"
  [ $rc -ge 124 ] && exit $rc
done
./tools/ab7.sh base:: dma1:dma1: || exit $?
AB_ARGS="--workload cfg2nv12" ./tools/ab7.sh nv12:: || exit $?
exit 0
