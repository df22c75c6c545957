#!/bin/bash
# round 5: the ABI-7 host path (pinned frames, direct DMA): parity tests, then the --e2e line
# with pageable and with pinned host frames
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-r05h}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_abi.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/$tag/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$tag/tests.log; [ $rc -ne 0 ] && exit $rc
for m in "" "--e2e-pinned"; do
  n=${m:+pinned}; n=${n:-pageable}
  timeout -k 10 300 python3 -u bench.py --e2e --steps 10 --warmup 2 $m > gpurun_out/$tag/e2e_$n.log 2>&1 || { tail -5 gpurun_out/$tag/e2e_$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' gpurun_out/$tag/e2e_$n.log) $(grep -o '"h2d_GBps": [0-9.]*' gpurun_out/$tag/e2e_$n.log) $(grep -o '"d2h_GBps": [0-9.]*' gpurun_out/$tag/e2e_$n.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/$tag/e2e_$n.log)"
done
exit 0
