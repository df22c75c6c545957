#!/bin/bash
# round 5: the host path -- parity, then its shape: submit size, chunk size, pinned vs pageable
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-r05e}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python -u -m pytest tests/test_node.py tests/test_gpu_configs.py tests/test_gpu_hdr.py -m gpu -q \
    --timeout 150 --timeout-method thread > gpurun_out/$tag/tests.log 2>&1
rc=$?; echo "host-path tests rc=$rc $(tail -1 gpurun_out/$tag/tests.log)"; [ $rc -ne 0 ] && exit $rc
run() { # name, env, args
  local n=$1; shift
  env $1 timeout -k 10 300 python3 -u bench.py --e2e --steps 6 --warmup 2 $2 > gpurun_out/$tag/$n.log 2>&1 || { tail -3 gpurun_out/$tag/$n.log; exit 1; }
  echo "== $n $(grep -o '"value": [0-9.]*' gpurun_out/$tag/$n.log) $(grep -o '"h2d_GBps": [0-9.]*' gpurun_out/$tag/$n.log) $(grep -o '"d2h_GBps": [0-9.]*' gpurun_out/$tag/$n.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/$tag/$n.log)"
}
run page_128_32 X=1 ""
run pin_128_32 X=1 "--e2e-pinned"
run page_512_64 X=1 "--e2e-submit 512 --e2e-batch 64 --e2e-frames 256"
run pin_512_64 X=1 "--e2e-pinned --e2e-submit 512 --e2e-batch 64 --e2e-frames 256"
exit 0
