#!/bin/bash
# V sub-ablations + per-phase stamps of k_ladder7 on cfg2, then cfg3 / cfg4 / cfg5 lines + profiles
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/r03_abl2.sh || exit $?
timeout -k 10 240 python -u tools/stamp7.py > gpurun_out/stamp7.log 2>&1; rc=$?
echo "stamp rc=$rc"; grep -v "^{" gpurun_out/stamp7.log | tail -40
[ $rc -ne 0 ] && exit $rc
NOTESTS=1 bash tools/gpu_r03pass.sh r03a cfg3 cfg4 cfg5
