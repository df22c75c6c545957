#!/bin/bash
# p010 on k_ladder7: the HDR / p010 / ladder tests first, then all, then cfg3 + cfg2 lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hdr.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_hdr.log 2>&1; rc=$?
echo "hdr tests rc=$rc"; tail -15 gpurun_out/t_hdr.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/t_all.log
[ $rc -ge 124 ] && exit $rc
AB_ARGS="--workload=cfg3" ./tools/ab7.sh c3_v7:: c3_v4::DTS_LADDER=4 || exit $?
./tools/ab7.sh c2:: || exit $?
exit 0
