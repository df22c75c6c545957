#!/bin/bash
# every -m gpu test, then cfg3 (HDR chunk / second stream A/B) and the nv12-source line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/t_all.log
[ $rc -ge 124 ] && exit $rc
AB_ARGS="--workload=cfg3" ./tools/ab7.sh c3_1s256::DTS_HDR_STREAMS=1,DTS_HDR_CHUNK=256 c3_2s256::DTS_HDR_CHUNK=256 c3_2s32::DTS_HDR_CHUNK=32 c3_2s16::DTS_HDR_CHUNK=16 c3_auto:: c3_1sauto::DTS_HDR_STREAMS=1 || exit $?
AB_ARGS="--workload=cfg2nv12" ./tools/ab7.sh nv12:: || exit $?
exit 0
