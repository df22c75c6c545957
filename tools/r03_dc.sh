#!/bin/bash
# decoupled staging: every gpu test, then cfg2 / cfg2nv12 / cfg3 A/B against the coupled build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/t_all.log
[ $rc -ne 0 ] && exit $rc
./tools/ab7.sh dc2:: dc0:dc0: dc1:dc1: dc2b:: dc0b:dc0: || exit $?
AB_ARGS="--workload=cfg2nv12" ./tools/ab7.sh nv_dc2:: nv_dc0:dc0: || exit $?
AB_ARGS="--workload=cfg3" ./tools/ab7.sh c3_dc2:: c3_dc0:dc0: || exit $?
exit 0
