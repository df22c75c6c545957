#!/bin/bash
# fused quality: its GPU tests, then all GPU tests, then cfg5 / cfg4 lines fused vs DTS_QFUSE=0 and cfg2
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DTS_QFUSE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_qfuse.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_qf.log 2>&1; rc=$?
echo "qfuse tests rc=$rc"; tail -12 gpurun_out/t_qf.log
[ $rc -ne 0 ] && exit $rc
DTS_QFUSE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/t_all.log
[ $rc -ne 0 ] && exit $rc
AB_ARGS="--workload=cfg5 --steps 6 --warmup 2" ./tools/ab7.sh c5_qf::DTS_QFUSE=1 c5_sep::DTS_QFUSE=0 || exit $?
AB_ARGS="--workload=cfg4" ./tools/ab7.sh c4_qf::DTS_QFUSE=1 c4_sep::DTS_QFUSE=0 || exit $?
./tools/ab7.sh c2:: || exit $?
exit 0
