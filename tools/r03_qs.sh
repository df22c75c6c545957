#!/bin/bash
# the separate quality pass on a second stream: all GPU tests, then cfg4 / cfg5 A/B (one stream,
# chunk sizes, the fused path)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/t_all.log
[ $rc -ne 0 ] && exit $rc
AB_ARGS="--workload=cfg4" ./tools/ab7.sh c4_2s:: c4_1s::DTS_QSTREAM=0 c4_c8::DTS_QCHUNK=8 c4_c32::DTS_QCHUNK=32 c4_qf::DTS_QFUSE=1 || exit $?
AB_ARGS="--workload=cfg5" ./tools/ab7.sh c5_2s:: c5_1s::DTS_QSTREAM=0 c5_c300::DTS_QCHUNK=300 c5_c64::DTS_QCHUNK=64 c5_qf::DTS_QFUSE=1 || exit $?
exit 0
