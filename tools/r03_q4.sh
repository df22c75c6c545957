#!/bin/bash
# k_quality walking kQWalk tiles per workgroup: the quality GPU tests, then cfg5 / cfg4 A/B against
# the previous kernel (libdts_oldq.so) and walks of 2 / 8 tiles (tools/build_qvar.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_quality.py tests/test_gpu_qfuse.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/q4_tests.log; [ $rc -ne 0 ] && exit $rc
AB_WORKLOADS="cfg5 cfg4" bash tools/ab_libs.sh oldq "" w2 w8
