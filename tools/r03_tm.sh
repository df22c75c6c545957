#!/bin/bash
# k_tonemap: the HDR parity tests on this build, then cfg3 A/B of variant builds (tools/build_tmvar.sh:
# noslp = -fno-slp-vectorize; abr / abf / abm / abrf = DTS_TM_ABLATE 1 / 2 / 4 / 3, diagnostic, wrong output)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hdr.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tm_tests.log 2>&1
rc=$?; tail -2 gpurun_out/tm_tests.log; [ $rc -ne 0 ] && exit $rc
AB_WORKLOADS=cfg3 bash tools/ab_libs.sh "" ${TM_VARS:-noslp abr abf abm abrf}
