#!/bin/bash
# round 5: k_yadif_t at 8 pixels per thread (1024-thread workgroups, 8 waves per SIMD) -- yadif
# parity, then the A/B against 16 pixels (np16), 8 pixels at 4 waves (np8w1) and the previous walk
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05yt
timeout -k 10 400 python -u -m pytest tests/test_gpu_yadif.py tests/test_gpu_configs.py -m gpu -q -k "yadif or deint" \
    --timeout 300 --timeout-method thread > gpurun_out/r05yt/tests.log 2>&1
rc=$?; echo "yadif tests rc=$rc $(tail -1 gpurun_out/r05yt/tests.log)"; [ $rc -ne 0 ] && exit $rc
AB_WORKLOADS=yadif bash tools/ab_libs.sh ${AB_LIBS:-base np16 np8w1 ytold base np16 np8w1 ytold}
