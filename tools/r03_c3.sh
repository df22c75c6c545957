#!/bin/bash
# round-3 closing pass in one call: part A of the round-end pass (tests + smoke, cfg2 / cfg3 / cfg1
# profiles), the walking k_quality candidate (lib/libdts_qwalk.so: its quality tests, cfg5 / cfg4
# kernel traces against this build), then part B (cfg4 / cfg5 / yadif / cfg2nv12 profiles, e2e line)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${1:-r03c}
bash tools/gpu_final_a.sh $tag || exit $?
DTS_LIB=$PWD/distributed-transcoding-server_amd/lib/libdts_qwalk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_quality.py tests/test_gpu_qfuse.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qwalk_tests.log 2>&1
rc=$?; echo "qwalk tests rc=$rc $(tail -1 gpurun_out/qwalk_tests.log)"; [ $rc -ge 124 ] && exit $rc
Q5_VARS="base qwalk" bash tools/r03_q5.sh || exit $?
bash tools/gpu_final_b.sh $tag
