#!/bin/bash
# round 5: k_quality in XCD order -- the quality parity tests, cfg5 / cfg4 lines, then their
# kernel traces and FETCH_SIZE / WRITE_SIZE passes (tools/prof_wl.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-r05q2}
mkdir -p gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_gpu_quality.py tests/test_gpu_cfg5.py tests/test_gpu_bench_paths.py tests/test_gpu_configs.py \
    -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$tag/tests.log 2>&1
rc=$?; echo "quality tests rc=$rc $(tail -1 gpurun_out/$tag/tests.log)"; [ $rc -ne 0 ] && { tail -20 gpurun_out/$tag/tests.log; exit $rc; }
for wl in cfg5 cfg4; do bash tools/prof_wl.sh $tag $wl || exit $?; done
exit 0
