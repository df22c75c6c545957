#!/bin/bash
# quick v5 loop: small parity, cfg2 bench line, per-phase stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r02x}
timeout -k 10 180 python -u -m pytest tests/test_gpu_ladder.py tests/test_gpu_configs.py -x -q --timeout 60 --timeout-method thread -k "v5 and (small or identity or 4k or odd or every) or cfg" > gpurun_out/t_$tag.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/t_$tag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b_$tag.log 2>&1; echo "bench rc=$?"; tail -n 1 gpurun_out/b_$tag.log | cut -c1-200
timeout -k 10 200 python tools/stamp5.py > gpurun_out/s_$tag.log 2>&1; echo "stamp rc=$?"; tail -n 7 gpurun_out/s_$tag.log
