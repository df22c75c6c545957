#!/bin/bash
# quick v5 check: small parity, cfg2 bench line, rocprofv3 kernel trace + PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r02x}
timeout -k 10 180 python -u -m pytest tests/test_gpu_ladder.py -x -q --timeout 60 --timeout-method thread -k "v5 and (small or identity or 4k)" > gpurun_out/t_$tag.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/t_$tag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b_$tag.log 2>&1; echo "bench rc=$?"; tail -n 1 gpurun_out/b_$tag.log | cut -c1-400
bash tools/profile.sh $tag --batch 256 > gpurun_out/p_$tag.log 2>&1; echo "prof rc=$?"
