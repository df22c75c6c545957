#!/bin/bash
# round-end pass, part 2: cfg4, cfg5 (8 steps), yadif and cfg2nv12 lines with their rocprofv3 passes,
# then the host-memory end-to-end line (cfg2)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r03b}
LINE=1 bash tools/prof_wl.sh $tag cfg4 || exit $?
LINE=1 bash tools/prof_wl.sh $tag cfg5 --steps 8 --warmup 2 || exit $?
LINE=1 bash tools/prof_wl.sh $tag yadif || exit $?
LINE=1 NOCPU=1 bash tools/prof_wl.sh $tag cfg2nv12 || exit $?
timeout -k 10 300 python -u bench.py --e2e --steps 10 --warmup 2 > gpurun_out/e2e_cfg2.log 2>&1; rc=$?
echo "e2e rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/e2e_cfg2.log) $(grep -o '"host_io_GBps": [0-9.]*' gpurun_out/e2e_cfg2.log)"
exit $rc
