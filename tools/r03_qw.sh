#!/bin/bash
# the walking k_quality build: every -m gpu test + smoke, then the cfg4 / cfg5 lines with their
# rocprofv3 passes (tools/prof_wl.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r03d}
bash tools/gpu_check.sh tests smoke || exit $?
grep -q "passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || { echo "tests not green"; exit 1; }
tail -1 gpurun_out/tests.log
LINE=1 bash tools/prof_wl.sh $tag cfg4 || exit $?
LINE=1 bash tools/prof_wl.sh $tag cfg5 --steps 8 --warmup 2 || exit $?
