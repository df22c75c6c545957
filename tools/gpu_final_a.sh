#!/bin/bash
# round-end pass, part 1: tests + smoke, then the cfg2 (with SQ counters), cfg3 and cfg1 lines with
# their rocprofv3 passes, all from this build on this box (tools/prof_wl.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r03b}
bash tools/gpu_check.sh tests smoke || exit $?
grep -q "passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || { echo "tests not green"; exit 1; }
SQ=1 LINE=1 bash tools/prof_wl.sh $tag cfg2 || exit $?
LINE=1 bash tools/prof_wl.sh $tag cfg3 || exit $?
LINE=1 bash tools/prof_wl.sh $tag cfg1 || exit $?
exit 0
