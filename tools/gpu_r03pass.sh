#!/bin/bash
# Round-3 GPU pass on one box: (tests + smoke unless NOTESTS), then per workload the unprofiled
# bench line and its rocprofv3 passes (tools/prof_wl.sh), all from this build.
# usage: tools/gpu_r03pass.sh TAG [workloads...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
if [ -z "$NOTESTS" ]; then bash tools/gpu_check.sh tests smoke || exit $?; fi
for w in "$@"; do
  extra=""
  [ $w = cfg5 ] && extra="--steps 8 --warmup 2"
  LINE=1 bash tools/prof_wl.sh $tag $w $extra || exit $?
done
exit 0
