#!/bin/bash
# Round-end GPU pass: every gpu test, smoke, the default bench line, the extra
# workload lines, and the cfg2 rocprofv3 kernel-trace + PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r01v9}
bash tools/gpu_check.sh tests smoke || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/final_cfg2.log 2>&1 || exit $?
tail -n 1 gpurun_out/final_cfg2.log
for wl in cfg3 cfg4 yadif; do
  timeout -k 10 300 python -u bench.py --workload $wl --cpu-seconds 8 > gpurun_out/final_$wl.log 2>&1 || exit $?
  echo "$wl $(grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"verified_vs_oracle": [a-z]*' gpurun_out/final_$wl.log | tr '\n' ' ')"
done
bash tools/profile.sh $tag
