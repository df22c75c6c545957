#!/bin/bash
# Round-2 final GPU pass: every gpu test, smoke, every bench line (with the CPU
# baseline), then the cfg2 rocprofv3 kernel trace + PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r02d}
bash tools/gpu_check.sh tests smoke || exit $?
for w in cfg2 cfg1 cfg3 cfg4 cfg5 yadif; do
  extra="--cpu-seconds 10"
  [ $w = cfg5 ] && extra="--steps 8 --warmup 2 --cpu-seconds 10"
  timeout -k 10 400 python -u bench.py --workload $w $extra > gpurun_out/final_$w.log 2>&1
  rc=$?
  echo "$w rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/final_$w.log | head -1) $(grep -o '"frac": [0-9.]*' gpurun_out/final_$w.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/final_$w.log)"
  [ $rc -ne 0 ] && exit $rc
done
bash tools/profile.sh $tag
