#!/bin/bash
# Full GPU pass: every gpu test, smoke, every bench workload (no CPU leg), short.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit $?
for w in ${WLS:-cfg2 cfg3 cfg4 cfg5 yadif}; do
  extra=""
  [ $w = cfg5 ] && extra="--steps 4 --warmup 1"
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --workload $w --no-cpu $extra > gpurun_out/all_$w.log 2>&1
  rc=$?
  echo "$w rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/all_$w.log) $(grep -o '"frac": [0-9.]*' gpurun_out/all_$w.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/all_$w.log)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
