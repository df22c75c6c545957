#!/bin/bash
# every bench line (cfg2 default, cfg3, cfg4, cfg5, yadif) -> gpurun_out/bench_<w>.log
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in cfg2 cfg3 cfg4 cfg5 yadif; do
  extra=""
  [ $w = cfg5 ] && extra="--steps 4 --warmup 1"
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --workload $w --cpu-seconds 8 $extra > gpurun_out/bench_$w.log 2>&1
  rc=$?
  echo "$w rc=$rc $(tail -n 1 gpurun_out/bench_$w.log | cut -c1-160)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
