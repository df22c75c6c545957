#!/bin/bash
# stamp breakdown and bench value vs batch / ring size (TLB / footprint sensitivity)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r02x}
for cfg in "256 512" "64 64" "32 32"; do
  set -- $cfg
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-verify --batch $1 --ring $2 > gpurun_out/b4_${tag}_$1.log 2>&1; rc=$?
  echo "batch $1 ring $2 rc=$rc $(tail -n 1 gpurun_out/b4_${tag}_$1.log | cut -c100-175)"
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 120 python tools/stamp5.py --batch $1 --ring $2 > gpurun_out/s4_${tag}_$1.log 2>&1; rc=$?
  tail -n 7 gpurun_out/s4_${tag}_$1.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
