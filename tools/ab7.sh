#!/bin/bash
# A/B of k_ladder7 builds / knobs on the cfg2 bench.  Args: name:lib-suffix:ENV=V,ENV=V ...
# ("" suffix = lib/libdts.so).  Diagnostic only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/distributed-transcoding-server_amd/lib
for a in "$@"; do
  IFS=: read -r name suf envs <<< "$a"
  lib=$L/libdts${suf:+_$suf}.so
  ( IFS=,; for e in $envs; do export "$e"; done
    DTS_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu ${AB_ARGS:-} > gpurun_out/ab7_$name.log 2>&1 )
  rc=$?
  echo "== $name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab7_$name.log) $(grep -o '"frac": [0-9.]*' gpurun_out/ab7_$name.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/ab7_$name.log)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
