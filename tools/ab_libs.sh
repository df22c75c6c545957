#!/bin/bash
# A/B of libdts builds on the cfg2 bench: tools/ab_libs.sh <lib-suffix>... ("" or base = lib/libdts.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=distributed-transcoding-server_amd/lib
for v in "$@"; do
  [ "$v" = base ] && v=""
  lib=$L/libdts${v:+_$v}.so
  for wl in ${AB_WORKLOADS:-cfg2}; do
    DTS_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --workload $wl > gpurun_out/ab_${v:-base}_$wl.log 2>&1
    rc=$?
    echo "== ${v:-base} $wl rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v:-base}_$wl.log) $(grep -o '"frac": [0-9.]*' gpurun_out/ab_${v:-base}_$wl.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/ab_${v:-base}_$wl.log)"
    [ $rc -ge 124 ] && exit $rc
  done
done
exit 0
