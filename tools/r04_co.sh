#!/bin/bash
# round 4: cfg3 ladder / tonemap co-residency.  lib/libdts_diagtm5.so = the diagnostic knobs +
# the five-wave k_tonemap (tm5); DTS_L7_LDS_MIN=86016 holds k_ladder7 to one group per CU, which
# leaves 74 KB of LDS for two tm5 workgroups beside it when the tonemaps run on their own stream
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/distributed-transcoding-server_amd/lib
run() {  # name lib envs...
  local name=$1 lib=$2; shift 2
  ( for e in "$@"; do export "$e"; done
    DTS_LIB=$lib timeout -k 10 200 python -u bench.py --workload cfg3 --steps 10 --warmup 2 --no-cpu > gpurun_out/coab_$name.log 2>&1 )
  local rc=$?
  echo "== $name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/coab_$name.log) $(grep -o '"frac": [0-9.]*' gpurun_out/coab_$name.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/coab_$name.log)"
  [ $rc -ge 124 ] && exit $rc
  return 0
}
run base $L/libdts.so
run tm5 $L/libdts_diagtm5.so DTS_HDR_STREAMS=1 DTS_HDR_CHUNK=256
run tm5s2c64 $L/libdts_diagtm5.so DTS_HDR_STREAMS=2 DTS_HDR_CHUNK=64
run tm5s2c64l $L/libdts_diagtm5.so DTS_HDR_STREAMS=2 DTS_HDR_CHUNK=64 DTS_L7_LDS_MIN=86016
run tm5s2c32l $L/libdts_diagtm5.so DTS_HDR_STREAMS=2 DTS_HDR_CHUNK=32 DTS_L7_LDS_MIN=86016
run tm5s2c128l $L/libdts_diagtm5.so DTS_HDR_STREAMS=2 DTS_HDR_CHUNK=128 DTS_L7_LDS_MIN=86016
run s1l $L/libdts_diagtm5.so DTS_HDR_STREAMS=1 DTS_HDR_CHUNK=256 DTS_L7_LDS_MIN=86016
exit 0
