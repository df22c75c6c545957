#!/bin/bash
# round 4: cfg3 with the tonemaps on a stream of their own beside the next chunk's ladder
# (lib/libdts_diag.so reads DTS_HDR_STREAMS / DTS_HDR_CHUNK), against the default build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/distributed-transcoding-server_amd/lib
run() {  # name lib envs...
  local name=$1 lib=$2; shift 2
  ( for e in "$@"; do export "$e"; done
    DTS_LIB=$lib timeout -k 10 200 python -u bench.py --workload cfg3 --steps 10 --warmup 2 --no-cpu > gpurun_out/hdrab_$name.log 2>&1 )
  local rc=$?
  echo "== $name rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/hdrab_$name.log) $(grep -o '"frac": [0-9.]*' gpurun_out/hdrab_$name.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/hdrab_$name.log)"
  [ $rc -ge 124 ] && exit $rc
  return 0
}
run base $L/libdts.so
run s1c256 $L/libdts_diag.so DTS_HDR_STREAMS=1 DTS_HDR_CHUNK=256
run s2c128 $L/libdts_diag.so DTS_HDR_STREAMS=2 DTS_HDR_CHUNK=128
run s2c64 $L/libdts_diag.so DTS_HDR_STREAMS=2 DTS_HDR_CHUNK=64
run s2c32 $L/libdts_diag.so DTS_HDR_STREAMS=2 DTS_HDR_CHUNK=32
run s1c64 $L/libdts_diag.so DTS_HDR_STREAMS=1 DTS_HDR_CHUNK=64
run s2c16 $L/libdts_diag.so DTS_HDR_STREAMS=2 DTS_HDR_CHUNK=16
exit 0
