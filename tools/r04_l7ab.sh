#!/bin/bash
# round 4: k_ladder7 A/B builds on cfg2 (tools/build_v7var.sh: u4 = unroll by the ring length,
# nt = non-temporal row stores, aux1 = sc0 staging loads, roll = one
# staging batch per loop copy with a switch-selected ring slot), then instruction-cache PMC passes of
# base, u4 and roll (one SQ pass each: 8 SQ counters)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_libs.sh "" u4 roll nt aux1 "" u4 roll || exit $?
L=$PWD/distributed-transcoding-server_amd/lib
for v in base u4 roll; do
  lib=$L/libdts.so; [ $v != base ] && lib=$L/libdts_$v.so
  DTS_LIB=$lib timeout -k 10 -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
    -d gpurun_out/l7pmc_$v -o pmc --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-verify > gpurun_out/l7pmc_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/l7pmc_$v.log; exit $rc; }
done
exit 0
