#!/bin/bash
# cfg2 kernel time of each k_ladder5 ablation build (tools/build_ablate5.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
V="${*:-0 1 2 3 4 8 16 6}"
for n in $V; do
  lib=$PWD/distributed-transcoding-server_amd/lib/libdts_b$n.so
  [ "$n" = 0 ] && lib=$PWD/distributed-transcoding-server_amd/lib/libdts.so
  DTS_LIB=$lib timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/abl5_$n.log 2>&1
  rc=$?
  echo "ablate $n rc=$rc $(tail -n 1 gpurun_out/abl5_$n.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["roofline"]["kernel_ms_per_launch"])' 2>/dev/null)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
