#!/bin/bash
# round 5: k_ladder7 dispatch order, runs of luma-then-chroma over S frame octets (diagnostic
# DTS_L7_ORDER=3 DTS_L7_SUP=S, lib/libdts_diag.so) against order 1 (all luma first) and 0
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05o2
run() { # name env...
  local n=$1; shift
  env DTS_LIB=$PWD/distributed-transcoding-server_amd/lib/libdts_diag.so "$@" timeout -k 10 200 \
      python -u bench.py --workload ${WL:-cfg2} --steps 20 --warmup 3 --no-cpu > gpurun_out/r05o2/$n.log 2>&1 || exit 1
  echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/r05o2/$n.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/r05o2/$n.log)"
}
for rep in 1 2; do
  run o1 DTS_L7_ORDER=1
  run o0 DTS_L7_ORDER=0
  run s2 DTS_L7_ORDER=3 DTS_L7_SUP=2
  run s4 DTS_L7_ORDER=3 DTS_L7_SUP=4
  run s8 DTS_L7_ORDER=3 DTS_L7_SUP=8
  run s16 DTS_L7_ORDER=3 DTS_L7_SUP=16
done
