#!/bin/bash
# round 5: k_ladder7 dispatch order (diagnostic DTS_L7_ORDER, lib/libdts_diag.so): 0 frame octets in
# plan order (the default), 1 luma groups first, 2 chroma groups first
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05o
for wl in ${WLS:-cfg2}; do
  for o in ${ORDERS:-0 1 2 0 1 2}; do
    DTS_LIB=$PWD/distributed-transcoding-server_amd/lib/libdts_diag.so DTS_L7_ORDER=$o timeout -k 10 200 \
        python -u bench.py --workload $wl --steps 20 --warmup 3 --no-cpu > gpurun_out/r05o/${wl}_o$o.log 2>&1 || exit 1
    echo "$wl order=$o $(grep -o '"value": [0-9.]*' gpurun_out/r05o/${wl}_o$o.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/r05o/${wl}_o$o.log)"
  done
done
