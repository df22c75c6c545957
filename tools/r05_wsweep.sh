#!/bin/bash
# round 5: group width per workload (diagnostic DTS_L7_W, lib/libdts_diag.so), two rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05ws
for wl in ${WLS:-cfg4 cfg1 cfg5}; do
  for w in ${WIDTHS:-8 6 10 12 8 6 10 12}; do
    DTS_LIB=$PWD/distributed-transcoding-server_amd/lib/libdts_diag.so DTS_L7_W=$w timeout -k 10 200 \
        python -u bench.py --workload $wl --steps 15 --warmup 3 --no-cpu > gpurun_out/r05ws/${wl}_w$w.log 2>&1 || exit 1
    echo "$wl W=$w $(grep -o '"value": [0-9.]*' gpurun_out/r05ws/${wl}_w$w.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/r05ws/${wl}_w$w.log)"
  done
done
