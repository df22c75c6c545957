#!/bin/bash
# round 5: cfg3's p010 ladder at other group widths (diagnostic DTS_L7_W, lib/libdts_diag.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05w3
for w in ${WIDTHS:-8 12 16 8 12 16}; do
  DTS_LIB=$PWD/distributed-transcoding-server_amd/lib/libdts_diag.so DTS_L7_W=$w timeout -k 10 200 \
      python -u bench.py --workload ${WL:-cfg3} --steps 20 --warmup 3 --no-cpu > gpurun_out/r05w3/w$w.log 2>&1 || exit 1
  echo "W=$w $(grep -o '"value": [0-9.]*' gpurun_out/r05w3/w$w.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/r05w3/w$w.log)"
done
