#!/bin/bash
# round 5: cfg4's launch shape -- frames per launch (64 = the line, 150, 300 = one 10 s 8K30 segment)
# x group width (diagnostic DTS_L7_W 8 / 10, lib/libdts_diag.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05c4
for b in ${BATCHES:-64 150 300}; do
  for w in ${WIDTHS:-8 10}; do
    DTS_LIB=$PWD/distributed-transcoding-server_amd/lib/libdts_diag.so DTS_L7_W=$w timeout -k 10 300 \
        python -u bench.py --workload cfg4 --batch $b --ring $((b > 96 ? b : 96)) --steps 10 --warmup 2 --no-cpu \
        > gpurun_out/r05c4/b${b}_w$w.log 2>&1 || { tail -3 gpurun_out/r05c4/b${b}_w$w.log; exit 1; }
    echo "cfg4 batch=$b W=$w $(grep -o '"value": [0-9.]*' gpurun_out/r05c4/b${b}_w$w.log) $(grep -o '"frac": [0-9.]*' gpurun_out/r05c4/b${b}_w$w.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/r05c4/b${b}_w$w.log)"
  done
done
