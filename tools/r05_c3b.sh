#!/bin/bash
# round 5: cfg3 frames per launch (256 = the line, 600 = one 10 s 4K60 segment)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05c3b
for b in 256 600 256 600; do
  timeout -k 10 300 python -u bench.py --workload cfg3 --batch $b --steps 10 --warmup 2 --no-cpu > gpurun_out/r05c3b/b$b.log 2>&1 || { tail -3 gpurun_out/r05c3b/b$b.log; exit 1; }
  echo "cfg3 batch=$b $(grep -o '"value": [0-9.]*' gpurun_out/r05c3b/b$b.log) $(grep -o '"frac": [0-9.]*' gpurun_out/r05c3b/b$b.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/r05c3b/b$b.log)"
done
