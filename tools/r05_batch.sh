#!/bin/bash
# round 5: cfg2 frames per launch (the launch tail) -- 512 (the line) against 768 / 1024
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05b
for b in ${BATCHES:-512 1024 768 512 1024 768}; do
  timeout -k 10 200 python -u bench.py --workload cfg2 --batch $b --steps 20 --warmup 3 --no-cpu > gpurun_out/r05b/b$b.log 2>&1 || exit 1
  echo "batch=$b $(grep -o '"value": [0-9.]*' gpurun_out/r05b/b$b.log) $(grep -o '"frac": [0-9.]*' gpurun_out/r05b/b$b.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/r05b/b$b.log)"
done
