#!/bin/bash
# bench.py at several batch sizes (frames per ladder launch), kernel-only
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for B in "$@"; do
  R=$((B * 2)); [ $R -lt 96 ] && R=96
  timeout -k 5 200 python -u bench.py --steps 10 --warmup 2 --batch $B --ring $R --no-cpu --no-verify > gpurun_out/bs_$B.json 2>gpurun_out/bs_$B.err || { echo "B=$B failed"; tail -3 gpurun_out/bs_$B.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/bs_$B.json')); print('B=$B', j['value'], j['roofline']['kernel_ms_per_launch'], j['roofline']['frac'])"
done
