#!/bin/bash
# A/B the ladder builds in one box session: default lib + build_ablate/<name> variants.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
B=${BATCH:-120}
for a in base "$@"; do
  if [ $a = base ]; then L=; else L=build_ablate/$a/libdts.so; fi
  DTS_LIB=$L timeout -k 5 200 python -u bench.py --steps 10 --warmup 2 --batch $B --ring 240 --no-cpu --no-verify > gpurun_out/ab_$a.json 2>gpurun_out/ab_$a.err || { echo "$a failed"; tail -3 gpurun_out/ab_$a.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/ab_$a.json')); print('$a', j['value'], j['roofline']['kernel_ms_per_launch'])"
done
