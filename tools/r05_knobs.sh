#!/bin/bash
# round 5: k_ladder7 plan knobs re-measured after the dispatch order (diagnostic lib/libdts_diag.so):
# per-rendition groups (DTS_L7_GROUP=r), narrow one-K-block walks (DTS_L7_NARROW=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05k
run() { local n=$1; shift
  env DTS_LIB=$PWD/distributed-transcoding-server_amd/lib/libdts_diag.so "$@" timeout -k 10 200 \
      python -u bench.py --workload cfg2 --steps 20 --warmup 3 --no-cpu > gpurun_out/r05k/$n.log 2>&1 || exit 1
  echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/r05k/$n.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/r05k/$n.log)"
}
for rep in 1 2; do
  run base DTS_L7_ORDER=1
  run byrung DTS_L7_GROUP=r
  run narrow DTS_L7_NARROW=1
done
