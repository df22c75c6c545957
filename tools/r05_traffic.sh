#!/bin/bash
# round 5: where k_ladder7's fetched bytes come from -- cfg2 line + FETCH_SIZE / WRITE_SIZE
# passes for lib/libdts.so and the ablation builds of tools/build_v7var.sh
# (usage: tools/r05_traffic.sh TAG suffix...; "" = lib/libdts.so).  Outputs are wrong in the
# ablation builds (--no-verify); the numbers are for attribution only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; shift
L=distributed-transcoding-server_amd/lib
mkdir -p gpurun_out/$tag
for v in "$@"; do
  n=${v:-base}
  lib=$PWD/$L/libdts${v:+_$v}.so
  B="python3 bench.py --workload cfg2 --steps 8 --warmup 2 --no-cpu --no-verify"
  DTS_LIB=$lib timeout -k 10 200 python3 -u bench.py --workload cfg2 --steps 20 --warmup 3 --no-cpu --no-verify > gpurun_out/$tag/${n}_line.log 2>&1 || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    DTS_LIB=$lib timeout -k 10 -s KILL 200 rocprofv3 --pmc $c -d gpurun_out/$tag/${n}_$c -o $c --output-format csv -- $B > gpurun_out/$tag/${n}_$c.log 2>&1 || exit $?
  done
  echo "== $n $(grep -o '"value": [0-9.]*' gpurun_out/$tag/${n}_line.log) $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/$tag/${n}_line.log)"
done
exit 0
