#!/bin/bash
# round 5: cfg5 with the ladder + quality passes per sub-batch (diagnostic DTS_Q_SUB, diag build
# lib/libdts_qsub.so) against the whole-segment order: the line, then FETCH / WRITE of the best
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-r05q}
mkdir -p gpurun_out/$tag
lib=$PWD/distributed-transcoding-server_amd/lib/libdts_qsub.so
for n in ${SUBS:-0 600 300 100 48 24}; do
  DTS_LIB=$lib DTS_Q_SUB=$n timeout -k 10 300 python3 -u bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu > gpurun_out/$tag/sub$n.log 2>&1 || exit $?
  echo "== sub $n $(grep -o '"value": [0-9.]*' gpurun_out/$tag/sub$n.log) $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/$tag/sub$n.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/$tag/sub$n.log)"
done
for n in ${PMC_SUBS:-0 48}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    DTS_LIB=$lib DTS_Q_SUB=$n timeout -k 10 -s KILL 200 rocprofv3 --pmc $c -d gpurun_out/$tag/sub${n}_$c -o $c --output-format csv -- \
      python3 bench.py --workload cfg5 --steps 4 --warmup 1 --no-cpu --no-verify > gpurun_out/$tag/sub${n}_$c.log 2>&1 || exit $?
  done
done
exit 0
