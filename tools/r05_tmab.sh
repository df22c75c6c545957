#!/bin/bash
# round 5: k_tonemap_w knob A/B on cfg3 (tools/build_tmvar.sh libraries), parity of each first
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-r05n}; shift
mkdir -p gpurun_out/$tag
L=$PWD/distributed-transcoding-server_amd/lib
for v in "$@"; do
  lib=$L/libdts${v:+_$v}.so
  DTS_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_hdr.py tests/test_gpu_bench_paths.py -m gpu -x -q \
      --timeout 200 --timeout-method thread -k "hdr or cfg3 or tonemap" > gpurun_out/$tag/t_${v:-base}.log 2>&1 || { tail -20 gpurun_out/$tag/t_${v:-base}.log; exit 1; }
  DTS_LIB=$lib timeout -k 10 300 python3 -u bench.py --workload cfg3 --steps 10 --warmup 2 --no-cpu > gpurun_out/$tag/${v:-base}.log 2>&1 || exit $?
  echo "== ${v:-base} $(tail -1 gpurun_out/$tag/t_${v:-base}.log) $(grep -o '"value": [0-9.]*' gpurun_out/$tag/${v:-base}.log) $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/$tag/${v:-base}.log)"
done
exit 0
