#!/bin/bash
# round 5: k_tonemap_w parity (the HDR tests + the cfg3 bench path + the Node HDR10 job), then
# cfg3 lines for the column walk (lib/libdts.so) and the tiled kernel (diag build, DTS_TM_TILED=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-r05m}
mkdir -p gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_gpu_hdr.py tests/test_gpu_bench_paths.py tests/test_golden.py tests/test_node.py \
    -m gpu -x -q --timeout 200 --timeout-method thread -k "hdr or cfg3 or golden or tonemap" > gpurun_out/$tag/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$tag/tests.log; [ $rc -ne 0 ] && exit $rc
run() { # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --workload cfg3 --steps 10 --warmup 2 --no-cpu > gpurun_out/$tag/$n.log 2>&1 || exit $?
  echo "== $n $(grep -o '"value": [0-9.]*' gpurun_out/$tag/$n.log) $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/$tag/$n.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/$tag/$n.log)"
}
D=$PWD/distributed-transcoding-server_amd/lib/libdts_qsub.so
run walk X=1
run tiled DTS_LIB=$D DTS_TM_TILED=1
run walk2 X=1
run tiled2 DTS_LIB=$D DTS_TM_TILED=1
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/kt -o kt --output-format csv -- \
    python3 bench.py --workload cfg3 --steps 8 --warmup 2 --no-cpu --no-verify > gpurun_out/$tag/kt.log 2>&1 || exit $?
grep -h "tonemap\|ladder7" gpurun_out/$tag/kt/*kernel_stats.csv | cut -c1-200
exit 0
