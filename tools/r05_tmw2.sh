#!/bin/bash
# round 5: k_tonemap_w with buffer addressing + carried chroma -- HDR parity, then cfg3 A/B against
# the previous walk (lib/libdts_tmold.so) and a kernel trace of the new one
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05t2
timeout -k 10 300 python -u -m pytest tests/test_gpu_hdr.py tests/test_gpu_bench_paths.py -m gpu -q -k "hdr or cfg3 or tonemap or p010" \
    --timeout 150 --timeout-method thread > gpurun_out/r05t2/tests.log 2>&1
rc=$?; echo "hdr tests rc=$rc $(tail -1 gpurun_out/r05t2/tests.log)"; [ $rc -ne 0 ] && exit $rc
AB_WORKLOADS=cfg3 bash tools/ab_libs.sh ${AB_LIBS:-base} || exit 1
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05t2/kt -o kt --output-format csv -- \
    python3 bench.py --workload cfg3 --steps 8 --warmup 2 --no-cpu --no-verify > gpurun_out/r05t2/kt.log 2>&1
echo "kt rc=$?"
grep -h tonemap gpurun_out/r05t2/kt/kt_kernel_stats.csv | cut -c1-200
exit 0
