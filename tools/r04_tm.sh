#!/bin/bash
# round 4: k_tonemap occupancy variants (tools/build_tmvar.sh: tm5 = value-only tables + 5 waves per
# SIMD, tm5p = the same with the BT.709 OETF by v_log / v_exp): their HDR parity tests, then the
# cfg3 A/B against the default build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/distributed-transcoding-server_amd/lib
for v in tm5 tm5p; do
  DTS_LIB=$L/libdts_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_hdr.py "tests/test_gpu_bench_paths.py::test_cfg3_device_path_multi_chunk" > gpurun_out/tm_tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc $(tail -1 gpurun_out/tm_tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
AB_WORKLOADS=cfg3 bash tools/ab_libs.sh "" tm5 tm5p "" tm5 tm5p
