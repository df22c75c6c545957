#!/bin/bash
# k_quality variants by kernel time: rocprofv3 kernel traces of cfg5 and cfg4 for each build
# (base = walking k_quality, oldq = one tile per workgroup, np4 / np8 = no prefetch, walks of 4 / 8,
# w8 = walks of 8), then the quality tests on the base build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=$PWD/distributed-transcoding-server_amd/lib
for v in ${Q5_VARS:-base oldq np4 np8 w8}; do
  lib=$L/libdts.so; [ $v != base ] && lib=$L/libdts_$v.so
  for wl in cfg5 cfg4; do
    DTS_LIB=$lib bash tools/prof_kt.sh q5_${v}_$wl --workload $wl > /dev/null 2>&1 || { echo "$v $wl failed"; exit 1; }
    python3 - gpurun_out/prof_q5_${v}_$wl/q5_${v}_${wl}_kernel_stats.csv $v $wl <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_quality' in r['Name'] or 'k_ladder7' in r['Name']:
        print(sys.argv[2], sys.argv[3], r['Name'][:40], r['Calls'], round(float(r['TotalDurationNs']) / 1e6, 3))
PY
  done
done
[ -n "$Q5_TESTS" ] || exit 0
timeout -k 10 400 python -u -m pytest tests/test_gpu_quality.py tests/test_gpu_qfuse.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/q5_tests.log; exit $rc
