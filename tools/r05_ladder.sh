#!/bin/bash
# round 5: ladder parity (k_ladder7 suite + the bench paths), the cfg2 line, then the cfg2
# kernel trace / FETCH / WRITE passes (tools/prof_wl.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05a}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ladder.py tests/test_gpu_bench_paths.py tests/test_golden.py \
    tests/test_gpu_hdr.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
for wl in ${WLS:-cfg2}; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 3 --no-cpu > gpurun_out/${tag}_bench_$wl.log 2>&1
  rc=$?; echo "bench $wl rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bench_$wl.log) $(grep -o '"frac": [0-9.]*' gpurun_out/${tag}_bench_$wl.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/${tag}_bench_$wl.log)"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/${tag}_bench_$wl.log; exit $rc; }
done
if [ -n "$PROF" ]; then
  for wl in $PROF; do bash tools/prof_wl.sh $tag $wl || exit $?; done
fi
exit 0
