#!/bin/bash
# round-end closing pass on ONE box from one build: the GPU suite + smoke, then for every workload
# the unprofiled line (with its CPU baseline), a rocprofv3 kernel trace and the FETCH / WRITE /
# GRBM passes (tools/prof_wl.sh; cfg2 also the SQ counters), then the host-path e2e line.
# usage: tools/final.sh TAG [workloads...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r05f}; shift
wls=${*:-cfg2 cfg1 cfg3 cfg4 cfg5 yadif cfg2nv12}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
  rc=$?; echo "gpu tests rc=$rc $(tail -1 gpurun_out/${tag}_tests.log)"; [ $rc -ge 124 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/${tag}_smoke.log)"; [ $rc -ge 124 ] && exit $rc
fi
for wl in $wls; do
  sq=""; [ $wl = cfg2 ] && sq=1
  SQ=$sq LINE=1 NOCPU=${NOCPU:-} bash tools/prof_wl.sh $tag $wl || exit $?
done
if [ -z "$SKIP_E2E" ]; then
  for m in "" "--e2e-pinned"; do
    n=${m:+_pinned}
    timeout -k 10 300 python -u bench.py --e2e --steps 6 --warmup 2 --e2e-submit 512 --e2e-batch 64 --e2e-frames 256 $m \
        > gpurun_out/${tag}_e2e$n.log 2>&1
    echo "e2e$n rc=$? $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_e2e$n.log)"
  done
fi
exit 0
