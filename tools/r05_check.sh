#!/bin/bash
# round 5: the whole GPU suite + smoke, then the lines of the given workloads (unprofiled)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-r05c}; shift
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 gpurun_out/$tag/tests.log)"; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/$tag/tests.log | head -5; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/$tag/smoke.log)"; [ $rc -ne 0 ] && exit $rc
for wl in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu > gpurun_out/$tag/line_$wl.log 2>&1
  rc=$?; echo "$wl rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/$tag/line_$wl.log) $(grep -o '"frac": [0-9.]*' gpurun_out/$tag/line_$wl.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/$tag/line_$wl.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
