#!/bin/bash
# round 4: the whole GPU suite (incl. the temporal-walk yadif k_yadif_t and the worker's HDR10 /
# ffmpeg-boundary tests), the yadif line, a kernel trace and PMC passes of it
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 gpurun_out/r04_tests.log)"; [ $rc -ne 0 ] && { tail -40 gpurun_out/r04_tests.log; exit $rc; }
timeout -k 10 300 python -u bench.py --workload yadif --steps 20 --warmup 3 --no-cpu > gpurun_out/r04_yadif_line.log 2>&1
rc=$?; echo "yadif line rc=$rc"; grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"verified_vs_oracle": [a-z]*\|"kernel_ms_per_launch": [0-9.]*' gpurun_out/r04_yadif_line.log; [ $rc -ne 0 ] && { tail gpurun_out/r04_yadif_line.log; exit $rc; }
PROF_STEPS=8 bash tools/prof_wl.sh ${1:-r04a} yadif
