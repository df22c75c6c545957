#!/bin/bash
# Round-2 re-entry GPU pass: every gpu test, smoke, cfg2 bench line, kernel trace + PMC
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/b_cfg2.log 2>&1 || exit $?
tail -n 1 gpurun_out/b_cfg2.log
bash tools/profile.sh ${1:-r02b}
