#!/bin/bash
# per-phase stamps of k_ladder7 (diagnostic build) + the base line on the same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/stamp7.py > gpurun_out/stamp7.log 2>&1; rc=$?
echo "stamp rc=$rc"; grep -v "^{" gpurun_out/stamp7.log | tail -60
[ $rc -ge 124 ] && exit $rc
./tools/ab7.sh base::
