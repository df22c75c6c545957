#!/bin/bash
# k_ladder7 A/B: wait tree, heavy-wave priority, nt stores, group width, staging wave
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
./tools/ab7.sh base:: tree:tree: prio2:prio2: nt:nt: w7::DTS_L7_W=7 w9::DTS_L7_W=9 stg::DTS_L7_STAGER=1 base2:: || exit $?
exit 0
