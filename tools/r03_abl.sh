#!/bin/bash
# k_ladder7 ablations on cfg2 (diagnostic builds, wrong outputs except base): what each phase costs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_ARGS="--no-verify" ./tools/ab7.sh base:: abl2:abl2: abl4:abl4: abl8:abl8: abl16:abl16: base2:: || exit $?
exit 0
