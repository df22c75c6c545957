#!/bin/bash
# k_ladder7 V-phase sub-ablations on cfg2 (diagnostic builds, wrong outputs except base)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_ARGS="--no-verify" ./tools/ab7.sh base:: abl32:abl32: abl64:abl64: abl128:abl128: abl192:abl192: abl8:abl8: || exit $?
exit 0
