#!/bin/bash
# stamp breakdown of the product build and of stamp ablations (tools/build_stamp5.sh N...)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${1:-r02x}; shift
for n in "" "$@"; do
  lib=libdts_stamp${n:+_b$n}.so
  STAMP_LIB=$lib timeout -k 10 120 python tools/stamp5.py > gpurun_out/s5_${tag}_$n.log 2>&1; rc=$?
  echo "== $lib rc=$rc"; tail -n 7 gpurun_out/s5_${tag}_$n.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
