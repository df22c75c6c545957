#!/bin/bash
# fragment / store-destination ablations on cfg2, cfg3 / cfg4 / cfg5 lines + profiles, then the
# per-phase stamps of k_ladder7 with and without the V stores (last: diagnostic process)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_ARGS="--no-verify" ./tools/ab7.sh base:: abl256:abl256: abl512:abl512: abl768:abl768: abl32:abl32: || exit $?
NOTESTS=1 bash tools/gpu_r03pass.sh r03a cfg3 cfg4 cfg5 || exit $?
for s in stamp7 stamp7a; do
  STAMP_LIB=libdts_$s.so timeout -k 10 240 python -u tools/stamp7.py > gpurun_out/$s.log 2>&1; rc=$?
  echo "$s rc=$rc"; grep -v "^{" gpurun_out/$s.log | grep -v amdgpu.ids | head -60
  [ $rc -ne 0 ] && exit $rc
done
exit 0
