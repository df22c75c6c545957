#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace/stats, then separate
# PMC passes (gpurun: never combine --pmc with tracing domains).
# usage: tools/profile.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-r01}; shift
B="python3 bench.py --steps 4 --warmup 1 --no-cpu --no-verify $*"
out=gpurun_out/prof_$tag
mkdir -p $out
run() {  # name, rocprof args...
  local name=$1; shift
  echo "=== $name ($(date +%T))"
  timeout -k 10 -s KILL 240 rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- $B > $out/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 $out/$name.log
  if [ $rc -ge 124 ]; then echo "stop"; exit $rc; fi
}
run kt --kernel-trace --stats
run pmc_sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
run pmc_sq2 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT
find $out -name "*.csv" | head -30
