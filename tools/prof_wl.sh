#!/bin/bash
# Per-workload rocprofv3 passes on ONE box, from one build:
#   kt     kernel trace + stats over a bench run that prints its own line (the line and the
#          trace come from the same process and clock);
#   fetch  --pmc FETCH_SIZE;  write --pmc WRITE_SIZE;  grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT
#   (one counter group per pass: gpurun never combines --pmc with tracing);
#   sq1/sq2 (with SQ=1) the SQ instruction / wait counters.
# Then tools/prof_wl.py condenses them into profiles/<tag>_<wl>.json.
# usage: tools/prof_wl.sh <tag> <workload> [extra bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; wl=$2; shift 2
steps=${PROF_STEPS:-8}; warm=${PROF_WARM:-2}
B="python3 bench.py --workload $wl --steps $steps --warmup $warm --no-cpu --no-verify $*"
out=gpurun_out/prof_${tag}_$wl
mkdir -p $out
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 -s KILL 200 rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- $B > $out/$name.log 2>&1
  local rc=$?
  echo "  $wl/$name rc=$rc $(grep -o '"value": [0-9.]*' $out/$name.log | head -1)"
  if [ $rc -ne 0 ]; then echo "stop ($wl/$name)"; tail -5 $out/$name.log; exit $rc; fi
}
if [ -n "$LINE" ]; then   # the unprofiled line first (with the CPU baseline unless NOCPU)
  cpu="--cpu-seconds 10"; [ -n "$NOCPU" ] && cpu="--no-cpu"
  timeout -k 10 400 python3 -u bench.py --workload $wl $cpu $* > $out/line.log 2>&1
  rc=$?
  echo "  $wl/line rc=$rc $(grep -o '"value": [0-9.]*' $out/line.log | head -1) $(grep -o '"frac": [0-9.]*' $out/line.log) $(grep -o '"verified_vs_oracle": [a-z]*' $out/line.log)"
  if [ $rc -ne 0 ]; then echo "stop ($wl/line)"; tail -5 $out/line.log; exit $rc; fi
fi
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT
if [ -n "$SQ" ]; then
  run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
  run sq2 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM
fi
exit 0
