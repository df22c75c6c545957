#!/bin/bash
# round 5: SQ instruction / wait / LDS counters of one workload's kernels (two --pmc passes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; wl=$2; shift 2
B="python3 bench.py --workload $wl --steps 6 --warmup 2 --no-cpu --no-verify $*"
out=gpurun_out/prof_${tag}_$wl
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 -s KILL 200 rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- $B > $out/$name.log 2>&1
  local rc=$?; echo "  $wl/$name rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out/$name.log; exit $rc; }
  return 0
}
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
run sq2 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM
run sq3 --pmc SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32
exit 0
