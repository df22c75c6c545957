#!/bin/bash
# SQ counters of the kernels in $PMC_KERNELS on the $PMC_WL bench line (default: k_tonemap / k_ladder4 on cfg3; diagnostic only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
WL=${PMC_WL:-cfg3}; KS=${PMC_KERNELS:-k_tonemap k_ladder4}
out=gpurun_out/pmc_tm_$WL; mkdir -p $out
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
for i in 1 2; do eval C=\$P$i
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $C -d $out/p$i -o p --output-format csv -- python3 bench.py --workload $WL --steps 3 --warmup 1 --no-cpu --no-verify > $out/p$i.log 2>&1 || exit 1
done
KS="$KS" OUT=$out python3 - <<'PY'
import csv, glob, collections, os
for K in os.environ["KS"].split():
    tot = collections.defaultdict(float); cnt = collections.Counter()
    for f in glob.glob(os.environ["OUT"] + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if K in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    print(K, {k: f"{tot[k] / max(cnt[k], 1):.3g}" for k in sorted(tot)})
PY
