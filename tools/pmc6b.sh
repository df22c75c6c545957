#!/bin/bash
# memory-path PMC passes (TCP / TCC / TA / TD) of the cfg2 bench for $KERNEL (default
# k_ladder6); per-launch averages.  usage: tools/pmc6b.sh <tag> [lib suffixes].  Diagnostic only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-m6}; shift
K=${KERNEL:-k_ladder6}
out=gpurun_out/pmcb_$tag
mkdir -p $out
P1="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_READ_sum"
P2="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT"
for v in "${@:-}"; do
  lib=$PWD/distributed-transcoding-server_amd/lib/libdts${v:+_$v}.so
  for i in 1 2; do
    eval C=\$P$i
    DTS_LIB=$lib timeout -k 10 -s KILL 90 rocprofv3 --pmc $C -d $out/${v:-base}_p$i -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify > $out/${v:-base}_p$i.log 2>&1
    rc=$?
    echo "${v:-base} pass $i rc=$rc"
    [ $rc -ne 0 ] && { tail -n 5 $out/${v:-base}_p$i.log; exit $rc; }
  done
done
python3 - "$out" "$K" <<'PY'
import csv, glob, os, sys, collections
out, K = sys.argv[1], sys.argv[2]
runs = sorted({os.path.basename(d).rsplit("_p", 1)[0] for d in glob.glob(out + "/*_p1")})
for n in runs:
    tot = collections.defaultdict(float); cnt = collections.Counter()
    for i in range(1, 3):
        for f in glob.glob(f"{out}/{n}_p{i}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if K in r["Kernel_Name"]:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    print(n, {k: f"{tot[k] / max(cnt[k], 1):.4g}" for k in sorted(tot)})
PY
