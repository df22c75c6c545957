#!/bin/bash
# SQ instruction / wait counters of k_ladder5 per ablation build (tools/build_ablate5.sh):
# where the VALU / SALU / LDS instructions and the wave cycles go.  Diagnostic only.
# usage: tools/pmc_abl5.sh <tag> [ablation numbers, 0 = the product build]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-abl}; shift
V="${*:-0 1 2 4}"
out=gpurun_out/pmcabl_$tag
mkdir -p $out
for n in $V; do
  lib=$PWD/distributed-transcoding-server_amd/lib/libdts_b$n.so
  [ "$n" = 0 ] && lib=$PWD/distributed-transcoding-server_amd/lib/libdts.so
  for pass in 1 2; do
    if [ $pass = 1 ]; then C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
    else C="SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; fi
    DTS_LIB=$lib timeout -k 10 -s KILL 120 rocprofv3 --pmc $C -d $out/b${n}_p$pass -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify > $out/b${n}_p$pass.log 2>&1
    rc=$?
    echo "abl $n pass $pass rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
done
python3 - "$out" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(out + "/b*_p1")):
    n = os.path.basename(d)[:-3]
    tot = collections.defaultdict(float); cnt = collections.Counter()
    for p in (d, d[:-1] + "2"):
        for f in glob.glob(p + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_ladder5" in r["Kernel_Name"]:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    print(n, {k: f"{tot[k] / max(cnt[k], 1):.4g}" for k in sorted(tot)})
PY
