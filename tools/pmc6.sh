#!/bin/bash
# PMC passes of the cfg2 bench (one rocprofv3 --pmc run per pass, no tracing) for
# the kernel named by $KERNEL (default k_ladder7); per-launch averages printed.
# usage: tools/pmc6.sh <tag> [lib suffixes; "" = lib/libdts.so].  Diagnostic only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-p6}; shift
K=${KERNEL:-k_ladder7}
out=gpurun_out/pmc_$tag
mkdir -p $out
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_IFETCH"
P3="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_FLAT"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
for v in "${@:-}"; do
  lib=$PWD/distributed-transcoding-server_amd/lib/libdts${v:+_$v}.so
  for i in 1 2 3 4 5; do
    eval C=\$P$i
    DTS_LIB=$lib timeout -k 10 -s KILL 90 rocprofv3 --pmc $C -d $out/${v:-base}_p$i -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify > $out/${v:-base}_p$i.log 2>&1
    rc=$?
    echo "${v:-base} pass $i rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
done
python3 - "$out" "$K" <<'PY'
import csv, glob, os, sys, collections
out, K = sys.argv[1], sys.argv[2]
runs = sorted({os.path.basename(d).rsplit("_p", 1)[0] for d in glob.glob(out + "/*_p1")})
for n in runs:
    tot = collections.defaultdict(float); cnt = collections.Counter()
    for i in range(1, 6):
        for f in glob.glob(f"{out}/{n}_p{i}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if K in r["Kernel_Name"]:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    print(n, {k: f"{tot[k] / max(cnt[k], 1):.4g}" for k in sorted(tot)})
PY
