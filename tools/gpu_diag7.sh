#!/bin/bash
# k_ladder7 diagnostics: per-phase stamps, PMC passes (diagnostic only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/stamp7.py > gpurun_out/stamp7.log 2>&1 || exit $?
grep -v '^{' gpurun_out/stamp7.log | tail -n 60
KERNEL=k_ladder7 bash tools/pmc6.sh ${1:-p7} || exit $?
timeout -k 10 -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d gpurun_out/pmc7_tcc -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify > gpurun_out/pmc7_tcc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob("gpurun_out/pmc7_tcc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_ladder7" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
print("tcc", {k: f"{tot[k] / max(cnt[k], 1):.4g}" for k in sorted(tot)})
PY
