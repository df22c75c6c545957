#!/bin/bash
# k_ladder6 diagnostics: A/B of variant libs, per-phase stamps, MFMA PMC pass (diagnostic only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_libs.sh "" ${AB_LIBS:-} || exit $?
timeout -k 10 200 python -u tools/stamp6.py > gpurun_out/stamp6.log 2>&1 || exit $?
grep -v '^{' gpurun_out/stamp6.log | tail -n 40
K=k_ladder6
timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU SQ_WAVE_CYCLES -d gpurun_out/pmc_d3 -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify > gpurun_out/pmc_d3.log 2>&1 || exit $?
timeout -k 10 -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/pmc_d4 -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-verify > gpurun_out/pmc_d4.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
for d in ("pmc_d3", "pmc_d4"):
    tot = collections.defaultdict(float); cnt = collections.Counter()
    for f in glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_ladder6" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    print(d, {k: f"{tot[k] / max(cnt[k], 1):.4g}" for k in sorted(tot)})
PY
