#!/bin/bash
# cfg5 kernel traces of the XCD-paired U/V k_quality build and the previous one (lib/libdts_oldq.so),
# then the A/B lines in the other order
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/prof_kt.sh q3new --workload cfg5 || exit $?
DTS_LIB=$PWD/distributed-transcoding-server_amd/lib/libdts_oldq.so bash tools/prof_kt.sh q3old --workload cfg5 || exit $?
for tg in q3new q3old; do echo "== $tg"; grep -E "k_quality|k_qreduce|k_ladder7" gpurun_out/prof_$tg/${tg}_kernel_stats.csv | cut -d, -f1-4; done
AB_WORKLOADS="cfg5" bash tools/ab_libs.sh oldq ""
