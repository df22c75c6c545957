#!/bin/bash
# rocprofv3 kernel-trace + stats pass over a short bench run of one workload.
# usage: tools/prof_kt.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-r01}; shift
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- \
    python3 bench.py --steps 4 --warmup 1 --no-cpu --no-verify "$@" > $out/kt.log 2>&1
rc=$?
echo "=== kt $tag rc=$rc"; tail -n 2 $out/kt.log
find $out -name "*kernel_stats.csv" -exec cp {} $out/${tag}_kernel_stats.csv \;
exit $rc
