#!/bin/bash
# A/B the k_ladder4 ablation builds (DTS_L4_ABLATE: 1 skip H, 2 skip V, 4 skip loads)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=distributed-transcoding-server_amd/lib
for v in libdts libdts_a1 libdts_a2 libdts_a3 libdts_a4 libdts_a5 libdts_a6 libdts_a7; do
  [ -f $L/$v.so ] || continue
  r=$(DTS_LIB=$PWD/$L/$v.so timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-verify 2>/dev/null | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['roofline']['kernel_ms_per_launch'])")
  rc=$?
  echo "$v $r"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
