cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ladder.py > gpurun_out/t_ladder.log 2>&1; rc=$?; tail -n 2 gpurun_out/t_ladder.log; [ $rc -ne 0 ] && exit $rc
DTS_LIB=$PWD/distributed-transcoding-server_amd/lib/libdts_pair.so DTS_L7_NS=2 DTS_L7_PB=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ladder.py -k v7 > gpurun_out/t_pair.log 2>&1; rc=$?; tail -n 2 gpurun_out/t_pair.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab7.sh base:: pair:pair:DTS_L7_NS=2,DTS_L7_PB=2 base2:: pair2:pair:DTS_L7_NS=2,DTS_L7_PB=2
