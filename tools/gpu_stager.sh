cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ladder.py -k v7 > gpurun_out/t_ladder.log 2>&1; rc=$?; tail -n 2 gpurun_out/t_ladder.log; [ $rc -ne 0 ] && exit $rc
DTS_L7_STAGER=1 DTS_L7_W=7 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ladder.py -k v7 > gpurun_out/t_st.log 2>&1; rc=$?; tail -n 2 gpurun_out/t_st.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab7.sh base:: st::DTS_L7_STAGER=1,DTS_L7_W=7 base2:: st2::DTS_L7_STAGER=1,DTS_L7_W=7
