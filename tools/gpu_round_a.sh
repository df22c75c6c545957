cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_yadif.py tests/test_gpu_hdr.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_yadif.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 4 gpurun_out/t_yadif.log
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
bash tools/ab_libs.sh "" hs hs4 hsv hsv4
