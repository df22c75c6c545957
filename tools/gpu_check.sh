#!/bin/bash
# One GPU-box session: warm torch, parity tests, smoke, short bench.
# Stops at the first step that ends with a signal / timeout / abort
# (exit >= 124 or a negative python status); plain test failures (exit 1)
# do not stop the later steps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping after $name (rc=$rc)"; exit $rc
  fi
  return 0
}
step warm 240 python -c "import torch; print(torch.__version__, torch.cuda.is_available(), torch.cuda.get_device_name(0))"
for s in "$@"; do
  case $s in
    tests)  step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    quick)  step tests_quick 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "small or quality or identity or device_path" ;;
    all)    step tests_all 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 300 python -u bench.py --steps 20 --warmup 3 ;;
    bench:*) wl=${s#bench:}; step bench_$wl 300 python -u bench.py --steps 10 --warmup 2 --workload $wl --no-cpu ;;
    benchq) step benchq 300 python -u bench.py --steps 20 --warmup 3 --no-cpu ;;
    benchv3) DTS_LADDER=3 step benchv3 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-verify ;;
    benchw4) DTS_LIB=$PWD/distributed-transcoding-server_amd/lib/libdts_w4.so step benchw4 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-verify ;;
    probe)  step probe 60 ./tools/probe_mfma_i8 ;;
    new)    step tests_new 600 python -u -m pytest tests/test_gpu_configs.py tests/test_node.py -m gpu -v --timeout 300 --timeout-method thread ;;
    v5small) step v5small 180 python -u -m pytest tests/test_gpu_ladder.py -x -v --timeout 60 --timeout-method thread -k "v5 and (small or identity)" ;;
    v5all)  step v5all 600 python -u -m pytest tests/test_gpu_ladder.py tests/test_gpu_configs.py tests/test_golden.py -v --timeout 120 --timeout-method thread -m gpu -k "v5 or configs or golden" ;;
    v4small) step v4small 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "v4 and (small or 4k_one)" ;;
    *) echo "unknown step $s" ;;
  esac
done
