#!/bin/bash
# r03 first pass: the new parity tests (cfg5 segments, default-tonemap cfg3, golden),
# then the k_ladder7 no-halo ablation A/B, the rocprofv3 counter list and the L2
# hit / miss counters of k_ladder7.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 12 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "=== stop ($rc)"; exit $rc; fi
  return 0
}
step warm 240 python -c "import torch; print(torch.__version__, torch.cuda.is_available())"
step t_new 600 python -u -m pytest tests/test_gpu_cfg5.py tests/test_golden.py tests/test_gpu_hdr.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cfg5 or golden or 4k or params"
./tools/ab7.sh base:: own:own: || exit $?
step counters 60 rocprofv3 -L
L=distributed-transcoding-server_amd/lib
step tcc 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/tcc -o tcc --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-verify
exit 0
