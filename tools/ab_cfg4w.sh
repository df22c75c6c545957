D=$PWD/distributed-transcoding-server_amd/lib/libdts_diag.so
for rep in 1 2; do
for w in 10 7 6 4; do
  DTS_L7_W=$w DTS_LIB=$D timeout -k 10 200 python -u bench.py --workload cfg4 --steps 10 --warmup 2 --no-cpu > gpurun_out/c4w$w.log 2>&1 || exit $?
  echo "cfg4 W=$w $(grep -o '"value": [0-9.]*' gpurun_out/c4w$w.log) $(grep -o '"frac": [0-9.]*' gpurun_out/c4w$w.log) $(grep -o '"verified_vs_oracle": [a-z]*' gpurun_out/c4w$w.log)"
done
done
