#!/bin/bash
# Diagnostic builds of libdts with k_ladder5 ablations (DTS_L5_ABLATE bits:
# 1 skip H, 2 skip V, 4 skip source loads, 8 skip V stores, 16 skip the H
# epilogue) -> lib/libdts_b<N>.so, for tools/ablate5.sh.  Never used by
# tests or bench defaults.
set -e
cd "$(dirname "$0")/../distributed-transcoding-server_amd"
make -s lib/libdts.so
V="${*:-1 2 3 4 8 16 6}"
for n in $V; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DDTS_L5_ABLATE=$n -c csrc/ladder5.hip -o build/ladder5_b$n.o &
done
wait
for n in $V; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libdts_b$n.so build/api.o build/filters.o build/plan5.o build/kernels.o build/ladder4.o build/ladder5_b$n.o build/hdr.o build/deint.o -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libdts.so
done
