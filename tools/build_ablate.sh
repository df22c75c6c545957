#!/bin/bash
# Diagnostic builds of libdts with k_ladder4 ablations (DTS_L4_ABLATE bits:
# 1 skip H, 2 skip V, 4 skip source loads) -> lib/libdts_a<N>.so, for
# tools/ablate4.sh.  Never used by tests or bench defaults.
set -e
cd "$(dirname "$0")/../distributed-transcoding-server_amd"
make -s lib/libdts.so
for n in 1 2 3 4 5 6 7; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DDTS_L4_ABLATE=$n -c csrc/ladder4.hip -o build/ladder4_a$n.o &
done
wait
for n in 1 2 3 4 5 6 7; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libdts_a$n.so build/api.o build/filters.o build/kernels.o build/ladder4_a$n.o build/hdr.o build/deint.o -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libdts.so
done
ls -la lib/
