#!/bin/bash
# Diagnostic build: k_ladder5 with per-phase s_memtime sums -> lib/libdts_stamp.so (tools/stamp5.py)
set -e
cd "$(dirname "$0")/../distributed-transcoding-server_amd"
make -s lib/libdts.so
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -DDTS_L5_STAMP=1"
/opt/rocm/bin/hipcc $F -c csrc/ladder5.hip -o build/ladder5_stamp.o &
/opt/rocm/bin/hipcc $F -x hip -c csrc/api.cpp -o build/api_stamp.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libdts_stamp.so build/api_stamp.o build/filters.o build/plan5.o build/kernels.o build/ladder4.o build/ladder5_stamp.o build/hdr.o build/deint.o -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libdts.so
