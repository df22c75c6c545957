#!/bin/bash
# Diagnostic build: k_ladder7 with per-variant, per-phase s_memtime sums -> lib/libdts_stamp7.so
# (tools/stamp7.py); extra args = extra hipcc defines for the kernel.  Never used by tests or bench defaults.
set -e
cd "$(dirname "$0")/../distributed-transcoding-server_amd"
make -s lib/libdts.so
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DDTS_L7_STAMP=1 -x hip -c csrc/api.cpp -o build/api_stamp7.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm --amdgpu-mfma-vgpr-form -DDTS_L7_STAMP=1 "$@" \
    -c csrc/ladder7.hip -o build/ladder7_stamp.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libdts_stamp7.so build/api_stamp7.o build/filters.o \
    build/plan5.o build/plan6.o build/kernels.o build/ladder4.o build/ladder5.o build/ladder7_stamp.o \
    build/hdr.o build/deint.o -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libdts.so
