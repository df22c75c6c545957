#!/bin/bash
# Diagnostic build: k_ladder5 with per-phase s_memtime sums -> lib/libdts_stamp.so (tools/stamp5.py);
# with an argument N, also the ablation N (DTS_L5_ABLATE) -> lib/libdts_stamp_bN.so
set -e
cd "$(dirname "$0")/../distributed-transcoding-server_amd"
make -s lib/libdts.so
build() {  # suffix, extra flags
  local F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -DDTS_L5_STAMP=1 $2"
  /opt/rocm/bin/hipcc $F -c csrc/ladder5.hip -o build/ladder5_stamp$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libdts_stamp$1.so build/api_stamp.o build/filters.o build/plan5.o build/kernels.o build/ladder4.o build/ladder5_stamp$1.o build/hdr.o build/deint.o -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libdts.so
}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DDTS_L5_STAMP=1 -x hip -c csrc/api.cpp -o build/api_stamp.o
build "" ""
for n in "$@"; do build _b$n "-DDTS_L5_ABLATE=$n"; done
