#!/bin/bash
# Host code under AddressSanitizer + UBSan: the C-ABI's host objects (api, filters, planners)
# rebuilt with -fsanitize on the host side only (the device code is the ordinary build), linked
# into tools/asan_host (asan_host.cpp) and run here -- no GPU, no LD_PRELOAD (the executable
# carries the runtime).  Usage: tools/asan_host.sh
set -e
cd "$(dirname "$0")/../distributed-transcoding-server_amd"
make -s lib/libdts.so
B=build/asan; mkdir -p $B
F="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Xarch_host -fsanitize=address,undefined -Xarch_host -fno-omit-frame-pointer"
for f in api filters plan5 plan6; do
  /opt/rocm/bin/hipcc $F -x hip -c csrc/$f.cpp -o $B/$f.o
done
/opt/rocm/bin/hipcc $F -x hip -c ../tools/asan_host.cpp -o $B/asan_host.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fsanitize=address,undefined -pthread -o ../tools/asan_host $B/asan_host.o \
    $B/api.o $B/filters.o $B/plan5.o $B/plan6.o build/kernels.o build/ladder4.o build/ladder5.o build/ladder7.o \
    build/hdr.o build/deint.o -Wl,-rpath,/opt/rocm/lib
cd .. && ASAN_OPTIONS=detect_leaks=1:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 ./tools/asan_host
