#!/bin/bash
# Diagnostic builds of libdts with k_ladder7 knobs -> lib/libdts_<name>.so, for
# tools/ab_libs.sh.  Args: name=DEFINES.  Never used by tests or bench defaults.
set -e
cd "$(dirname "$0")/../distributed-transcoding-server_amd"
make -s lib/libdts.so
OBJS="build/api.o build/filters.o build/plan5.o build/plan6.o build/kernels.o build/ladder4.o build/ladder5.o build/hdr.o build/deint.o"
for a in "$@"; do
  n=${a%%=*}; d=${a#*=}
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm --amdgpu-mfma-vgpr-form $d -c csrc/ladder7.hip \
      -o build/ladder7_$n.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E " VGPRs:|Occupancy|Spill|Scratch" | sed "s/^.*remark: */$n: /" ) &
done
wait
for a in "$@"; do
  n=${a%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libdts_$n.so $OBJS build/ladder7_$n.o \
      -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libdts.so
done
