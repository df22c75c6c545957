#!/bin/bash
# Diagnostic builds of libdts with k_yadif_t knobs -> lib/libdts_<name>.so, for
# tools/ab_libs.sh.  Args: name=DEFINES.  Never used by tests or bench defaults.
set -e
cd "$(dirname "$0")/../distributed-transcoding-server_amd"
make -s lib/libdts.so
OBJS="build/api.o build/filters.o build/plan5.o build/plan6.o build/kernels.o build/ladder4.o build/ladder5.o build/ladder7.o build/hdr.o"
for a in "$@"; do
  n=${a%%=*}; d=${a#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $d -c csrc/deint.hip -o build/deint_$n.o &
done
wait
for a in "$@"; do
  n=${a%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libdts_$n.so $OBJS build/deint_$n.o \
      -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libdts_$n.so
done
