#!/bin/bash
# Diagnostic builds of libdts with k_quality knobs (api.cpp and kernels.hip rebuilt) ->
# lib/libdts_<name>.so, for tools/ab_libs.sh.  Args: name=DEFINES; name=@REV builds kernels.hip
# and dts_internal.h/api.cpp as of git revision REV.  Never used by tests or bench defaults.
set -e
cd "$(dirname "$0")/../distributed-transcoding-server_amd"
make -s lib/libdts.so
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-value -Wno-unused-result"
OBJS="build/filters.o build/plan5.o build/plan6.o build/ladder4.o build/ladder5.o build/ladder7.o build/hdr.o build/deint.o"
for a in "$@"; do
  n=${a%%=*}; d=${a#*=}
  if [ "${d:0:1}" = "@" ]; then
    tmp=$(mktemp -d); mkdir -p $tmp/x/csrc $tmp/include; cp ../include/dts.h $tmp/include/
    for f in kernels.hip api.cpp dts_internal.h; do git show ${d:1}:distributed-transcoding-server_amd/csrc/$f > $tmp/x/csrc/$f; done
    for f in csrc/*.h; do [ -f $tmp/x/$f ] || cp $f $tmp/x/$f; done
    /opt/rocm/bin/hipcc $F -c $tmp/x/csrc/kernels.hip -o build/kernels_$n.o
    /opt/rocm/bin/hipcc $F -x hip -c $tmp/x/csrc/api.cpp -o build/api_$n.o
    rm -rf $tmp
  else
    /opt/rocm/bin/hipcc $F $d -c csrc/kernels.hip -o build/kernels_$n.o
    /opt/rocm/bin/hipcc $F $d -x hip -c csrc/api.cpp -o build/api_$n.o
  fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libdts_$n.so build/api_$n.o build/kernels_$n.o $OBJS \
      -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libdts.so
done
