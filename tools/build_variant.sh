#!/bin/bash
# A timing variant of libnvrx_hip.so for interleaved A/B (tools/ab_c3_pair.py, tools/ab_zipf.py):
# tools/ab_<name>/nvidia_resiliency_ext = a copy of the Python package whose library has
# segment_stats.hip (or the sources VARIANT_SRCS names) compiled with extra flags (build-time tuning constants); the other objects
# are the tree's.  Usage: tools/build_variant.sh <name> -DNAME=VALUE ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/nvidia-resiliency-ext-x_amd/csrc
name=$1; shift
D=$R/tools/ab_$name
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function"
rm -rf "$D" && mkdir -p "$D/obj" && cp -r "$R/nvidia-resiliency-ext-x_amd/nvidia_resiliency_ext" "$D/"
find "$D" -name __pycache__ -prune -exec rm -rf {} \;
cp "$C"/build/*.o "$D/obj/"
for src in ${VARIANT_SRCS:-segment_stats}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS "$@" -c "$C/$src.hip" -o "$D/obj/$src.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$D/nvidia_resiliency_ext/straggler/libnvrx_hip.so" "$D"/obj/*.o \
    -lamdhip64 -L/opt/rocm/lib -lrocprofiler-sdk -Wl,-rpath,/opt/rocm/lib
rm -rf "$D/obj"
