#!/bin/bash
# A/B of the stats library against a variant build (csrc/build_<name>/libnvrx_hip.so) on
# C3 (4096 x 2048 x 1024) and C2 (64 x 2048 x 10000, cap 8192).  Usage: ab_variant.sh name
set -e
V=$1
LIB=nvidia-resiliency-ext-x_amd/nvidia_resiliency_ext/straggler/libnvrx_hip.so
cp $LIB /tmp/base.so
for rep in 1 2; do
  for which in base $V; do
    if [ $which = base ]; then cp /tmp/base.so $LIB; else cp nvidia-resiliency-ext-x_amd/csrc/build_$V/libnvrx_hip.so $LIB; fi
    echo -n "$which: "; timeout -k 10 120 python tools/ab_c3.py 10 2>/dev/null | tail -1
    echo -n "$which: "; AB_R=64 AB_S=10000 timeout -k 10 120 python tools/ab_c3.py 20 2>/dev/null | tail -1
  done
done
cp /tmp/base.so $LIB
