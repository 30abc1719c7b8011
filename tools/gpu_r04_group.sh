#!/bin/bash
# configs[1] statistics kernel (64 x 2048 x 10,000 pushed, 8192 kept): segments per wave of the
# group kernel, build variants tools/ab_g<k> (k segments per wave; the library: 4) interleaved
# three times on one box.  Output: gpurun_out/r04_group/ab.log
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r04_group
mkdir -p "$OUT"
cd "$R"
: > "$OUT/ab.log"
for round in 1 2 3; do
  for v in tree g2 g3 g5 g6 g8; do
    if [ $v = tree ]; then PKG=$R/nvidia-resiliency-ext-x_amd; else PKG=$R/tools/ab_$v; fi
    AB_R=64 AB_S=10000 timeout -k 10 120 python3 tools/ab_c3_pair.py $PKG 50 >> "$OUT/ab.log" 2> "$OUT/err_$v.log" || { echo "fail $v"; tail -3 "$OUT/err_$v.log"; exit 1; }
    tail -1 "$OUT/ab.log"
  done
done
