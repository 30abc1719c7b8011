#!/bin/bash
# Same-box comparison: configs[2] read ceiling (tools/mb_c2), configs[2] statistics kernel and
# configs[3] record statistics, saved library (tools/ab_pkg) vs the tree's, interleaved.
# Output: gpurun_out/r03_c2c3/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_c2c3
mkdir -p "$OUT"
cd "$R"
timeout -k 10 120 tools/build/mb_c2 > "$OUT/mb_c2.log" 2>&1 || exit 1
cat "$OUT/mb_c2.log"
for i in 1 2 3; do
  timeout -k 5 120 python3 tools/ab_c3_pair.py "$R/tools/ab_pkg" 10 2>&1 | grep ms= || exit 1
  timeout -k 5 120 python3 tools/ab_c3_pair.py "$R/nvidia-resiliency-ext-x_amd" 10 2>&1 | grep ms= || exit 1
done | tee "$OUT/ab_c2.log"
for i in 1 2 3; do
  AB_PKG=$R/tools/ab_pkg timeout -k 5 180 python3 tools/ab_zipf.py 10 2>&1 | grep records_stats_ms || exit 1
  timeout -k 5 180 python3 tools/ab_zipf.py 10 2>&1 | grep records_stats_ms || exit 1
done | tee "$OUT/ab_c3.log"
