#!/bin/bash
# configs[3] record statistics, interleaved A/B of package roots (tools/ab_<v>, built by
# tools/build_variant.sh) against the tree: VARIANTS="c4 w8 ..." (default below), ROUNDS rounds.
# The first round dumps every variant's statistics and checks them against the tree's
# (tools/ab_compare.py: NUM/MIN/MAX/MED bits, AVG/STD).  Output: gpurun_out/r04_zab${TAG}/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r04_zab${TAG}
mkdir -p "$OUT"
cd "$R"
VARIANTS=${VARIANTS:-"c4 w8 w8c4 w8c8 w8l96c4"}
: > "$OUT/ab.log"
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in tree $VARIANTS; do
    if [ $v = tree ]; then PKG=$R/nvidia-resiliency-ext-x_amd; else PKG=$R/tools/ab_$v; fi
    DUMP=""; [ $round = 1 ] && DUMP="/tmp/zab_$v.pt"  # 0.8 GB each: kept off gpurun_out
    AB_DUMP=$DUMP AB_PKG=$PKG timeout -k 10 240 python3 tools/ab_zipf.py 10 >> "$OUT/ab.log" 2> "$OUT/err_$v.log" || { echo "fail $v"; tail -5 "$OUT/err_$v.log"; exit 1; }
    tail -1 "$OUT/ab.log"
  done
done
for v in $VARIANTS; do python3 tools/ab_compare.py /tmp/zab_tree.pt /tmp/zab_$v.pt $v | tee -a "$OUT/ab.log"; done
