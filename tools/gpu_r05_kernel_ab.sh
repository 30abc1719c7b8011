#!/bin/bash
# Statistics kernels of a build variant (tools/ab_<v>, tools/build_variant.sh) against the tree,
# interleaved: configs[1] and configs[2] (tools/ab_c3_pair.py, ms per launch) and configs[3]
# (tools/ab_zipf.py, record statistics ms), ROUNDS rounds.  gpurun_out/r05_kab${TAG}/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_kab${TAG}
mkdir -p "$OUT"
cd "$R"
: > "$OUT/ab.log"
for round in $(seq 1 ${ROUNDS:-3}); do
  for v in tree $VARIANTS; do
    if [ $v = tree ]; then PKG=$R/nvidia-resiliency-ext-x_amd; else PKG=$R/tools/ab_$v; fi
    AB_R=64 AB_S=10000 timeout -k 10 120 python3 tools/ab_c3_pair.py "$PKG" 50 >> "$OUT/ab.log" 2>>"$OUT/err.log" || { echo "fail c1 $v"; tail -5 "$OUT/err.log"; exit 1; }
    timeout -k 10 200 python3 tools/ab_c3_pair.py "$PKG" 10 >> "$OUT/ab.log" 2>>"$OUT/err.log" || { echo "fail c2 $v"; exit 1; }
    AB_PKG=$PKG timeout -k 10 240 python3 tools/ab_zipf.py 10 >> "$OUT/ab.log" 2>>"$OUT/err.log" || { echo "fail c3 $v"; exit 1; }
    tail -3 "$OUT/ab.log" | cut -c1-150
  done
done
