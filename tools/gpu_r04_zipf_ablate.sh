#!/bin/bash
# configs[3] bucketing-kernel breakdown: kernel traces of the record
# statistics with the library and with the timing-only ablation builds of records.hip
# (tools/build_variant.sh abl<k> -DNVRX_RB_ABLATE=k, built beforehand with VARIANT_SRCS=records):
#   abl1 = pass 1 + scans, abl2 = + pass 2, abl3 = + staged copy-out (no tiny stats), tree = all.
# Interleaved twice.  Output: gpurun_out/r04_ablate/<variant>_<round>/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r04_ablate
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for v in tree abl1 abl2 abl3; do
    if [ $v = tree ]; then PKG=$R/nvidia-resiliency-ext-x_amd; else PKG=$R/tools/ab_$v; fi
    AB_PKG=$PKG timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/${v}_$round" -o t -- python3 "$R/tools/ab_zipf.py" 10 > "$OUT/${v}_$round.log" 2>&1 || exit 1
    tail -1 "$OUT/${v}_$round.log"
  done
done
