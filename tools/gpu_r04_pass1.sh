#!/bin/bash
# configs[3] pass-1 probes: kernel traces of the bucketing kernel in timing-only builds --
# abl1 (pass 1 + scans), abl4 (pass 1's loads without the LDS slot counts), abl1u16 (abl1 with 16
# loads in flight per lane for the stream's tail) -- and the full kernel with 16 (u16) against the
# library; interleaved twice.  Output: gpurun_out/r04_pass1/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r04_pass1${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for v in ${VARIANTS:-tree abl1 abl4 abl1u16 u16}; do
    if [ $v = tree ]; then PKG=$R/nvidia-resiliency-ext-x_amd; else PKG=$R/tools/ab_$v; fi
    AB_PKG=$PKG timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/${v}_$round" -o t -- python3 "$R/tools/ab_zipf.py" 10 > "$OUT/${v}_$round.log" 2>&1 || exit 1
    echo "$v $round $(grep -o 'records_stats_ms=[0-9.]*' $OUT/${v}_$round.log) bucket_avg_ns=$(grep records_bucket_kernel $OUT/${v}_$round/t_kernel_stats.csv | python3 -c 'import sys,csv; print(list(csv.reader(sys.stdin))[0][3])')"
  done
done
