#!/bin/bash
# configs[2] statistics kernel (4096 x 2048 x 1024, seg_stats_lean_group_kernel<16>): FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes over tools/ab_c3_pair.py, plus its kernel-trace summary.
# Output: gpurun_out/pmc_cfg2/; tools/pmc_configs2_json.py writes profiles/pmc_configs2_segment_stats.json
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_cfg2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- \
    python3 "$R/tools/ab_c3_pair.py" "$R/nvidia-resiliency-ext-x_amd" 5 > "$OUT/trace.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o p -- \
      python3 "$R/tools/ab_c3_pair.py" "$R/nvidia-resiliency-ext-x_amd" 3 > "$OUT/pmc_$c.log" 2>&1
done
echo done
