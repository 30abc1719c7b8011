#!/bin/bash
# configs[3] record-stream path (16,384 Zipf streams): kernel-trace summary plus the memory-side
# traffic of every kernel of compute_stats_records from separate --pmc passes (FETCH_SIZE,
# WRITE_SIZE, L2 hit/miss).  Output under gpurun_out/pmc_zt/; tools/pmc_zipf_json.py turns it
# into profiles/pmc_zipf_bucket.json + profiles/pmc_zipf_stats.json.
set -e
R=$GRAFT_REPO_ROOT
OUT=${OUT:-$R/gpurun_out/pmc_zt}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export AB_R=${AB_R:-16384}
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- \
    python3 "$R/tools/ab_zipf.py" 3 > "$OUT/trace.log" 2>&1
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo "$grp" | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_$tag" -o p -- \
      python3 "$R/tools/ab_zipf.py" 2 > "$OUT/pmc_$tag.log" 2>&1
done
echo done
