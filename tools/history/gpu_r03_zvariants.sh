#!/bin/bash
# configs[3] record statistics: the tree against its build variants (tools/ab_<name>) and the
# round-start library (tools/ab_pkg), interleaved, AB_ROUNDS rounds.  Output: gpurun_out/r03_zvariants/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${RUN_TAG:-r03_zvariants}
mkdir -p "$OUT"
cd "$R"
for i in $(seq ${AB_ROUNDS:-3}); do
  for pkg in nvidia-resiliency-ext-x_amd $(ls -d tools/ab_* | grep -v '\.'); do
    AB_PKG=$R/$pkg timeout -k 5 180 python3 tools/ab_zipf.py 10 2>&1 | grep records_stats_ms || exit 1
  done
done | tee "$OUT/ab.log"
