#!/bin/bash
# configs[2] statistics: the tree against its build variants (tools/ab_<name>, tools/build_variant.sh)
# and the round-start library (tools/ab_pkg), interleaved, AB_ROUNDS rounds.  Output: gpurun_out/r03_variants/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${RUN_TAG:-r03_variants}
mkdir -p "$OUT"
cd "$R"
for i in $(seq ${AB_ROUNDS:-3}); do
  for pkg in nvidia-resiliency-ext-x_amd $(ls -d tools/ab_* | grep -v '\.'); do
    timeout -k 5 120 python3 tools/ab_c3_pair.py "$R/$pkg" ${AB_REPS:-10} 2>&1 | grep ms= || exit 1
  done
done | tee "$OUT/ab.log"
