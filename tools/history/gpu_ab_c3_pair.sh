#!/bin/bash
# A/B (interleaved, same box): configs[2] stats kernel, saved library (tools/ab_pkg) vs the tree's.
R=$GRAFT_REPO_ROOT
cd "$R"
for i in 1 2 3; do
  timeout -k 5 120 python3 tools/ab_c3_pair.py "$R/tools/ab_pkg" 10 2>&1 | grep ms= || exit 1
  timeout -k 5 120 python3 tools/ab_c3_pair.py "$R/nvidia-resiliency-ext-x_amd" 10 2>&1 | grep ms= || exit 1
done
