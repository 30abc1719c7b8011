#!/bin/bash
# configs[1] stats kernel: this tree vs _ab_old, interleaved on one box.
R=$GRAFT_REPO_ROOT
cd "$R"
for i in 1 2 3; do
  for tree in new old; do
    d=$R; [ $tree = old ] && d=$R/_ab_old
    cd "$d"
    echo -n "$tree c1: "; AB_R=64 AB_S=10000 timeout -k 10 120 python tools/ab_c3.py 50 2>&1 | grep ms= || exit 1
  done
done
