#!/bin/bash
# branchless candidate compaction: segment-stats parity tests, then configs[2] / configs[1]
# stats-kernel timing, this tree vs _ab_old (round 1), interleaved.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_compact
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_segment_stats.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
echo "pytest rc=$?"; tail -2 "$OUT/pytest.log"
for i in 1 2 3; do
  for tree in new old; do
    d=$R; [ $tree = old ] && d=$R/_ab_old
    cd "$d"
    echo -n "$tree c3: "; timeout -k 10 120 python tools/ab_c3.py 10 2>&1 | grep ms=
    echo -n "$tree c2: "; AB_R=64 AB_S=10000 timeout -k 10 120 python tools/ab_c3.py 50 2>&1 | grep ms=
  done
done
