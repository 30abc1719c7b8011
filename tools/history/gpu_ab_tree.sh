#!/bin/bash
# This tree against _ab_old (a build of the previous commit), interleaved on one box: parity
# tests of this tree first, then configs[1] / configs[2] statistics (tools/ab_c3.py) and
# configs[3] record statistics (tools/ab_zipf.py) from each tree in turn.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_tree
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_segment_stats.py tests/test_gpu_batch.py tests/test_gpu_profiler_records.py tests/test_gpu_fullsize.py tests/test_gpu_report.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for tree in new old; do
    d=$R; [ $tree = old ] && d=$R/_ab_old
    cd "$d"
    echo -n "$tree c1: "; AB_R=64 AB_S=10000 timeout -k 10 120 python tools/ab_c3.py 50 2>&1 | grep -o "ms=[0-9.]*" || exit 1
    echo -n "$tree c2: "; timeout -k 10 120 python tools/ab_c3.py 10 2>&1 | grep -o "ms=[0-9.]*" || exit 1
    echo -n "$tree c3: "; timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep -o "records_stats_ms=[0-9.]*" || exit 1
  done
done
