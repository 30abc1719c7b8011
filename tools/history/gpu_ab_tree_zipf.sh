#!/bin/bash
# record-path parity tests, then configs[3] record statistics: this tree vs _ab_old
# (interleaved), and a kernel trace of this tree.  OUT tag: $1 (default ab_tree).
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-ab_tree}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_profiler_records.py tests/test_gpu_fullsize.py tests/test_gpu_segment_stats.py -m gpu -x -q --timeout 300 --timeout-method thread -k "records or zipf or bucket or profiler or config3 or ragged" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for tree in new old; do
    d=$R; [ $tree = old ] && d=$R/_ab_old
    cd "$d"
    echo -n "$tree zipf: "; timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep -o "records_stats_ms=[0-9.]*" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- python3 "$R/tools/ab_zipf.py" 5 > "$OUT/trace.log" 2>&1 || exit 1
grep -h "records_bucket" "$OUT"/trace/*kernel_stats.csv | cut -c1-150
