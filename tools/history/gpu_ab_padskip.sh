#!/bin/bash
# fast_body padding counted by bin 0's initial value (no per-padding-slot LDS atomics):
# segment-stats / record parity tests, then configs[3] record statistics, this tree vs
# _ab_old (HEAD before the change), interleaved; kernel-trace of both.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_padskip
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_segment_stats.py tests/test_gpu_batch.py tests/test_gpu_profiler_records.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for tree in new old; do
    d=$R; [ $tree = old ] && d=$R/_ab_old
    cd "$d"
    echo -n "$tree zipf: "; timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep -o "records_stats_ms=[0-9.]*" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for tree in new old; do
  d=$R; [ $tree = old ] && d=$R/_ab_old
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$tree" -o t -- python3 "$d/tools/ab_zipf.py" 5 > "$OUT/trace_$tree.log" 2>&1 || exit 1
done
echo traces done
