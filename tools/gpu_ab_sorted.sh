#!/bin/bash
# chunk-sorted bucket scatter: parity tests, then configs[3] record statistics A/B (interleaved).
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_sorted
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_profiler_records.py tests/test_gpu_batch.py -m gpu -x -q --timeout 200 --timeout-method thread -k "records or zipf or bucket or profiler" > "$OUT/pytest.log" 2>&1
echo "pytest rc=$?"; tail -3 "$OUT/pytest.log"
for i in 1 2 3; do
  for v in 0 1; do
    NVRX_RB_SORTED=$v timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep records_stats_ms
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- python3 "$R/tools/ab_zipf.py" 5 > "$OUT/trace.log" 2>&1
grep -h "records_bucket" "$OUT"/trace/*kernel_stats.csv | cut -c1-200
