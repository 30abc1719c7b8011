#!/bin/bash
# Ragged class kernels dealt over side streams (NVRX_RAGGED_STREAMS 1..4), the lane<16> class,
# and the bucketing kernel's own class lists (NVRX_RB_CLASSIFY=0: the three classification
# launches): segment-stats / record parity tests, then configs[3] record statistics per
# variant, interleaved; kernel-trace of 1 and 3 streams.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_streams
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_segment_stats.py tests/test_gpu_batch.py tests/test_gpu_profiler_records.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  echo -n "streams=1 (again): "
  NVRX_RAGGED_STREAMS=1 timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep -o "records_stats_ms=[0-9.]*" || exit 1
  for s in 1 2 3 4; do
    echo -n "streams=$s: "
    NVRX_RAGGED_STREAMS=$s timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep -o "records_stats_ms=[0-9.]*" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for s in 1 3; do
  NVRX_RAGGED_STREAMS=$s timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_s$s" -o t -- python3 "$R/tools/ab_zipf.py" 5 > "$OUT/trace_s$s.log" 2>&1 || exit 1
done
echo traces done
