#!/bin/bash
# register-held pairs with 4 waves x 64 pairs / lane vs 8 waves x 32 pairs / lane (two
# waves per SIMD to hide pass 2's LDS-atomic latency): parity, then interleaved timing.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_waves_regs
mkdir -p "$OUT"
cd "$R"
for w in 16 8; do
  NVRX_RB_WAVES=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_profiler_records.py -m gpu -x -q --timeout 200 --timeout-method thread -k "records or zipf or bucket or profiler" > "$OUT/pytest_$w.log" 2>&1
  rc=$?; echo "waves=$w pytest rc=$rc"; tail -1 "$OUT/pytest_$w.log"; [ $rc -eq 0 ] || exit 1
done
for i in 1 2 3; do
  for w in 4 8 16; do
    echo -n "waves=$w "; NVRX_RB_WAVES=$w timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep -o "records_stats_ms=[0-9.]*" || exit 1
  done
done
