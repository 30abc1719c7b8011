#!/bin/bash
# per-slot LDS counter copies in records_bucket_kernel: parity tests under each copy count,
# then configs[3] record statistics A/B (NVRX_RB_COPIES 1 / 2 / 4, interleaved).
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_copies
mkdir -p "$OUT"
cd "$R"
for c in 2 1 4; do
  NVRX_RB_COPIES=$c timeout -k 10 400 python -u -m pytest tests/test_gpu_profiler_records.py tests/test_gpu_batch.py -m gpu -x -q --timeout 200 --timeout-method thread -k "records or zipf or bucket or profiler" > "$OUT/pytest_$c.log" 2>&1
  rc=$?; echo "copies=$c pytest rc=$rc"; tail -2 "$OUT/pytest_$c.log"
  [ $rc -eq 0 ] || exit 1
done
for i in 1 2 3; do
  for c in 1 2 4; do
    NVRX_RB_COPIES=$c timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep records_stats_ms || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for c in 1 2 4; do
  NVRX_RB_COPIES=$c timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace$c" -o t -- python3 "$R/tools/ab_zipf.py" 5 > "$OUT/trace$c.log" 2>&1 || exit 1
  echo "copies=$c"; grep -h "records_bucket" "$OUT"/trace$c/*kernel_stats.csv | cut -c1-160
done
