#!/bin/bash
# Level-0 histogram bins kept in registers (lean_body / fast_body, short segments): parity
# tests, then configs[2] stats kernel with NVRX_LEAN_KEEPBIN=1/0 interleaved, configs[3] record
# statistics (list classes), and a kernel trace of each.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_keepbin
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_segment_stats.py tests/test_gpu_batch.py tests/test_gpu_profiler_records.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for kb in 1 0; do
    echo -n "configs[2] keepbin=$kb: "
    NVRX_LEAN_KEEPBIN=$kb timeout -k 10 120 python tools/ab_c3.py 10 2>&1 | grep -o "ms=[0-9.]* TB/s=[0-9.]*" || exit 1
  done
  echo -n "configs[3]: "
  timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep -o "records_stats_ms=[0-9.]*" || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c3" -o t -- python3 "$R/tools/ab_zipf.py" 5 > "$OUT/trace_c3.log" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c2" -o t -- python3 "$R/tools/ab_c3.py" 5 > "$OUT/trace_c2.log" 2>&1 || exit 1
echo traces done
