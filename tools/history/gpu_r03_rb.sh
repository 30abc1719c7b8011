#!/bin/bash
# records_bucket_kernel iteration: record-path parity tests, configs[3] timing + kernel trace,
# then full-world configs[3] parity.  gpurun_out/r03_rb/
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_rb
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_profiler_records.py tests/test_gpu_batch.py > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/ab_zipf.py 10 2>&1 | grep -v amdgpu.ids | tee "$OUT/ab.log" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- \
    python3 "$R/tools/ab_zipf.py" 3 > "$OUT/trace.log" 2>&1 || exit 1
cd "$R" && timeout -k 10 400 python -u -m pytest -x -q --timeout 380 --timeout-method thread \
    tests/test_gpu_fullsize.py -k config3 > "$OUT/full.log" 2>&1
rc=$?; tail -3 "$OUT/full.log"; exit $rc
