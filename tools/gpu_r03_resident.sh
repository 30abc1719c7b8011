#!/bin/bash
# records_resident.hip bring-up: record-path parity tests, then configs[3] timing + kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_res
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_profiler_records.py tests/test_gpu_batch.py -k "records_stats or zipf" > "$OUT/tests.log" 2>&1
rc=$?; tail -5 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/ab_zipf.py 10 > "$OUT/ab.log" 2>&1 || exit 1
cat "$OUT/ab.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- \
    python3 "$R/tools/ab_zipf.py" 3 > "$OUT/trace.log" 2>&1 || exit 1
cd "$R" && timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread \
    tests/test_gpu_fullsize.py -k config3 > "$OUT/full.log" 2>&1
rc=$?; tail -5 "$OUT/full.log"; exit $rc
