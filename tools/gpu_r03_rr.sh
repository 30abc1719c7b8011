#!/bin/bash
# records_resident.hip iteration: record-path parity tests, ablation timings, then full-world configs[3].
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_rr
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_profiler_records.py tests/test_gpu_batch.py -k "records_stats or zipf or wide or durations" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for m in 0 1 3 7 15; do timeout -k 5 60 ./tools/rr_bench_$m 16384 5 || exit 1; done | tee "$OUT/ab.log"
timeout -k 10 400 python -u -m pytest -x -q --timeout 380 --timeout-method thread \
    tests/test_gpu_fullsize.py -k config3 > "$OUT/full.log" 2>&1
rc=$?; tail -3 "$OUT/full.log"; exit $rc
