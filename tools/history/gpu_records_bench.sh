#!/bin/bash
# record-path GPU tests (+ the RCCL exchange test), then the default bench line and its trace.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/recb
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_profiler_records.py tests/test_gpu_fullsize.py tests/test_gpu_rccl.py tests/test_gpu_live.py -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; echo "bench rc=$?"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"; echo "trace rc=$?"
