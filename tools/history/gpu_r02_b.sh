#!/bin/bash
# round-2 check B: the profiler / capture / detector / functional GPU tests.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02b
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests/test_gpu_profiler_records.py tests/test_gpu_detector.py \
  tests/test_gpu_capture.py tests/test_gpu_capture_fidelity.py tests/test_gpu_live.py \
  tests/test_gpu_functional_ddp.py -m gpu -v -s --timeout 400 --timeout-method thread > "$OUT/pytest.log" 2>&1 || echo "pytest rc=$?"
tail -5 "$OUT/pytest.log"
