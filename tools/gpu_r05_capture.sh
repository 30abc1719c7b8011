#!/bin/bash
# Round 5: the counted capture flush -- the capture test files, then the
# completeness A/B under host load.  Logs under gpurun_out/r05_cap/.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_cap
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_capture_complete.py tests/test_gpu_capture.py tests/test_gpu_capture_fidelity.py \
  tests/test_gpu_live.py > "$OUT/tests.log" 2>&1 || { tail -60 "$OUT/tests.log"; exit 1; }
tail -15 "$OUT/tests.log"
timeout -k 10 600 python -u tools/capture_complete_ab.py --repeats 2 --out "$OUT/complete_ab.json" > "$OUT/ab.log" 2>&1 || { tail -30 "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
