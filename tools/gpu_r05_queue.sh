#!/bin/bash
# Round 5: queue delivery (NVRX_CAPTURE_DELIVERY=queue, capture.cpp "Queue delivery") -- its
# per-dispatch cost against callback delivery, the capture tests in that mode, and the GPT-2 step
# overhead.  gpurun_out/r05_queue${TAG}/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_queue${TAG}
mkdir -p "$OUT"
cd "$R"
: > "$OUT/cost.jsonl"
for rep in 1 2; do
  for dl in queue callback; do
    for mode in stopped started; do
      NVRX_CAPTURE_DELIVERY=$dl timeout -k 5 60 ./tools/capture_cost $mode 20000 >> "$OUT/cost.jsonl" 2> "$OUT/err_${dl}_$mode.log" || { echo "fail $dl $mode"; tail -5 "$OUT/err_${dl}_$mode.log"; exit 1; }
      tail -1 "$OUT/cost.jsonl" | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$dl $mode', d['launch_us_per_dispatch'], d['records_delivered'], d['flush_us'], d.get('enqueues_counted'), d['kernels'])"
    done
  done
done
if [ -n "$NOTESTS" ]; then exit 0; fi
NVRX_CAPTURE_DELIVERY=queue timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_capture.py tests/test_gpu_capture_fidelity.py tests/test_gpu_capture_complete.py tests/test_gpu_live.py} > "$OUT/tests.log" 2>&1 || { tail -60 "$OUT/tests.log"; exit 1; }
tail -15 "$OUT/tests.log"
