#!/bin/bash
# Round 5: queue delivery (NVRX_CAPTURE_DELIVERY=queue, capture.cpp "Queue delivery") -- its
# per-dispatch cost against callback delivery, the capture tests in that mode, and the GPT-2 step
# overhead.  gpurun_out/r05_queue${TAG}/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_queue${TAG}
mkdir -p "$OUT"
cd "$R"
if [ -z "$NOCOST" ]; then
: > "$OUT/cost.jsonl"
for rep in 1 2; do
  for dl in queue callback; do
    for mode in stopped started; do
      NVRX_CAPTURE_DELIVERY=$dl timeout -k 5 60 ./tools/capture_cost $mode 20000 >> "$OUT/cost.jsonl" 2> "$OUT/err_${dl}_$mode.log" || { echo "fail $dl $mode"; tail -5 "$OUT/err_${dl}_$mode.log"; exit 1; }
      tail -1 "$OUT/cost.jsonl" | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$dl $mode', d['launch_us_per_dispatch'], d['drain_us_per_dispatch'], d['flush_us'], d.get('enqueues_counted'), d['kernels'])"
    done
  done
done
fi
if [ -z "$NOTESTS" ]; then
NVRX_CAPTURE_DELIVERY=queue timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_capture.py tests/test_gpu_capture_fidelity.py tests/test_gpu_capture_complete.py tests/test_gpu_live.py} > "$OUT/tests.log" 2>&1 || { tail -60 "$OUT/tests.log"; exit 1; }
tail -15 "$OUT/tests.log"
fi
if [ -n "$NOLIVE" ]; then exit 0; fi
export MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
port=29611
for rep in $(seq 1 ${LREPS:-2}); do
  for dl in queue callback; do
    NVRX_CAPTURE_DELIVERY=$dl MASTER_PORT=$port timeout -k 10 240 python -u tools/live_gpt2.py --batch 8 --profiling-interval 1 \
        --steps 64 --report-every 32 --base-steps 30 --out "$OUT/live_r${rep}_$dl.json" > "$OUT/live_r${rep}_$dl.log" 2>&1 || { echo "fail live $rep $dl"; tail -5 "$OUT/live_r${rep}_$dl.log"; exit 1; }
    port=$((port+1))
    python -c "import json;d=json.load(open('$OUT/live_r${rep}_$dl.json'));print('live $rep $dl', round(d['step_ms_without_detector'],2), round(d['step_ms_with_detector'],2), round(d['detector_overhead_pct'],2), d['records_per_report'], round(d['report_ms_median'],2), d['capture_flush_ms_median'], d['kernel_keys'])"
  done
done
