#!/bin/bash
# Detector overhead and report-time flush on the live GPT-2 loop (batch 8), capture delivery
# buffer vs callback_counted (the default) at profiling_interval 1 and 16, interleaved twice on
# one box; gpurun_out/r04_live/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r04_live${TAG}
mkdir -p "$OUT"
cd "$R"
export MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
port=29571
for rep in $(seq 1 ${REPS:-2}); do
  for dl in ${DELIVERIES:-buffer callback_counted}; do
    for pi in ${INTERVALS:-1 16}; do
      NVRX_CAPTURE_DELIVERY=$dl MASTER_PORT=$port timeout -k 10 240 python -u tools/live_gpt2.py --batch 8 --profiling-interval $pi \
          --steps 64 --report-every 32 --base-steps 30 --out "$OUT/r${rep}_${dl}_pi$pi.json" > "$OUT/r${rep}_${dl}_pi$pi.log" 2>&1 || { echo "fail $rep $dl $pi"; tail -5 "$OUT/r${rep}_${dl}_pi$pi.log"; exit 1; }
      port=$((port+1))
      python -c "import json;d=json.load(open('$OUT/r${rep}_${dl}_pi$pi.json'));print('$rep $dl $pi', round(d['step_ms_without_detector'],2), round(d['step_ms_with_detector'],2), round(d['detector_overhead_pct'],2), d['records_per_report'], round(d['report_ms_median'],2), round(d['capture_flush_ms_median'],3), round(d['empty_flush_ms_median'],3), flush=True)"
    done
  done
done
