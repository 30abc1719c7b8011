#!/bin/bash
# GPT-2 small DDP (world of one) Detector overhead by capture delivery x profiling_interval x batch,
# interleaved ROUNDS times on one box.  gpurun_out/r05_lm/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_lm
mkdir -p "$OUT"
cd "$R"
export MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
port=29701
for rep in $(seq 1 ${ROUNDS:-2}); do
  for cfg in "queue 8 1" "callback 8 1" "queue 8 4" "callback 8 4" "queue 8 16" "callback 8 16" "queue 32 1" "callback 32 1"; do
    set -- $cfg
    tag="r${rep}_$1_b$2_pi$3"
    NVRX_CAPTURE_DELIVERY=$1 MASTER_PORT=$port timeout -k 10 300 python -u tools/live_gpt2.py --batch $2 --profiling-interval $3 \
        --steps 64 --report-every 32 --base-steps 30 --out "$OUT/$tag.json" > "$OUT/$tag.log" 2>&1 || { echo "fail $tag"; tail -5 "$OUT/$tag.log"; exit 1; }
    port=$((port+1))
    python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', round(d['step_ms_without_detector'],2), round(d['step_ms_with_detector'],2), round(d['detector_overhead_pct'],2), d['records_per_report'], round(d['report_ms_median'],2))"
  done
done
