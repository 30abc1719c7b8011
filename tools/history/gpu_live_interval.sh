#!/bin/bash
# detector overhead vs profiling_interval on the live GPT-2 loop; gpurun_out/live_pi/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/live_pi
mkdir -p "$OUT"
cd "$R"
export MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
port=29561
for cfg in "8 1" "8 4" "8 16" "32 1" "32 16"; do
  set -- $cfg
  MASTER_PORT=$port timeout -k 10 300 python -u tools/live_gpt2.py --batch $1 --profiling-interval $2 \
      --steps 64 --report-every 32 --base-steps 30 --out "$OUT/b$1_pi$2.json" > "$OUT/b$1_pi$2.log" 2>&1 || { echo "fail $cfg"; tail -5 "$OUT/b$1_pi$2.log"; exit 1; }
  port=$((port+1))
  python -c "import json;d=json.load(open('$OUT/b$1_pi$2.json'));print('$cfg', round(d['step_ms_without_detector'],2), round(d['step_ms_with_detector'],2), round(d['detector_overhead_pct'],2), d['records_per_report'], round(d['report_ms_median'],2))"
done
