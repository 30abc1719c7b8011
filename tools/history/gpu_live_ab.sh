#!/bin/bash
# live-capture overhead, this tree vs the round-1 tree (_ab_old), interleaved; gpurun_out/live_ab/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/live_ab
mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
port=29571
for i in 1 2 3; do
  for tree in new old; do
    d=$R; [ $tree = old ] && d=$R/_ab_old
    cd "$d"
    MASTER_PORT=$port timeout -k 10 300 python -u tools/live_gpt2.py --batch 8 --steps 64 --report-every 32 --base-steps 30 \
        --out "$OUT/${tree}_$i.json" > "$OUT/${tree}_$i.log" 2>&1 || { echo "fail $tree"; tail -5 "$OUT/${tree}_$i.log"; exit 1; }
    port=$((port+1))
    python -c "import json;d=json.load(open('$OUT/${tree}_$i.json'));print('$tree', round(d['step_ms_without_detector'],2), round(d['step_ms_with_detector'],2), round(d['detector_overhead_pct'],2), round(d['capture_flush_ms_median'],2), round(d['report_ms_median'],2))"
  done
done
