#!/bin/bash
# GPT-2 small batch-8 Detector overhead at profiling_interval 1 by capture setting, interleaved
# LREPS times: MODES entries are delivery:queue_diag[:pc0] (pc0: sections with profile_cuda=False,
# the Detector's own CPU cost).  gpurun_out/r05_live${TAG}/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_live${TAG}
mkdir -p "$OUT"
cd "$R"
if [ -n "$COST" ]; then
  for dl in queue callback; do
    NVRX_CAPTURE_DELIVERY=$dl timeout -k 5 60 ./tools/capture_cost started 20000 > "$OUT/cost_$dl.json" 2> "$OUT/cost_$dl.err" || { echo "fail cost $dl"; tail -5 "$OUT/cost_$dl.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/cost_$dl.json'));print('cost $dl', d['launch_us_per_dispatch'], d['drain_us_per_dispatch'], d['flush_us'])"
  done
fi
export MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
port=29641
for rep in $(seq 1 ${LREPS:-2}); do
  for m in ${MODES:-queue:0 queue:1 queue:2 callback:0 queue:0:pc0}; do
    IFS=: read dl diag pc <<< "$m"
    pcf=1; [ "$pc" = "pc0" ] && pcf=0
    tag="${dl}_d${diag}_pc${pcf}"
    NVRX_CAPTURE_DELIVERY=$dl NVRX_CAPTURE_QUEUE_DIAG=$diag MASTER_PORT=$port timeout -k 10 240 python -u tools/live_gpt2.py --batch ${BATCH:-8} \
        --profiling-interval ${PI:-1} --profile-cuda $pcf --steps 64 --report-every 32 --base-steps 30 \
        --out "$OUT/live_r${rep}_$tag.json" > "$OUT/live_r${rep}_$tag.log" 2>&1 || { echo "fail live $rep $tag"; tail -5 "$OUT/live_r${rep}_$tag.log"; exit 1; }
    port=$((port+1))
    python -c "import json;d=json.load(open('$OUT/live_r${rep}_$tag.json'));print('live $rep $tag', round(d['step_ms_without_detector'],2), round(d['step_ms_with_detector'],2), round(d['detector_overhead_pct'],2), d['records_per_report'], round(d['report_ms_median'],2), d['kernel_keys'])"
  done
done
