#!/bin/bash
# Round 5: the capture's per-dispatch cost attributed per rocprofiler-sdk
# service -- tools/capture_cost, one process per setting, interleaved REPS times:
#   none | stopped | started x delivery (callback, buffer, callback_counted) x marking (1, 0),
#   and started/callback without code-object tracing (NVRX_CAPTURE_SYMBOLS=0)
# then the GPT-2 small batch-8 step overhead at profiling_interval 1 (default mode, and marking
# off) and 16.  gpurun_out/r05_cost/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_cost
mkdir -p "$OUT"
cd "$R"
: > "$OUT/cost.jsonl"
run() {  # label env... -- mode
  local label=$1; shift
  env "$@" timeout -k 5 60 ./tools/capture_cost $MODE 20000 > "$OUT/one.json" 2> "$OUT/err_$label.log" || { echo "fail $label"; tail -3 "$OUT/err_$label.log"; exit 1; }
  python -c "import json,sys;d=json.load(open('$OUT/one.json'));d['label']='$label';print(json.dumps(d))" >> "$OUT/cost.jsonl"
}
for rep in $(seq 1 ${REPS:-3}); do
  MODE=none run none X=1
  MODE=stopped run stopped X=1
  for dl in callback buffer callback_counted; do
    for mk in 1 0; do
      MODE=started run "started_${dl}_m$mk" NVRX_CAPTURE_DELIVERY=$dl NVRX_CAPTURE_MARKING=$mk
    done
  done
  MODE=started run started_callback_m1_nosym NVRX_CAPTURE_SYMBOLS=0
done
python - "$OUT/cost.jsonl" <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
by = collections.defaultdict(list)
for r in rows:
    by[r["label"]].append(r["launch_us_per_dispatch"])
for k, v in by.items():
    v = sorted(v)
    print(f"{k:32s} launch us/dispatch median {v[len(v)//2]:.3f}  all {[round(x,3) for x in v]}")
PY
export MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
port=29581
for rep in $(seq 1 ${LREPS:-2}); do
  for cfg in "m1 1" "m0 1" "m1 16"; do
    set -- $cfg
    NVRX_CAPTURE_MARKING=${1#m} MASTER_PORT=$port timeout -k 10 240 python -u tools/live_gpt2.py --batch 8 --profiling-interval $2 \
        --steps 64 --report-every 32 --base-steps 30 --out "$OUT/live_r${rep}_$1_pi$2.json" > "$OUT/live_r${rep}_$1_pi$2.log" 2>&1 || { echo "fail live $rep $cfg"; tail -5 "$OUT/live_r${rep}_$1_pi$2.log"; exit 1; }
    port=$((port+1))
    python -c "import json;d=json.load(open('$OUT/live_r${rep}_$1_pi$2.json'));print('live $rep $1 pi$2', round(d['step_ms_without_detector'],2), round(d['step_ms_with_detector'],2), round(d['detector_overhead_pct'],2), d['records_per_report'], round(d['report_ms_median'],2), d['capture_flush_ms_median'], flush=True)"
  done
done
