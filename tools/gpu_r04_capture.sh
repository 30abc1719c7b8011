#!/bin/bash
# Live-capture delivery modes: tools/capture_cost per tool state x
# NVRX_CAPTURE_DELIVERY (buffer / callback / callback_counted), interleaved twice; one process
# per run (the tool configures before the runtime initialises).  gpurun_out/r04_cap/cost.jsonl
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r04_cap
mkdir -p "$OUT"
cd "$R"
: > "$OUT/cost.jsonl"
for rep in 1 2; do
  for dl in buffer callback callback_counted; do
    for mode in none started cycle; do
      NVRX_CAPTURE_DELIVERY=$dl timeout -k 5 60 ./tools/capture_cost $mode 20000 >> "$OUT/cost.jsonl" 2> "$OUT/err_${dl}_$mode.log" || { echo "fail $dl $mode"; tail -3 "$OUT/err_${dl}_$mode.log"; exit 1; }
    done
  done
done
cat "$OUT/cost.jsonl"
