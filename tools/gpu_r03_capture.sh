#!/bin/bash
# Live-capture cost: tools/capture_cost in each mode, interleaved 3 times
# (one process per run: the tool configures before the runtime initialises).  gpurun_out/r03_cap/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_cap
mkdir -p "$OUT"
cd "$R"
: > "$OUT/cost.jsonl"
for rep in 1 2 3; do
  for mode in none stopped started cycle; do
    timeout -k 5 60 ./tools/capture_cost $mode 20000 >> "$OUT/cost.jsonl" 2> "$OUT/err_$mode.log" || { echo "fail $mode"; tail -3 "$OUT/err_$mode.log"; exit 1; }
  done
done
cat "$OUT/cost.jsonl"
