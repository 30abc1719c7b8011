#!/bin/bash
# Round profile: kernel-trace summary of the default bench run, and the HBM traffic of the
# C2 stats kernel from separate --pmc passes (FETCH_SIZE, WRITE_SIZE).  Output under
# gpurun_out/round/; tools/pmc_c2_json.py turns the passes into profiles/pmc_c2_segment_stats.json.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/round
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
    python3 "$R/bench.py" > "$OUT/bench_trace.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o p -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 --no-latency4096 --no-zipf --no-cpu-baseline \
      > "$OUT/pmc_$c.log" 2>&1
done
echo done
