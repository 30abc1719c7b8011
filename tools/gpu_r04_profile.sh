#!/bin/bash
# Round-4 measurement: the default bench line, its kernel-trace summary, the configs[1] stats
# kernel's FETCH_SIZE / WRITE_SIZE passes, and the configs[3] per-kernel traffic.
# Output: gpurun_out/r04_prof/
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${PROF_TAG:-r04_prof}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
tail -1 "$OUT/bench.json" | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
    python3 "$R/bench.py" > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
echo trace done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o p -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 --no-latency4096 --no-zipf --no-cpu-baseline \
      > "$OUT/pmc_$c.log" 2>&1
done
echo pmc done
OUT=$OUT/zipf bash "$R/tools/pmc_zipf_traffic.sh"
