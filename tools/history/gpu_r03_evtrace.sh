#!/bin/bash
# The bench's HIP-event time of the configs[1] stats kernel against rocprofv3's kernel trace of the
# same process.  Output: gpurun_out/r03_evtrace/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_evtrace
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o b -- \
    python3 "$R/bench.py" --steps 200 --no-latency4096 --no-zipf --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
tail -1 "$OUT/bench.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('events', d['roofline']['kernel_ms'], 'step', d['ms_per_step'])"
grep "lean_group_kernel<128" "$OUT"/trace/*kernel_stats.csv | cut -d, -f1-4
