#!/bin/bash
# Pipelined reports on two streams (default) against whole-report graphs on one stream
# (NVRX_PIPE_MODE=whole): the pipelined / batch / launcher GPU tests, the in-process interleaved
# probe (tools/probe_pipe_streams.py), then ROUNDS interleaved bench lines of each mode (no CPU
# baseline).  gpurun_out/r05_pipe${TAG}/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_pipe${TAG}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_pipelined.py tests/test_gpu_batch.py tests/test_bench_launcher.py > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 300 python3 tools/probe_pipe_streams.py 300 8 > "$OUT/probe.log" 2>&1 || { tail -20 "$OUT/probe.log"; exit 1; }
tail -1 "$OUT/probe.log" | cut -c1-200
for round in $(seq 1 ${ROUNDS:-2}); do
  for mode in alt whole; do
    NVRX_PIPE_MODE=$mode timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$OUT/bench_${mode}_r${round}.json" 2> "$OUT/bench_${mode}_r${round}.err" || { tail -30 "$OUT/bench_${mode}_r${round}.err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/bench_${mode}_r${round}.json'))
z=d['zipf_16384_ranks']
print('$mode', 'value', d['value'], 'ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],4), 'zipf report', round(z['ms_per_report'],4), 'zipf stats', round(z['bucket_plus_stats_ms'],4))"
  done
done
