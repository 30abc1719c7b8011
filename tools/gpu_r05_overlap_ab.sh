#!/bin/bash
# Pipelined reports, overlapped phases (default) against one whole-report graph per report
# (NVRX_PIPE_OVERLAP=0): the pipelined tests, then ROUNDS interleaved bench lines of each
# (no CPU baseline).  gpurun_out/r05_overlap${TAG}/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_overlap${TAG}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipelined.py ${TESTS} > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
for round in $(seq 1 ${ROUNDS:-2}); do
  for ov in 1 0; do
    NVRX_PIPE_OVERLAP=$ov timeout -k 10 400 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench_ov${ov}_r${round}.json" 2> "$OUT/bench_ov${ov}_r${round}.err" || { tail -30 "$OUT/bench_ov${ov}_r${round}.err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/bench_ov${ov}_r${round}.json'))
z=d.get('zipf_16384_ranks') or {}
print('overlap=$ov', 'value', d['value'], 'ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],4), 'launch', d['config']['launch'][:40], 'zipf report', z.get('ms_per_report'), 'zipf stats', z.get('bucket_plus_stats_ms'))"
  done
done
