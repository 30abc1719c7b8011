#!/bin/bash
# Round 5 quick check: named test files (TESTS) then the default bench line.  gpurun_out/r05_quick/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_quick${TAG}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu ${TESTS} > "$OUT/tests.log" 2>&1 || { tail -60 "$OUT/tests.log"; exit 1; }
tail -8 "$OUT/tests.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'phases', d['ms_per_step_graph_phases'], d['graph_phases']['launch'], 'frac', d['roofline']['frac'])
z=d['zipf_16384_ranks']; print('zipf bucket+stats', z['bucket_plus_stats_ms'], 'report', z['ms_per_report'])
l=d['latency_4096_ranks']; print('c2 report', l['ms_per_report'], 'kernel', l['stats_kernel_ms'])
"
