#!/bin/bash
# Pipelined whole-report graphs: their GPU tests, the bench/report GPU tests, then the default
# bench line.  Output: gpurun_out/r03_pipe/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_pipe
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipelined.py tests/test_gpu_batch.py tests/test_bench_launcher.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
tail -1 "$OUT/bench.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'], d['latency_4096_ranks']['ms_per_report'], d['zipf_16384_ranks']['ms_per_report'])"
