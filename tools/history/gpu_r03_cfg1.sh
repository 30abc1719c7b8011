#!/bin/bash
# Ragged / record parity after the list-kernel chunk epilogue, then the read ceilings
# (tools/mb_c2) and the configs[1] bench line on the same box.  Output: gpurun_out/r03_cfg1/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_cfg1
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_segment_stats.py tests/test_gpu_batch.py tests/test_gpu_profiler_records.py tests/test_gpu_fullsize.py -k "not config1_full and not config2_full" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/build/mb_c2 > "$OUT/mb_c2.log" 2>&1 || exit 1
grep cfg1 "$OUT/mb_c2.log"
timeout -k 10 200 python3 bench.py --steps 50 --no-latency4096 --no-zipf --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
tail -1 "$OUT/bench.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline'])"
