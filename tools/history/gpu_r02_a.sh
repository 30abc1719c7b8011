#!/bin/bash
# round-2 check A: full-size parity tests, the 2-rank launcher rehearsal, then the default bench.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02a
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_bench_launcher.py -m gpu -x -v -s --timeout 400 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 500 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo ok
