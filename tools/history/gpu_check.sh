#!/bin/bash
# Round check on the GPU box: gpu parity tests, smoke, default bench.  Logs under gpurun_out/check/.
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/check
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo ok
