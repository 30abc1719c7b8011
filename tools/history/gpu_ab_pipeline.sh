#!/bin/bash
# configs[3] pipelined bucketing / statistics: parity, then A/B over the batch count.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_pipe
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config3 or zipf" > "$OUT/pytest.log" 2>&1
echo "pytest rc=$?"; tail -2 "$OUT/pytest.log"
for i in 1 2; do
  for b in 1 2 4 8; do
    NVRX_RS_BATCHES=$b timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep records_stats_ms
  done
done
