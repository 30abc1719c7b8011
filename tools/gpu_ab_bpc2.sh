#!/bin/bash
# two 8-wave bucketing blocks per CU (phases of two streams overlap) vs one 16-wave block:
# record parity under the 2-block shape, then interleaved timing over staging sizes.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_bpc2
mkdir -p "$OUT"
cd "$R"
NVRX_RB_WAVES=8 NVRX_RB_BPC=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_profiler_records.py -m gpu -x -q --timeout 300 --timeout-method thread -k "records or zipf or bucket or profiler" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  for v in "16 1 96" "8 2 56" "8 2 40" "8 2 24"; do
    set -- $v
    echo -n "waves=$1 bpc=$2 stage=$3 "; NVRX_RB_WAVES=$1 NVRX_RB_BPC=$2 NVRX_RB_STAGE_KB=$3 timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep -o "records_stats_ms=[0-9.]*" || exit 1
  done
done
