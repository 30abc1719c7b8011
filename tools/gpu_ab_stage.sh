#!/bin/bash
# cold-bucket LDS staging: record / ragged parity tests (default and cold=8192, all staged
# where it fits), then configs[3] record statistics over NVRX_RB_STAGE_KB / NVRX_RB_COLD,
# interleaved with _ab_old (the tree before staging).
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_stage
mkdir -p "$OUT"
cd "$R"
if [ -z "${GRID_SET:-}" ]; then GRID=("0 64" "48 64" "72 64" "96 64" "72 16" "72 128" "96 128"); else eval "GRID=($GRID_SET)"; fi
for c in ${TEST_COLDS-64 8192}; do
  NVRX_RB_COLD=$c timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_profiler_records.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "records or zipf or bucket or profiler or config3" > "$OUT/pytest_$c.log" 2>&1
  rc=$?; echo "cold=$c pytest rc=$rc"; tail -1 "$OUT/pytest_$c.log"; [ $rc -eq 0 ] || exit 1
done
for i in 1 2; do
  cd "$R/_ab_old"; echo -n "old: "; timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep -o "records_stats_ms=[0-9.]*" || exit 1
  cd "$R"
  for v in "${GRID[@]}"; do
    set -- $v
    echo -n "stage_kb=$1 cold=$2 coldest=${3:-16} "; NVRX_RB_STAGE_KB=$1 NVRX_RB_COLD=$2 NVRX_RB_COLDEST=${3:-16} timeout -k 10 120 python tools/ab_zipf.py 10 2>&1 | grep -o "records_stats_ms=[0-9.]*" || exit 1
  done
done
