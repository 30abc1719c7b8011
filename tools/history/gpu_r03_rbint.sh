#!/bin/bash
# Interleaved register head in the bucketing kernel: record-path parity, then configs[3] record
# statistics against the previous bucketing kernel (tools/ab_prev) and the round-start library.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${RUN_TAG:-r03_rbint}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_segment_stats.py tests/test_gpu_profiler_records.py tests/test_gpu_batch.py tests/test_gpu_fullsize.py tests/test_gpu_rccl.py -k "not config1_full and not config2_full" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=3 RUN_TAG=${RUN_TAG:-r03_rbint}_ab bash tools/gpu_r03_zvariants.sh
