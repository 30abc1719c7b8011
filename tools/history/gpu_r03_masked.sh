#!/bin/bash
# Masked lean body for ragged / misaligned segments: the full GPU suite, then configs[3] record
# statistics against tools/ab_pkg, interleaved.  Output: gpurun_out/r03_masked/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${RUN_TAG:-r03_masked}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  AB_PKG=$R/tools/ab_pkg timeout -k 5 180 python3 tools/ab_zipf.py 10 2>&1 | grep records_stats_ms || exit 1
  timeout -k 5 180 python3 tools/ab_zipf.py 10 2>&1 | grep records_stats_ms || exit 1
done | tee "$OUT/ab_c3.log"
