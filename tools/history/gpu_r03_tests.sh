#!/bin/bash
# Round-3 full GPU suite, one process; gpurun_out/r03_tests/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_tests
mkdir -p "$OUT"
cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -5 "$OUT/pytest.log"
exit $rc
