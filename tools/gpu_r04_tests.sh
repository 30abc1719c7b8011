#!/bin/bash
# Round-4 full GPU suite, one process; gpurun_out/r04_tests${TAG}/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r04_tests${TAG}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 170 --timeout-method thread ${PYTEST_ARGS} > "$OUT/pytest.log" 2>&1
rc=$?
tail -15 "$OUT/pytest.log"
exit $rc
