#!/bin/bash
# The -m gpu suite in one process (run through gpurun): gpurun_out/${TAG:-tests}/pytest.log
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-tests}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS} > "$OUT/pytest.log" 2>&1
rc=$?
tail -15 "$OUT/pytest.log"
exit $rc
