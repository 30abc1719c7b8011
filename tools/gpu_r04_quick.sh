#!/bin/bash
# Round-4 quick GPU check: the given tests (PYTEST_ARGS) then a short default bench line.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r04_quick${TAG}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 170 --timeout-method thread ${PYTEST_ARGS} > "$OUT/pytest.log" 2>&1
rc=$?
tail -15 "$OUT/pytest.log"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cat "$OUT/bench.json"
exit $rc
