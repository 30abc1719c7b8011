#!/bin/bash
# the whole GPU suite in the driver's order, then smoke; logs under gpurun_out/full/.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/full
mkdir -p "$OUT"
cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > "$OUT/pytest.log" 2>&1
echo "pytest rc=$?"
tail -12 "$OUT/pytest.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; echo "smoke rc=$?"
