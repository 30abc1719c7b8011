#!/bin/bash
# Group-epilogue lean kernel: configs[2] parity tests, then an interleaved A/B of the configs[2]
# statistics kernel against the saved library in tools/ab_pkg.  Output: gpurun_out/r03_group/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_group
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_segment_stats.py tests/test_gpu_fullsize.py -k "not config3_full and not config1_full and not ragged" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_c3_pair.sh 2>&1 | tee "$OUT/ab.log"
