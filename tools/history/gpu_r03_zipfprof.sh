#!/bin/bash
# configs[3] record statistics after this round's class-kernel changes: kernel trace and the SQ
# counters (tools/pmc_zipf_sq.sh).  Output: gpurun_out/r03_zipfprof/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03_zipfprof
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- \
    python3 "$R/tools/ab_zipf.py" 3 > "$OUT/trace.log" 2>&1 || exit 1
OUT=$OUT/sq bash "$R/tools/pmc_zipf_sq.sh" || exit 1
python3 "$R/tools/pmc_sum.py" "$R/gpurun_out/r03_zipfprof/sq/p1" "$R/gpurun_out/r03_zipfprof/sq/p2" > "$R/gpurun_out/r03_zipfprof/sq.txt" 2>&1
