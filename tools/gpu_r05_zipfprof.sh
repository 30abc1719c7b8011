#!/bin/bash
# configs[3] record statistics: rocprofv3 kernel-trace summary of tools/ab_zipf.py.  gpurun_out/r05_zprof${TAG}/
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_zprof${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- python3 "$R/tools/ab_zipf.py" 5 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
grep records_stats_ms "$OUT/trace.log"
f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:24]: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
