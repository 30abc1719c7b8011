#!/bin/bash
# queue-delivery capture under rocprofv3 --kernel-trace (tools/probe_rocprof_coexist.py)
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_coexist
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for dl in queue callback; do
  NVRX_CAPTURE_DELIVERY=$dl timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$dl" -o t -- python3 "$R/tools/probe_rocprof_coexist.py" > "$OUT/$dl.log" 2>&1 || { echo "fail $dl"; tail -20 "$OUT/$dl.log"; exit 1; }
  grep RESULT "$OUT/$dl.log"
  f=$(find "$OUT/$dl" -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'stragglers' in r['Name']: print('$dl rocprofv3 saw', r['Name'][:40], r['Calls'])"
done
