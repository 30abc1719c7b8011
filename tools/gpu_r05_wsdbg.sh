#!/bin/bash
# WS kernel debug: output diff at small R, then per-kernel times of both kernels at full size
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_wsdbg
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
if [ -n "$DIFF" ]; then
  AB_R=512 timeout -k 10 120 python -u tools/ws_diff.py ${SPLIT:-8x8} > "$OUT/diff.log" 2>&1 || { tail -20 "$OUT/diff.log"; exit 1; }
  cat "$OUT/diff.log"
fi
for ws in 0 ${SPLITS:-8x8}; do
  NVRX_RB_WS=$ws timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$ws" -o run -- python3 tools/ab_zipf.py 5 > "$OUT/prof_$ws.log" 2>&1 || { tail -20 "$OUT/prof_$ws.log"; exit 1; }
  f=$(find "$OUT/prof_$ws" -name "*kernel_stats.csv" | head -1)
  python -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:6]: print('$ws', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')"
done
