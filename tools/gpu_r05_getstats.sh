#!/bin/bash
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r05_gs${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 "$R/tools/probe_get_stats.py" 2>&1 | grep RESULT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o t -- python3 "$R/tools/probe_get_stats.py" > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
f=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# the last report's kernels: after the last records_bucket
idx = max(i for i, r in enumerate(rows) if "records_bucket" in r["Kernel_Name"])
t0 = int(rows[idx]["Start_Timestamp"])
prev = None
for r in rows[idx - 2: idx + 24]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:7.1f}  gap {((s - prev) / 1e3 if prev else 0):7.1f}  {r['Kernel_Name'][:70]}")
    prev = e
PY
