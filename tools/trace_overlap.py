"""Split one kernel's launches in a rocprofv3 kernel trace into isolated ones and ones that overlap
another launch of the same kernel (two-stream pipelined reports run consecutive statistics kernels
side by side, so the trace's --stats average mixes both).  Usage:
python tools/trace_overlap.py <kernel_trace.csv> <kernel-name substring> > summary.json"""
import csv
import json
import statistics
import sys

path, key = sys.argv[1], sys.argv[2]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            for r in csv.DictReader(open(path)) if key in r["Kernel_Name"])
iso, ovl = [], []
for i, (s, e) in enumerate(ks):
    o = (i > 0 and ks[i - 1][1] > s) or (i + 1 < len(ks) and ks[i + 1][0] < e)
    (ovl if o else iso).append((e - s) / 1e6)
# wall time the overlapped launches cover together (union of their intervals), per launch
wall, cur = 0, None
for i, (s, e) in enumerate(ks):
    o = (i > 0 and ks[i - 1][1] > s) or (i + 1 < len(ks) and ks[i + 1][0] < e)
    if not o:
        continue
    if cur and s <= cur[1]:
        cur = (cur[0], max(cur[1], e))
    else:
        if cur:
            wall += cur[1] - cur[0]
        cur = (s, e)
if cur:
    wall += cur[1] - cur[0]
print(json.dumps(dict(
    trace=path, kernel=key, launches=len(ks),
    all_mean_ms=statistics.mean((e - s) / 1e6 for s, e in ks) if ks else None,
    isolated=dict(launches=len(iso), mean_ms=statistics.mean(iso) if iso else None,
                  median_ms=statistics.median(iso) if iso else None),
    overlapped=dict(launches=len(ovl), mean_ms=statistics.mean(ovl) if ovl else None,
                    wall_ms_per_launch=wall / 1e6 / len(ovl) if ovl else None)), indent=1))
