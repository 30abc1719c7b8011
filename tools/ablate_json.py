"""Summarise tools/gpu_r04_zipf_ablate.sh's kernel traces (gpurun_out/r04_ablate/<variant>_<round>/
*_kernel_stats.csv) into the phases of records_bucket_kernel: pass 1 + scans (abl1), pass 2
scatter (abl2 - abl1), staged copy-out (abl3 - abl2), tiny statistics (tree - abl3).
Usage: python3 tools/ablate_json.py gpurun_out/r04_ablate > out.json"""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
runs = {}
for d in sorted(glob.glob(os.path.join(root, "*_*"))):
    if not os.path.isdir(d):
        continue
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "records_bucket_kernel" in r["Name"]:
                runs[os.path.basename(d)] = dict(bucket_kernel_avg_ms=float(r["AverageNs"]) / 1e6,
                                                 calls=int(r["Calls"]))


def mean(v):
    xs = [x["bucket_kernel_avg_ms"] for k, x in runs.items() if k.rsplit("_", 1)[0] == v]
    return sum(xs) / len(xs) if xs else None


a1, a2, a3, t = mean("abl1"), mean("abl2"), mean("abl3"), mean("tree")
out = dict(runs=runs)
if None not in (a1, a2, a3, t):
    out["phases_ms"] = dict(pass1_plus_scan=a1, pass2_scatter=a2 - a1, staged_copy_out=a3 - a2,
                            tiny_stats=t - a3, whole_kernel=t)
print(json.dumps(out, indent=1))
