"""profiles/pmc_zipf_{bucket,stats}.json from tools/pmc_zipf_traffic.sh's passes.

Per kernel of the configs[3] record-stream statistics (median over dispatches): FETCH_SIZE x2
(gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md HBM section; note that
Infinity-Cache hits are counted too), WRITE_SIZE, L2 hit rate, and bytes per record against the
8 B/record algorithmic figure.  Usage: python tools/pmc_zipf_json.py [dir] [tag]."""
import collections
import csv
import glob
import json
import os
import statistics
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_zt"
tag = sys.argv[2] if len(sys.argv) > 2 else ""
R, K = int(os.environ.get("AB_R", 16384)), 2048
RECS_PER_STREAM = 47_482
NREC = R * RECS_PER_STREAM


def short(name):
    base = name.replace("(anonymous namespace)::", "").split("(")[0]
    return base.replace("void ", "").replace("nvrx::", "").strip()


def counters(sub):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{src}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def trace():
    out = {}
    for f in glob.glob(f"{src}/trace/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Name"])] = float(r["AverageNs"]) * 1e-6
    return out


c = {}
for sub in ("pmc_FETCH_SIZE", "pmc_WRITE_SIZE", "pmc_TCC_HIT_sum"):
    c.update(counters(sub))
ms = trace()
kernels = sorted({k for k, _ in c} | set(ms))
rows = {}
for k in kernels:
    if not any(t in k for t in ("records_", "seg_stats", "classify", "kref")) or "synth" in k:
        continue  # the stats path only (synth_records_kernel generates the input)
    fetch = c.get((k, "FETCH_SIZE"))
    write = c.get((k, "WRITE_SIZE"))
    hit, miss = c.get((k, "TCC_HIT_sum")), c.get((k, "TCC_MISS_sum"))
    row = {"avg_ms": ms.get(k)}
    if fetch is not None:
        row["fetch_bytes_x2"] = 2 * fetch * 1024
    if write is not None:
        row["write_bytes"] = write * 1024
    if fetch is not None and write is not None:
        row["bytes_per_record"] = (2 * fetch + write) * 1024 / NREC
        if row["avg_ms"]:
            row["memory_side_GBps"] = (2 * fetch + write) * 1024 / (row["avg_ms"] * 1e-3) / 1e9
    if hit is not None and miss is not None and hit + miss > 0:
        row["l2_hit_rate"] = hit / (hit + miss)
    rows[k] = row

method = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum+TCC_MISS_sum in separate passes over "
          f"tools/ab_zipf.py (AB_R={R}: {R} streams x {RECS_PER_STREAM} records, {K} slots, cap 8192); "
          "median over dispatches; FETCH_SIZE doubled per MI355X_MICROARCH.md (Infinity-Cache hits "
          "are counted as memory-side traffic too); KB x 1024; kernel times from the --kernel-trace "
          "--stats pass of the same script")
common = {"workload": f"configs[3]: {R} Zipf record streams, {NREC} records of 8 B",
          "alg_bytes_per_record": 8, "alg_bytes_per_launch": 8 * NREC, "method": method}
bucket = {k: v for k, v in rows.items() if k.startswith("records_")}
stats = {k: v for k, v in rows.items() if not k.startswith("records_")}
for name, part in (("bucket", bucket), ("stats", stats)):
    tot = {f: sum(v.get(f, 0.0) or 0.0 for v in part.values())
           for f in ("avg_ms", "fetch_bytes_x2", "write_bytes")}
    tot["bytes_per_record"] = (tot["fetch_bytes_x2"] + tot["write_bytes"]) / NREC
    doc = dict(common, kernels=part, total=tot)
    path = f"profiles/pmc_zipf_{name}{tag}.json"
    json.dump(doc, open(path, "w"), indent=1)
    print(path)
    print(json.dumps(doc, indent=1))
