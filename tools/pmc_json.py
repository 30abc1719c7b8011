"""profiles/pmc_*.json from tools/gpu_profile.sh's --pmc passes (median over dispatches).

FETCH_SIZE is doubled (gfx950 reports half of wide coalesced streaming reads; Infinity-Cache hits
count as memory-side traffic too) and KB are x 1024, per MI355X_MICROARCH.md's HBM section.
Usage: python tools/pmc_json.py <gpurun_out/PROF_TAG> [c2|c3|zipf ...]"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

src = sys.argv[1]
which = sys.argv[2:] or ["c2", "c3", "zipf"]
NOTE = ("rocprofv3 --pmc, one counter group per run; median over dispatches; FETCH_SIZE doubled per "
        "MI355X_MICROARCH.md; KB x 1024")


def short(name):
    base = name.replace("(anonymous namespace)::", "").split("(")[0]
    return base.replace("void ", "").replace("nvrx::", "").strip()


def counters(sub):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{src}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: (statistics.median(v), len(v)) for k, v in vals.items()}


def trace_ms(sub):
    out = {}
    for f in glob.glob(f"{src}/{sub}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Name"])] = float(r["AverageNs"]) * 1e-6
    return out


def one_kernel(prefix, kernel_sub, alg, workload, out_name):
    c = {**counters(f"{prefix}_FETCH_SIZE"), **counters(f"{prefix}_WRITE_SIZE")}
    keys = [k for k, cn in c if kernel_sub in k and cn == "FETCH_SIZE"]
    assert keys, f"no {kernel_sub} dispatches under {src}/{prefix}_FETCH_SIZE"
    k = keys[0]
    (fetch, n), (write, _) = c[(k, "FETCH_SIZE")], c[(k, "WRITE_SIZE")]
    hbm = (2 * fetch + write) * 1024
    out = dict(workload=workload, kernel=k, method=NOTE, fetch_size_kb_median=fetch,
               write_size_kb_median=write, dispatches=n, hbm_bytes_per_launch=hbm,
               alg_bytes_per_launch=alg, traffic_over_alg=hbm / alg)
    json.dump(out, open(f"profiles/{out_name}", "w"), indent=1)
    print(out_name, json.dumps(out))


if "c2" in which:  # configs[1]: 4 B per retained sample + 24 B of statistics per segment
    one_kernel("c2", "seg_stats_lean_group_kernel<128", 4 * 64 * 2048 * 8192 + 24 * 64 * 2048,
               "c2: 64 ranks x 2048 kernels x 8192 retained samples (S_push 10000)",
               "pmc_c2_segment_stats.json")
if "c3" in which:
    one_kernel("c3", "seg_stats_lean_group_kernel<16", 4 * 4096 * 2048 * 1024 + 24 * 4096 * 2048,
               "configs[2]: 4096 ranks x 2048 kernels x 1024 samples", "pmc_configs2_segment_stats.json")
if "zipf" in which:  # configs[3]: 8 B per record
    R = int(os.environ.get("AB_R", 16384))
    NREC = R * 47_482
    c = {}
    for sub in ("zipf_FETCH_SIZE", "zipf_WRITE_SIZE", "zipf_TCC_HIT_sum"):
        c.update({k: v[0] for k, v in counters(sub).items()})
    ms = trace_ms("zipf_trace")
    rows = {}
    for k in sorted({k for k, _ in c} | set(ms)):
        if not any(t in k for t in ("records_", "seg_stats", "classify", "kref")) or "synth" in k:
            continue  # the statistics path only
        fetch, write = c.get((k, "FETCH_SIZE")), c.get((k, "WRITE_SIZE"))
        hit, miss = c.get((k, "TCC_HIT_sum")), c.get((k, "TCC_MISS_sum"))
        row = {"avg_ms": ms.get(k)}
        if fetch is not None and write is not None:
            row.update(fetch_bytes_x2=2 * fetch * 1024, write_bytes=write * 1024,
                       bytes_per_record=(2 * fetch + write) * 1024 / NREC)
            if row["avg_ms"]:
                row["memory_side_GBps"] = (2 * fetch + write) * 1024 / (row["avg_ms"] * 1e-3) / 1e9
        if hit is not None and miss is not None and hit + miss > 0:
            row["l2_hit_rate"] = hit / (hit + miss)
        rows[k] = row
    common = {"workload": f"configs[3]: {R} Zipf record streams, {NREC} records of 8 B",
              "alg_bytes_per_record": 8, "alg_bytes_per_launch": 8 * NREC,
              "method": NOTE + f"; tools/ab_zipf.py (AB_R={R}); kernel times from its --kernel-trace pass"}
    for name, part in (("bucket", {k: v for k, v in rows.items() if k.startswith("records_")}),
                       ("stats", {k: v for k, v in rows.items() if not k.startswith("records_")})):
        tot = {f: sum(v.get(f, 0.0) or 0.0 for v in part.values())
               for f in ("avg_ms", "fetch_bytes_x2", "write_bytes")}
        tot["bytes_per_record"] = (tot["fetch_bytes_x2"] + tot["write_bytes"]) / NREC
        json.dump(dict(common, kernels=part, total=tot), open(f"profiles/pmc_zipf_{name}.json", "w"), indent=1)
        print(name, json.dumps(tot))
