"""Average per-dispatch counter values of the stats kernels from rocprofv3 --pmc output dirs."""
import collections
import csv
import glob
import sys

def short(name):
    base = name.replace("(anonymous namespace)::", "").split("(")[0]
    base = base.replace("void ", "").replace("nvrx::", "")
    return base[-42:]


for d in sys.argv[1:]:
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if any(t in r["Kernel_Name"] for t in ("seg_", "records_", "classify")):
                agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    waves = {k[0]: sum(v) / len(v) for k, v in agg.items() if k[1] == "SQ_WAVES"}
    for (kn, c), v in sorted(agg.items()):
        m = sum(v) / len(v)
        w = waves.get(kn)
        print(f"{kn:42s} {c:24s} {m:16.0f}" + (f"  per-wave {m / w:10.2f}" if w else ""))
