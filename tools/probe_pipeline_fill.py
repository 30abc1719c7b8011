"""Where the fixed cost of a short timed region of pipelined configs[1] reports goes: the host
time at which each report lands, for a 20- and a 100-report run back to back (same pipe), after
the bench's own warm-up; prints per-report landing intervals (ms).  Usage: python3
tools/probe_pipeline_fill.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from nvidia_resiliency_ext.straggler import batch  # noqa: E402

dev = torch.device("cuda:0")
cfg = bench.C2
ns, kidx = bench.make_shard(cfg["R"], cfg["K"], cfg["s_push"], 1, 0, dev)
rep = batch.MatrixReporter(cfg["R"], len(kidx), cap=cfg["cap"], thr_rel=bench.THR, thr_ind=bench.THR,
                           device=dev)
for _ in range(5):
    rep.report(ns, cfg["s_push"])
pipe = rep.pipelined(ns, cfg["s_push"])
for _ in range(5):
    pipe.submit()
    pipe.collect()
out = {}
for idle_ms, steps in ((0, 20), (0, 100), (50, 20), (50, 100), (-1, 20), (0, 20)):
    if idle_ms < 0:  # a long busy period right before: 150 reports, then the 20 timed
        for _ in range(150):
            pipe.submit()
            pipe.collect()
        idle_ms = 0
        tag = "hot"
    else:
        tag = ""
    if True:
        torch.cuda.synchronize()
        time.sleep(idle_ms / 1e3)
        t0 = time.perf_counter()
        land = []
        pipe.submit()
        for i in range(steps):
            if i + 1 < steps:
                pipe.submit()
            pipe.collect()
            land.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        d = np.diff([0.0] + land) * 1e3
        out[f"{tag}idle{idle_ms}_n{steps}" + ("_again" if f"{tag}idle{idle_ms}_n{steps}" in out else "")] = dict(ms_per_report=el / steps * 1e3, first=float(d[0]),
                                              second=float(d[1]), median=float(np.median(d[2:])),
                                              last=float(d[-1]))
# host cost of the calls themselves (20-report burst): submit() = graph replay + event record
torch.cuda.synchronize()
sub, col = [], []
t0 = time.perf_counter()
a = time.perf_counter(); pipe.submit(); sub.append(time.perf_counter() - a)
for i in range(20):
    if i + 1 < 20:
        a = time.perf_counter(); pipe.submit(); sub.append(time.perf_counter() - a)
    a = time.perf_counter(); pipe.collect(); col.append(time.perf_counter() - a)
torch.cuda.synchronize()
out["host_us"] = dict(submit=[round(x * 1e6, 1) for x in sub[:4]], submit_median=float(np.median(sub) * 1e6),
                      collect=[round(x * 1e6, 1) for x in col[:4]], collect_median=float(np.median(col) * 1e6))
g = pipe.full[0]
out["raw_graph_exec"] = hasattr(g, "raw_cuda_graph_exec")
print(json.dumps(out, indent=1))
