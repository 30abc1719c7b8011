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
for idle_ms in (0, 50):
    for steps in (20, 100):
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
        out[f"idle{idle_ms}_n{steps}"] = dict(ms_per_report=el / steps * 1e3, first=float(d[0]),
                                              second=float(d[1]), median=float(np.median(d[2:])),
                                              last=float(d[-1]))
print(json.dumps(out, indent=1))
