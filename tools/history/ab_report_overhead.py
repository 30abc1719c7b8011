"""A/B of the configs[1] report's fixed cost outside the stats kernel (MI355X).

Variants, each N back-to-back reports on the same resident inputs:
  two_graphs   -- ReportGraph.run() (stats graph, then scores + copy graph), event-polled wait
  one_graph    -- stats + scores + copy captured in ONE graph, event-polled wait
  *_events/_bracket -- the same with the bench's timing events (around the stats graph /
                  around the whole one-graph report)
  stats_only   -- the stats graph alone with a synchronize (the floor for a report)
Prints one JSON line of ms per report.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))

import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import batch, synth  # noqa: E402

R, K, S, CAP = 64, 2048, 10000, 8192
N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda:0")
ns = synth.synth_matrix(R, K, S, device=dev)
rep = batch.MatrixReporter(R, K, cap=CAP, thr_rel=0.8, thr_ind=0.8, device=dev)
g = rep.graph(ns, S)
one = torch.cuda.CUDAGraph()
with torch.cuda.graph(one):
    rep.compute_stats(ns, S)
    rep.compute_scores()
    rep.h_out.copy_(rep.out, non_blocking=True)

try:
    XA, XB = (torch.cuda.Event(enable_timing=True, external=True),
              torch.cuda.Event(enable_timing=True, external=True))
    onex = torch.cuda.CUDAGraph()
    with torch.cuda.graph(onex):
        XA.record()
        rep.compute_stats(ns, S)
        XB.record()
        rep.compute_scores()
        rep.h_out.copy_(rep.out, non_blocking=True)
    XERR = None
except Exception as e:  # noqa: BLE001
    onex, XERR = None, repr(e)
XMS = []

# the same through HIP directly: timing events recorded as external event nodes of the graph
import ctypes  # noqa: E402

HIP = ctypes.CDLL("libamdhip64.so")
HIP.hipEventRecordWithFlags.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
HIP.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
HIP.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
HA, HB = ctypes.c_void_p(), ctypes.c_void_p()
assert HIP.hipEventCreate(ctypes.byref(HA)) == 0 and HIP.hipEventCreate(ctypes.byref(HB)) == 0
HERR = []
try:
    onex = torch.cuda.CUDAGraph()
    with torch.cuda.graph(onex):
        sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        HERR.append(HIP.hipEventRecordWithFlags(HA, sh, 1))
        rep.compute_stats(ns, S)
        HERR.append(HIP.hipEventRecordWithFlags(HB, sh, 1))
        rep.compute_scores()
        rep.h_out.copy_(rep.out, non_blocking=True)
    if any(HERR):
        onex = None
except Exception as e:  # noqa: BLE001
    onex = None
    HERR.append(repr(e))


def timed(fn):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / N * 1e3


def one_graph():
    one.replay()
    batch._wait(dev)
    return rep._unpack()


EV = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N + 10)]
_i = [0]


def two_graphs_events():
    a, b = EV[_i[0] % len(EV)]
    _i[0] += 1
    a.record()
    g.run_stats()
    b.record()
    return g.run_rest()


def one_graph_bracket():
    a, b = EV[_i[0] % len(EV)]
    _i[0] += 1
    a.record()
    one.replay()
    b.record()
    batch._wait(dev)
    return rep._unpack()


def one_graph_ext_events():
    onex.replay()
    batch._wait(dev)
    ms = ctypes.c_float()
    rc = HIP.hipEventElapsedTime(ctypes.byref(ms), HA, HB)
    XMS.append(ms.value if rc == 0 else -float(rc))
    return rep._unpack()


def stats_timed_alone():
    a, b = EV[0]
    a.record()
    g.stats.replay()
    b.record()
    torch.cuda.synchronize()
    XMS2.append(a.elapsed_time(b))


XMS2 = []


def stats_only():
    g.stats.replay()
    torch.cuda.synchronize()


VARIANTS = [("two_graphs", g.run), ("two_graphs_events", two_graphs_events), ("one_graph", one_graph),
            ("one_graph_bracket", one_graph_bracket), ("stats_only", stats_only),
            ("stats_timed_alone", stats_timed_alone)]
if onex is not None:
    VARIANTS.append(("one_graph_ext_events", one_graph_ext_events))
out = {}
for rnd in range(3):
    for name, fn in VARIANTS:
        out.setdefault(name, []).append(timed(fn))
out = {k: [round(x, 4) for x in v] for k, v in out.items()}
out["ext_event_err"] = XERR
out["hip_ext_err"] = HERR
if XMS:
    out["ext_kernel_ms"] = [round(sum(XMS) / len(XMS), 4), round(min(XMS), 4), round(max(XMS), 4)]
if XMS2:
    out["stats_alone_event_ms"] = [round(sum(XMS2) / len(XMS2), 4), round(min(XMS2), 4)]
print(json.dumps(out))
