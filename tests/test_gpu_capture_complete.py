"""GPU: completeness of the report-time flush of the live capture (capture.cpp, "Flush
completeness").  The reference drains every completed activity record before it computes
statistics -- cuptiActivityFlushAll(0) inside getStats (CuptiProfiler.cpp:136-146), after the
Detector's torch.cuda.synchronize() (straggler.py:234-243) -- so a report holds exactly the
kernels launched in its interval.  rocprofiler-sdk hands completions over on the runtime's
signal-handler thread, late when the host is loaded; the flush therefore waits for every job
dispatch counted at enqueue.  These cases check it where a timing heuristic would fail:

  * a known number of launches on two streams per interval, every host core kept busy by other
    processes through generate_report: each interval's num_calls equal the launched counts
    exactly, the next interval holds none of the previous one's records, no flush timed out;
  * reports on two threads at once (an external tracer's ingest loop against get_stats) never
    capture the library's own kernels as the job's (each thread is marked on its own).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nvidia-resiliency-ext-x_amd")
# mangled name of nvrx::stragglers_kernel(const double*, long, double, unsigned char*)
STRAG = "_ZN4nvrx17stragglers_kernelEPKdldPh"


def _child(code, env=None, timeout=300):
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {PKG!r})\n" + code],
                       capture_output=True, text=True, timeout=timeout, env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1][7:])


LOADED = r"""
import ctypes, json
from nvidia_resiliency_ext.straggler import cupti, ops, _native
cupti.enable_capture()  # before the first HIP call
import torch
from nvidia_resiliency_ext import straggler
D, S = straggler.Detector, straggler.Statistic
D.initialize(profiling_interval=1, report_time_interval=1e9)
small = torch.rand(1000, dtype=torch.float64, device="cuda")    # 4 blocks of 256
big = torch.rand(70000, dtype=torch.float64, device="cuda")     # 274 blocks
m1 = torch.empty(1000, dtype=torch.uint8, device="cuda")
m2 = torch.empty(70000, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
ops.stragglers(small, 0.5, out=m1); ops.stragglers(big, 0.5, out=m2)  # code objects loaded
torch.cuda.synchronize()
D.generate_report()
c0 = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c0))
got, want = [], []
for it in range(8):
    n1, n2 = 300 + 97 * it, 200 + 31 * it
    with D.detection_section("work", profile_cuda=True):
        for i in range(max(n1, n2)):  # interleaved on two streams, no synchronize
            if i < n1:
                ops.stragglers(small, 0.5, out=m1, stream=s1)
            if i < n2:
                ops.stragglers(big, 0.5, out=m2, stream=s2)
    rep = D.generate_report()  # synchronize + get_stats (the counted flush) + reset
    got.append({k: int(v[S.NUM]) for k, v in rep.local_kernel_summaries.items()})
    want.append({STRAG + "_blk_256_1_1_grid_4_1_1": n1, STRAG + "_blk_256_1_1_grid_274_1_1": n2})
c1 = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c1))
D.shutdown()
d = lambda f: getattr(c1, f) - getattr(c0, f)
print("RESULT " + json.dumps({"got": got, "want": want, "delivery": c1.delivery,
      "marking": c1.marking, "counted": d("counted_flushes"), "quiet": d("quiet_flushes"),
      "timeouts": d("flush_timeouts"), "abandoned": d("owed_abandoned"),
      "enqueues": d("enqueues_counted"), "flush_ms": d("flush_ns") / 1e6 / max(1, d("flushes")),
      "ring": d("ring_records"), "pool": d("pool_signals"), "chained": d("chained_signals"),
      "anomalies": c1.ring_anomalies}))
""".replace("STRAG", repr(STRAG))


def _busy(n):
    """n processes that keep a host core each busy (the box's CPU share is 16)."""
    return [subprocess.Popen([sys.executable, "-c", "while True: pass"]) for _ in range(n)]


DELIVERY = {"callback": 1, "queue": 3}
# queue delivery with a device ring of 64 records: most dispatches of an interval fall back to
# pooled HSA signals (the ring is full until the next harvest) -- the counts stay exact
RINGS = {"callback": None, "queue": None, "queue_ring64": "64"}


@pytest.mark.parametrize("mode", sorted(RINGS))
def test_flush_is_complete_under_host_load(mode):
    delivery = mode.split("_")[0]
    env = {"NVRX_CAPTURE_DELIVERY": delivery}
    if RINGS[mode]:
        env["NVRX_CAPTURE_RING"] = RINGS[mode]
    ncpu = len(os.sched_getaffinity(0))
    hogs = _busy(min(32, 2 * ncpu))
    try:
        out = _child(LOADED, env=env)
    finally:
        for h in hogs:
            h.kill()
        for h in hogs:
            h.wait()
    assert out["delivery"] == DELIVERY[delivery], out
    if delivery == "callback":  # counted through the external-correlation-id request
        assert out["marking"] == 1, out
    for i, (g, w) in enumerate(zip(out["got"], out["want"])):
        assert g == w, (i, g, w)  # exact per interval: none lost, none carried over
    assert out["counted"] >= 8 and out["quiet"] == 0, out
    assert out["timeouts"] == 0 and out["abandoned"] == 0, out
    if delivery == "queue":
        launched = sum(sum(w.values()) for w in out["want"])
        assert out["ring"] + out["pool"] == launched and out["anomalies"] == 0, out
        assert (out["pool"] > 0) == (mode == "queue_ring64"), out
    # every launch of the 8 intervals was counted at enqueue (the Detector's own kernels run
    # with the profiler stopped, or marked)
    assert out["enqueues"] == sum(sum(w.values()) for w in out["want"]), out


TWO_THREADS = r"""
import ctypes, json, threading
from nvidia_resiliency_ext.straggler import cupti, ops, _native
import torch
p = cupti.KernelProfiler(statsMaxLenPerKernel=8192, capture=True)
p.initialize()
names = ["ext_kernel_%d" % i for i in range(4)]
slots = [p.register_kernel(n) for n in names]
gen = p.generation
recs = torch.tensor([[slots[i % 4], 1000 + i] for i in range(4096)], dtype=torch.int32, device="cuda")
score = torch.rand(1000, dtype=torch.float64, device="cuda")
m = torch.empty(1000, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
p.start()  # the inputs above were made before: only the threads' launches below count
c0 = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c0))
N_INGEST, N_JOB = 400, 2000
stop = threading.Event()
def tracer():  # an external tracer's device ingest (the library's own copy kernel) on its own thread
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(N_INGEST):
            p.ingest(recs, s, generation=gen)
    s.synchronize()
def job():
    for _ in range(N_JOB):
        ops.stragglers(score, 0.5, out=m)
    torch.cuda.synchronize()
ts = [threading.Thread(target=tracer), threading.Thread(target=job)]
for t in ts:
    t.start()
reports = 0
while any(t.is_alive() for t in ts):  # get_stats (bucketing + statistics kernels) meanwhile
    p.get_stats()
    reports += 1
for t in ts:
    t.join()
torch.cuda.synchronize()
st = {k: v.num_calls for k, v in p.get_stats().items()}
c1 = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c1))
p.stop()
p.shutdown()
print("RESULT " + json.dumps({"stats": st, "reports": reports, "own": c1.own_kernels - c0.own_kernels,
                              "n_ingest": N_INGEST, "n_job": N_JOB}))
"""


def test_concurrent_reports_never_capture_own_kernels():
    """one process-wide marked thread let a second report's end unmark the first's
    kernels.  Ingest (own copy kernels) on one thread, get_stats on another, a job thread
    launching: the summaries hold the job's kernel and the ingested names, nothing else."""
    out = _child(TWO_THREADS)
    st = out["stats"]
    job_key = STRAG + "_blk_256_1_1_grid_4_1_1"
    assert st.get(job_key) == out["n_job"], st
    ingested = {k: v for k, v in st.items() if k.startswith("ext_kernel_")}
    # 400 x 4096 records over 4 names: each ring keeps its last 8192
    assert ingested == {f"ext_kernel_{i}": 8192 for i in range(4)}, ingested
    assert set(st) == {job_key} | set(ingested), sorted(st)  # no kernel of the library's own
    assert out["reports"] >= 2 and out["own"] > 0, out


DURATIONS = r"""
import ctypes, json
from nvidia_resiliency_ext.straggler import cupti, _native
import torch
p = cupti.KernelProfiler(statsMaxLenPerKernel=1024, capture=True)
p.initialize()
torch.cuda._sleep(1000)  # the spin kernel's code object loaded
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(40)]
p.start()
for a, b in ev:
    a.record()
    torch.cuda._sleep(2_000_000)  # ~1 ms of device spin
    b.record()
torch.cuda.synchronize()
st = {k: [v.num_calls, v.median, v.min, v.max] for k, v in p.get_stats().items()}
c = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c))
p.stop()
p.shutdown()
ms = sorted(a.elapsed_time(b) for a, b in ev)
print("RESULT " + json.dumps({"stats": st, "event_median_us": ms[len(ms) // 2] * 1e3, "delivery": c.delivery,
                              "ring": c.ring_records, "pool": c.pool_signals, "anomalies": c.ring_anomalies,
                              "chained": c.chained_signals}))
"""


@pytest.mark.parametrize("delivery", sorted(DELIVERY))
def test_captured_durations_match_event_timing(delivery):
    """A ~1 ms device spin launched 40 times between two timing events: the captured duration
    of each dispatch (the packet processor's timestamps) agrees with the events' elapsed time,
    which brackets the kernel plus its launch gap, in every delivery mode."""
    out = _child(DURATIONS, env={"NVRX_CAPTURE_DELIVERY": delivery})
    assert out["delivery"] == DELIVERY[delivery], out
    spin = {k: v for k, v in out["stats"].items() if "sleep" in k.lower() or "spin" in k.lower()}
    assert len(spin) == 1, out["stats"]
    (num, med, mn, mx), = spin.values()
    assert num == 40, out
    ev = out["event_median_us"]
    assert 0.9 * ev <= med <= 1.01 * ev, (med, ev)
    if delivery == "queue":  # device completion records, nothing past the expected values
        assert out["ring"] >= 40 and out["anomalies"] == 0, out


PROBE = os.path.join(ROOT, "tests", "native", "grid_probe.hsaco")
EXT_EVENTS = r"""
import ctypes, json
from nvidia_resiliency_ext.straggler import cupti, _native
import torch
p = cupti.KernelProfiler(statsMaxLenPerKernel=1024, capture=True)
p.initialize()
hip = ctypes.CDLL("libamdhip64.so")
mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
assert hip.hipModuleLoad(ctypes.byref(mod), PROBE.encode()) == 0
assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"nvrx_spin_alu") == 0
buf = torch.zeros(64, dtype=torch.float32, device="cuda")
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
a_out, a_n = ctypes.c_void_p(buf.data_ptr()), ctypes.c_uint32(400000)
params = (ctypes.c_void_p * 2)(ctypes.cast(ctypes.byref(a_out), ctypes.c_void_p),
                               ctypes.cast(ctypes.byref(a_n), ctypes.c_void_p))
hip.hipExtModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [
    ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
    ctypes.c_void_p, ctypes.c_uint32]
hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
def launch(ev=None):
    s, e = ev if ev else (None, None)
    rc = hip.hipExtModuleLaunchKernel(fn, 64, 1, 1, 64, 1, 1, 0, stream, params, None, s, e, 0)
    assert rc == 0, rc
launch()
torch.cuda.synchronize()
c0 = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c0))
evs = []
for _ in range(20):
    s, e = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipEventCreate(ctypes.byref(s)) == 0 and hip.hipEventCreate(ctypes.byref(e)) == 0
    evs.append((s, e))
p.start()
for ev in evs:
    launch(ev)  # the runtime times the kernel itself for these events
for _ in range(20):
    launch()
torch.cuda.synchronize()
st = {k: [v.num_calls, v.median] for k, v in p.get_stats().items()}
c1 = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c1))
p.stop()
p.shutdown()
ms = []
for s, e in evs:
    f = ctypes.c_float()
    assert hip.hipEventElapsedTime(ctypes.byref(f), s, e) == 0
    ms.append(f.value)
ms.sort()
print("RESULT " + json.dumps({"stats": st, "event_median_us": ms[len(ms) // 2] * 1e3,
                              "chained": c1.chained_signals - c0.chained_signals, "delivery": c1.delivery}))
""".replace("PROBE", repr(PROBE))


@pytest.mark.parametrize("delivery", sorted(DELIVERY))
def test_runtime_timed_launches_keep_their_event_timing(delivery):
    """hipExtModuleLaunchKernel with start / stop events: the runtime times that kernel itself (its
    own completion signal on the packet, which queue delivery chains behind a completion record of
    ours).  The events' elapsed time still measures the kernel, and the capture counts all 40
    launches with the same duration."""
    assert os.path.exists(PROBE), "build tests/native first (__graft_entry__.build())"
    out = _child(EXT_EVENTS, env={"NVRX_CAPTURE_DELIVERY": delivery})
    assert out["delivery"] == DELIVERY[delivery], out
    spin = {k: v for k, v in out["stats"].items() if k.startswith("nvrx_spin_alu")}
    assert len(spin) == 1, out["stats"]
    (num, med), = spin.values()
    assert num == 40, out
    ev = out["event_median_us"]
    assert med > 50 and 0.8 * med <= ev <= 1.3 * med, (med, ev, out["chained"])
    if delivery == "queue":  # ROCm 7.2 gives exactly the 20 event-timed packets a signal: chained
        assert out["chained"] == 20, out
