"""GPU: fidelity of the live kernel-dispatch capture (capture.cpp) against the reference's CUPTI
path, each case in a fresh child process that configures capture before its first HIP call:

  * graph replay: profiling a replayed torch.cuda.CUDAGraph gives the same keys and counts as
    the same kernels launched one by one (test_cupti_ext.py:136-188);
  * composite keys pinned for launches of known block / grid dims ("%s_blk_%d_%d_%d_grid_%d_%d_%d"
    with the grid in BLOCKS, CuptiProfiler.cpp:182-185; rocprofiler reports it in work-items);
  * Detector(profiling_interval=2) profiles 2 of 4 section entries (test_det_section_api.py:83-103)
    and profile_cuda=False captures nothing (:105-123);
  * the drain of staged records at stop() (bufferSize watermark) keeps every record and records
    nothing of its own; profilers destroyed while dispatch records are still being delivered.
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


GRAPH = r"""
import json
from nvidia_resiliency_ext.straggler import cupti, ops
import torch
p = cupti.KernelProfiler(statsMaxLenPerKernel=1024, capture=True)
p.initialize()
model = torch.nn.Sequential(torch.nn.Linear(256, 256, bias=False), torch.nn.ReLU(),
                            torch.nn.Linear(256, 64, bias=False), torch.nn.Sigmoid()).cuda()
x = torch.randn(256, 256, device="cuda")
score = torch.rand(1000, dtype=torch.float64, device="cuda")
big = torch.rand(70000, dtype=torch.float64, device="cuda")
m1 = torch.empty(1000, dtype=torch.uint8, device="cuda")
m2 = torch.empty(70000, dtype=torch.uint8, device="cuda")
def body():
    y = model(x)
    for _ in range(3):
        ops.stragglers(score, 0.5, out=m1)
    ops.stragglers(big, 0.5, out=m2)
    return y
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):  # warm-up outside the capture (not profiled: stopped)
    body()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
torch.cuda.synchronize()
p.start()
for _ in range(4):
    g.replay()
torch.cuda.synchronize()
with_graph = {k: v.num_calls for k, v in p.get_stats().items()}
p.reset()
for _ in range(4):
    body()
torch.cuda.synchronize()
no_graph = {k: v.num_calls for k, v in p.get_stats().items()}
p.reset()
p.stop()
p.shutdown()
print("RESULT " + json.dumps({"graph": with_graph, "seq": no_graph,
                              "available": cupti.capture_available()}))
"""


def test_graph_replay_captures_like_sequential_launches():
    out = _child(GRAPH)
    assert out["available"]
    seq, graph = out["seq"], out["graph"]
    assert seq, "nothing captured"
    for k, n in seq.items():  # test_cupti_ext.py:183-188
        assert k in graph, (k, sorted(graph))
        assert graph[k] == n, k
    # our own launches, with known dims: 256-thread blocks, ceil(n / 256) blocks
    assert seq[f"{STRAG}_blk_256_1_1_grid_4_1_1"] == 12
    assert seq[f"{STRAG}_blk_256_1_1_grid_274_1_1"] == 4
    assert graph == seq


SECTIONS = r"""
import json
from nvidia_resiliency_ext.straggler import cupti
cupti.enable_capture()  # before the first HIP call
import torch
from nvidia_resiliency_ext import straggler
out = {}
for interval, profile_cuda in ((2, True), (1, False)):
    straggler.Detector.initialize(profiling_interval=interval)
    a = torch.randn(1000, 1000, device="cuda")
    b = torch.randn(1000, 1000, device="cuda")
    _ = torch.matmul(a, b)  # first call outside the sections (hipBLASLt's one-time workspace fill)
    torch.cuda.synchronize()
    for _ in range(4):
        with straggler.Detector.detection_section(name="one", profile_cuda=profile_cuda):
            _ = torch.matmul(a, b)
    torch.cuda.synchronize()
    rep = straggler.Detector.generate_report()
    S = straggler.Statistic
    out[f"{interval}_{profile_cuda}"] = {
        "kernels": {k: v[S.NUM] for k, v in rep.local_kernel_summaries.items()},
        "section_num": rep.local_section_summaries["one"][S.NUM]}
    straggler.Detector.shutdown()
print("RESULT " + json.dumps(out))
"""


def test_profiling_interval_and_profile_cuda_false():
    out = _child(SECTIONS)
    periodic, off = out["2_True"], out["1_False"]
    # 2 of 4 matmuls profiled: every kernel of the matmul counted twice (test_det_section_api
    # .py:95-103 expects the one GEMM kernel CUDA runs, NUM == 2)
    assert periodic["kernels"] and all(n == 2 for n in periodic["kernels"].values()), periodic
    assert periodic["section_num"] == 2
    assert off["kernels"] == {} and off["section_num"] == 4  # :105-123


DRAIN = r"""
import json
from nvidia_resiliency_ext.straggler import cupti, ops
import torch
out = {}
# bufferSize 8 KiB: at stop(), 1024 or more delivered records move to the device log
p = cupti.KernelProfiler(bufferSize=8 * 1024, statsMaxLenPerKernel=8192, capture=True)
p.initialize()
score = torch.rand(1000, dtype=torch.float64, device="cuda")
m = torch.empty(1000, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
for step in range(50):  # 50 sections of 100 launches
    p.start()
    for _ in range(100):
        ops.stragglers(score, 0.5, out=m)
    p.stop()
    if step % 10 == 9:
        torch.cuda.synchronize()
        cupti.N.call("nvrx_capture_flush")  # delivered -> staged; the next stop drains them
torch.cuda.synchronize()
st = p.get_stats()
out["keys"] = sorted(st)
out["num"] = {k: v.num_calls for k, v in st.items()}
p.close()
# profilers destroyed while their dispatch records are still being delivered (each close
# flushes the capture buffer into the handle being destroyed)
for i in range(25):
    q = cupti.KernelProfiler(statsMaxLenPerKernel=64, capture=True)
    q.initialize()
    q.start()
    for _ in range(400):
        ops.stragglers(score, 0.5, out=m)
    q.close()
torch.cuda.synchronize()
cupti.N.call("nvrx_capture_flush")  # records of the last launches: no profiler to take them
q = cupti.KernelProfiler(statsMaxLenPerKernel=64, capture=True)
q.initialize()
q.start()
for _ in range(10):
    ops.stragglers(score, 0.5, out=m)
torch.cuda.synchronize()
q.stop()
out["after"] = {k: v.num_calls for k, v in q.get_stats().items()}
q.close()
print("RESULT " + json.dumps(out))
"""


def test_drain_at_stop_and_destroy_while_delivering():
    out = _child(DRAIN)
    key = f"{STRAG}_blk_256_1_1_grid_4_1_1"
    assert out["num"].get(key) == 5000, out["num"]
    assert not [k for k in out["keys"] if "rocclr" in k], out["keys"]  # nothing of our own
    assert out["after"] == {key: 10}


PROBE = os.path.join(ROOT, "tests", "native", "grid_probe.hsaco")

RUNTIME = r"""
import ctypes, json, os
from nvidia_resiliency_ext.straggler import cupti, ops, _native
import torch
p = cupti.KernelProfiler(statsMaxLenPerKernel=1024, capture=True)
p.initialize()
hip = ctypes.CDLL("libamdhip64.so")
src = torch.rand(1 << 20, device="cuda")
dst = torch.empty_like(src)
score = torch.rand(1000, dtype=torch.float64, device="cuda")
m = torch.empty(1000, dtype=torch.uint8, device="cuda")
buf = torch.zeros(1024, dtype=torch.int32, device="cuda")
mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
assert hip.hipModuleLoad(ctypes.byref(mod), PROBE.encode()) == 0
assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"nvrx_grid_probe") == 0
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
a_out, a_n = ctypes.c_void_p(buf.data_ptr()), ctypes.c_uint32(1000)
params = (ctypes.c_void_p * 2)(ctypes.cast(ctypes.byref(a_out), ctypes.c_void_p),
                               ctypes.cast(ctypes.byref(a_n), ctypes.c_void_p))
hip.hipExtModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [
    ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
    ctypes.c_void_p, ctypes.c_uint32]
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
def section():
    dst.copy_(src)  # same device, contiguous: hipMemcpyAsync D2D (a runtime blit kernel)
    rc = hip.hipMemsetAsync(ctypes.c_void_p(dst.data_ptr()), 0, dst.numel() * 4, stream)
    assert rc == 0, ("hipMemsetAsync", rc)
    ops.stragglers(score, 0.5, out=m)  # the one real kernel: 256 threads, 4 blocks
    # a module kernel through the ext launch (global size in work-items): 1024 over workgroups
    # of 256 = 4 blocks.  (HIP refuses a global size that is not a multiple of the workgroup,
    # (round 4 probe, profiles/r05/README.md 3.6), so a partial last block -- counted by the capture's ceil, as
    # CUPTI's gridX counts it -- cannot be produced through HIP)
    rc = hip.hipExtModuleLaunchKernel(fn, 1024, 1, 1, 256, 1, 1, 0, stream, params, None,
                                      None, None, 0)
    hip.hipGetErrorString.restype = ctypes.c_char_p
    assert rc == 0, ("hipExtModuleLaunchKernel", rc, hip.hipGetErrorString(rc))
section()  # warm-up, stopped: nothing recorded
torch.cuda.synchronize()
c0 = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c0))
p.start()
for _ in range(3):
    section()
torch.cuda.synchronize()
stats = {k: v.num_calls for k, v in p.get_stats().items()}
c1 = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c1))
p.stop()
p.shutdown()
assert buf[:1000].tolist() == list(range(1000))
print("RESULT " + json.dumps({"stats": stats, "available": cupti.capture_available(),
                              "runtime": c1.runtime_kernels - c0.runtime_kernels}))
""".replace("PROBE", repr(PROBE))


def test_runtime_copies_and_fills_are_not_kernels():
    """CUPTI_ACTIVITY_KIND_CONCURRENT_KERNEL only (CuptiProfiler.cpp:118, 179): a section of
    copy_ + hipMemsetAsync + two kernels (one launched through the module / ext API with its
    global size in work-items) yields exactly the two kernels' keys (:182-185).  The capture's
    grid dims are ceil(grid_size / workgroup_size), as CUPTI's gridX counts a partial last block;
    that ceil branch cannot be reached through HIP (it refuses a global size that is not a
    multiple of the workgroup, round 4 probe), so only whole blocks are exercised."""
    assert os.path.exists(PROBE), "build tests/native first (__graft_entry__.build())"
    out = _child(RUNTIME)
    assert out["available"]
    assert out["stats"] == {f"{STRAG}_blk_256_1_1_grid_4_1_1": 3,
                            "nvrx_grid_probe_blk_256_1_1_grid_4_1_1": 3}, out["stats"]
    assert out["runtime"] >= 6, out  # the copies and fills were dispatched, and left out
    kept = _child(RUNTIME, env={"NVRX_CAPTURE_RUNTIME_KERNELS": "1"})
    blits = {k: n for k, n in kept["stats"].items() if k.startswith("__amd_rocclr_")}
    assert blits and sum(blits.values()) >= 6, kept["stats"]
    assert kept["runtime"] == 0


CONCURRENT = r"""
import ctypes, json, threading
from nvidia_resiliency_ext.straggler import cupti, ops, _native
import torch
p = cupti.KernelProfiler(statsMaxLenPerKernel=8192, capture=True)
p.initialize()
score = torch.rand(1000, dtype=torch.float64, device="cuda")
m = torch.empty(1000, dtype=torch.uint8, device="cuda")
ops.stragglers(score, 0.5, out=m)
torch.cuda.synchronize()
c0 = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c0))
p.start()
N = 3000
go = threading.Event()
def launcher():
    go.wait()
    for i in range(N):
        ops.stragglers(score, 0.5, out=m)
    torch.cuda.synchronize()
t = threading.Thread(target=launcher)
t.start()
go.set()
reports = 0
while t.is_alive():  # reports while the other thread launches (its kernels must all count)
    p.get_stats()
    reports += 1
t.join()
torch.cuda.synchronize()
stats = {k: v.num_calls for k, v in p.get_stats().items()}
c1 = _native.CaptureCounters(); _native.lib().nvrx_capture_stats(ctypes.byref(c1))
p.stop()
p.shutdown()
print("RESULT " + json.dumps({"stats": stats, "reports": reports,
                              "own": c1.own_kernels - c0.own_kernels}))
"""


def test_reports_leave_out_their_own_kernels_but_not_other_threads():
    """get_stats runs HIP kernels; they are not the job's (the reference's getStats is host code)
    and are left out by thread, so kernels another thread launches DURING the reports are all
    captured (CUPTI stays enabled through getStats, CuptiProfiler.cpp:136-146)."""
    out = _child(CONCURRENT)
    assert out["stats"] == {f"{STRAG}_blk_256_1_1_grid_4_1_1": 3000}, out
    assert out["reports"] >= 2 and out["own"] > 0, out
