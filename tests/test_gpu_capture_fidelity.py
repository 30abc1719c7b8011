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
