"""GPU: live kernel-dispatch capture through rocprofiler-sdk (capture.cpp), the replacement
of the CUPTI activity path (CuptiProfiler.cpp:96-203; test_cupti_ext.py's capture checks).

rocprofiler-sdk tools configure when the ROCm runtime initialises, so each case runs in a
fresh child process that creates the profiler before its first HIP call."""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
sys.path.insert(0, %(pkg)r)
from nvidia_resiliency_ext.straggler import cupti, ops
import torch
p = cupti.KernelProfiler(statsMaxLenPerKernel=%(cap)d, capture=True)
out = {"available": cupti.capture_available()}
p.initialize()
p.start()
x = torch.randn(256, 256, device="cuda")
for _ in range(5):
    y = x @ x
score = torch.rand(1000, dtype=torch.float64, device="cuda")
for _ in range(%(nstrag)d):
    ops.stragglers(score, 0.5)
torch.cuda.synchronize()
p.stop()
for _ in range(3):
    ops.stragglers(score, 0.5)  # stopped: not captured
torch.cuda.synchronize()
out["stats"] = {k: [v.num_calls, v.min, v.median, v.max] for k, v in p.get_stats().items()}
p.reset()
out["after_reset"] = len(p.get_stats())
print("RESULT " + json.dumps(out))
"""


def _run(cap, nstrag):
    code = CHILD % dict(pkg=os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"), cap=cap, nstrag=nstrag)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_dispatch_capture_keys_counts_and_start_stop():
    out = _run(cap=64, nstrag=7)
    assert out["available"]
    stats = out["stats"]
    key_re = re.compile(r"^(.+)_blk_(\d+)_(\d+)_(\d+)_grid_(\d+)_(\d+)_(\d+)$")
    assert stats and all(key_re.match(k) for k in stats), list(stats)[:5]
    strag = {k: v for k, v in stats.items() if "stragglers" in k}
    assert len(strag) == 1, list(stats)
    (k, (num, mn, med, mx)), = strag.items()
    assert num == 7                        # the 3 launches after stop() are not captured
    assert 0 < mn <= med <= mx < 1e5       # microseconds
    # torch's GEMM: 5 launches (one key per distinct launch shape)
    assert sum(v[0] for kk, v in stats.items() if "stragglers" not in kk) >= 5
    assert list(stats) == sorted(stats)    # std::map order (CuptiProfiler.cpp:137-145)
    assert out["after_reset"] == 0


def test_dispatch_capture_ring_cap():
    # statsMaxLenPerKernel=4: only the last 4 dispatches of a kernel count (num_calls == 4)
    out = _run(cap=4, nstrag=9)
    strag = [v for k, v in out["stats"].items() if "stragglers" in k]
    assert strag and strag[0][0] == 4


ASYNC_CHILD = r"""
import json, sys
sys.path.insert(0, %(pkg)r)
from nvidia_resiliency_ext.straggler import cupti, ops
import torch
p = cupti.KernelProfiler(statsMaxLenPerKernel=1024, capture=True)
p.initialize()
x = torch.randn(4096, 4096, device="cuda")
score = torch.rand(1000, dtype=torch.float64, device="cuda")
torch.cuda.synchronize()
p.start()
for _ in range(40):
    y = x @ x                 # keeps the queue busy well past stop()
for _ in range(7):
    ops.stragglers(score, 0.5)
p.stop()                      # no synchronize: the 7 launches have not run yet
pending = not torch.cuda.current_stream().query()
torch.cuda.synchronize()
st = p.get_stats()
out = {"pending_at_stop": pending,
       "strag": sum(v.num_calls for k, v in st.items() if "stragglers" in k)}
p.reset()
for _ in range(5):
    ops.stragglers(score, 0.5)  # stopped: not captured
torch.cuda.synchronize()
out["after_reset"] = len(p.get_stats())
print("RESULT " + json.dumps(out))
"""


def test_dispatch_completing_after_stop_is_captured():
    code = ASYNC_CHILD % dict(pkg=os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1][7:])
    assert out["pending_at_stop"]
    assert out["strag"] == 7      # enqueued while started, completed after stop
    assert out["after_reset"] == 0


BOUND_CHILD = r"""
import ctypes, json, sys
sys.path.insert(0, %(pkg)r)
from nvidia_resiliency_ext.straggler import cupti, ops, _native
import torch
p = cupti.KernelProfiler(statsMaxLenPerKernel=8192, capture=True)
p.initialize()
score = torch.rand(1000, dtype=torch.float64, device="cuda")
# started for a long time with no stop or flush: at most NVRX_CAPTURE_MAX_PENDING dispatches wait
p.start()
for _ in range(%(n)d):
    ops.stragglers(score, 0.5)
torch.cuda.synchronize()
c = _native.CaptureCounters()
_native.lib().nvrx_capture_stats(ctypes.byref(c))
dropped_while_started = c.dropped
p.stop()
num = sum(v.num_calls for k, v in p.get_stats().items() if "stragglers" in k)
p.reset()
# a section per step (start / stop, no flush): the start-time harvest keeps the ring turning
for _ in range(%(n)d):
    p.start()
    ops.stragglers(score, 0.5)
    p.stop()
torch.cuda.synchronize()
num2 = sum(v.num_calls for k, v in p.get_stats().items() if "stragglers" in k)
_native.lib().nvrx_capture_stats(ctypes.byref(c))
print("RESULT " + json.dumps(dict(dropped=dropped_while_started, num=num, num2=num2,
                                  dropped_after=c.dropped, delivery=c.delivery)))
"""


def test_queue_delivery_pending_bound_drops_and_counts():
    """a profiler left started never holds more than NVRX_CAPTURE_MAX_PENDING dispatches
    (the rest go out without a completion record and count as `dropped`, as the reference's buffer
    pool drops records when it is exhausted, BufferPool.cpp:44-52); with a ring of 2,048 records a
    start / stop per kernel (harvested at start once half the ring waits) loses nothing."""
    code = BOUND_CHILD % dict(pkg=os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"), n=3000)
    env = dict(os.environ, NVRX_CAPTURE_MAX_PENDING="2048", NVRX_CAPTURE_RING="2048")
    env.pop("NVRX_CAPTURE_DELIVERY", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1][7:])
    assert out["delivery"] == 3
    assert out["num"] == 2048 and out["dropped"] == 3000 - 2048, out
    assert out["num2"] == 3000 and out["dropped_after"] == out["dropped"], out
