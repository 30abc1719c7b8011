"""Probe (not part of the library): the live capture in queue delivery while rocprofv3 traces the
same process (run as `rocprofv3 --kernel-trace -- python3 tools/probe_rocprof_coexist.py`).  Prints
whether our capture saw the launches; rocprofv3's own trace shows whether it did."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
from nvidia_resiliency_ext.straggler import cupti, ops, _native  # noqa: E402

p = cupti.KernelProfiler(statsMaxLenPerKernel=1024, capture=True)
import torch  # noqa: E402

p.initialize()
score = torch.rand(1000, dtype=torch.float64, device="cuda")
m = torch.empty(1000, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
p.start()
for _ in range(50):
    ops.stragglers(score, 0.5, out=m)
torch.cuda.synchronize()
st = {k: v.num_calls for k, v in p.get_stats().items()}
c = _native.CaptureCounters()
_native.lib().nvrx_capture_stats(ctypes.byref(c))
p.stop()
print("RESULT " + json.dumps({"available": cupti.capture_available(), "stats": st, "delivery": c.delivery,
                              "queues": c.queues, "ring": c.ring_records}))
