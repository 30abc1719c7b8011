"""Diagnostics of the live capture on the GPU box: do the dispatch records of many launches all
arrive?  DIAG_N launches split over DIAG_SECTIONS start/stop sections, a capture flush every
DIAG_FLUSH_EVERY sections (0: none), DIAG_SYNC_EVERY sections a device synchronize;
nvrx_capture_stats (CaptureCounters) reports the capture's counters."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "nvidia-resiliency-ext-x_amd"))
from nvidia_resiliency_ext.straggler import cupti, ops  # noqa: E402

import torch  # noqa: E402

bs = int(os.environ.get("DIAG_BUFSIZE", str(8 * 1024 * 1024)))
n = int(os.environ.get("DIAG_N", "5000"))
nsec = int(os.environ.get("DIAG_SECTIONS", "1"))
fl = int(os.environ.get("DIAG_FLUSH_EVERY", "0"))
sy = int(os.environ.get("DIAG_SYNC_EVERY", "0"))
p = cupti.KernelProfiler(bufferSize=bs, statsMaxLenPerKernel=8192, capture=True)
p.initialize()
score = torch.rand(1000, dtype=torch.float64, device="cuda")
m = torch.empty(1000, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
t = time.perf_counter()
for s in range(nsec):
    p.start()
    for _ in range(n // nsec):
        ops.stragglers(score, 0.5, out=m)
    p.stop()
    if sy and s % sy == sy - 1:
        torch.cuda.synchronize()
    if fl and s % fl == fl - 1:
        cupti.N.call("nvrx_capture_flush")
torch.cuda.synchronize()
st = p.get_stats()
env = {k: v for k, v in os.environ.items() if k.startswith(("DIAG", "NVRX"))}
print(env, "launched", n, "captured", sum(v.num_calls for v in st.values()),
      f"{time.perf_counter() - t:.3f}s", flush=True)
p.close()
