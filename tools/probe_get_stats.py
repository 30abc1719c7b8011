"""Probe (not part of the library): KernelProfiler.get_stats latency on a live-report-sized record
log (NK kernels x PER records pushed), wall time per call; run under rocprofv3 --kernel-trace to see
the device timeline of one report."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
import numpy as np  # noqa: E402

from nvidia_resiliency_ext.straggler import cupti  # noqa: E402

NK, PER = int(os.environ.get("NK", 86)), int(os.environ.get("PER", 335))
p = cupti.KernelProfiler(statsMaxLenPerKernel=4096, capture=False)
p.initialize()
p.start()
rng = np.random.default_rng(0)
names = [f"kernel_{i}_blk_256_1_1_grid_{i + 1}_1_1" for i in range(NK)]
ts = []
for it in range(30):
    for n in names:
        p.push(n, rng.integers(2000, 2_000_000, PER, dtype=np.uint64))
    t0 = time.perf_counter()
    cols = p.get_stats_columns()
    ts.append((time.perf_counter() - t0) * 1e3)
    p.reset()
p.stop()
ts.sort()
print(f"RESULT get_stats_ms median {ts[len(ts) // 2]:.3f} min {ts[0]:.3f} keys {len(cols.names)} records {NK * PER}")
