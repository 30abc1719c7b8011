"""A/B of the C3 (4096 x 2048 x 1024) stats kernels in one process: run with NVRX_ROWS_MAX
set per invocation is not possible in-process, so this times whatever kernel the env selects."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import ops, synth  # noqa: E402

R, K, S = int(os.environ.get("AB_R", 4096)), 2048, int(os.environ.get("AB_S", 1024))
CAP = 8192
ns = synth.synth_matrix(R, K, S, device="cuda")
out = ops.SegmentStats.empty(R * K, "cuda")
for _ in range(2):
    ops.segment_stats_strided(ns.view(-1), R * K, S, 0, S, cap=CAP, out=out)
torch.cuda.synchronize()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(n):
    ops.segment_stats_strided(ns.view(-1), R * K, S, 0, S, cap=CAP, out=out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / n
keep = min(S, CAP)
print(f"R={R} S={S} ROWS_MAX={os.environ.get('NVRX_ROWS_MAX', 'default')} ms={ms:.3f} TB/s={R*K*keep*4/ms/1e9:.2f}")
