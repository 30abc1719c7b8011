"""A/B of the FAST stats kernel variants on the C2 workload (run under rocprofv3 --kernel-trace).
Interleaves: plain stats; stats + fused column reference."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import ops, synth  # noqa: E402

R, K, S, CAP = 64, 2048, 10000, 8192
ns = synth.synth_matrix(R, K, S, device="cuda")
out = ops.SegmentStats.empty(R * K, "cuda")
col = torch.empty(2 * K, dtype=torch.int32, device="cuda")
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    ops.segment_stats_strided(ns.view(-1), R * K, S, 0, S, cap=CAP, out=out)
    ops.segment_stats_strided(ns.view(-1), R * K, S, 0, S, cap=CAP, out=out, col_ref=col, ncols=K)
torch.cuda.synchronize()
print("done")
