"""Interleaved A/B of the configs[2] (4096 x 2048 x 1024; AB_R / AB_S: another shape, e.g.
configs[1] = 64 / 10000) statistics kernel: argv[1] = package
root to import (the current tree or a saved copy with another libnvrx_hip.so), argv[2] = reps.
Prints ms per launch."""
import os
import sys

sys.path.insert(0, sys.argv[1])
import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import ops, synth  # noqa: E402

R, K, S, CAP = int(os.environ.get("AB_R", 4096)), 2048, int(os.environ.get("AB_S", 1024)), 8192
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ns = synth.synth_matrix(R, K, S, device="cuda")
out = ops.SegmentStats.empty(R * K, "cuda")
for _ in range(3):
    ops.segment_stats_strided(ns.view(-1), R * K, S, 0, S, cap=CAP, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(n):
    ops.segment_stats_strided(ns.view(-1), R * K, S, 0, S, cap=CAP, out=out)
e1.record()
torch.cuda.synchronize()
st = out.cpu()
print(f"{os.path.basename(os.path.dirname(sys.argv[1].rstrip('/')))}/{os.path.basename(sys.argv[1].rstrip('/'))} "
      f"ms={e0.elapsed_time(e1) / n:.3f} med0={st.med[0].item():.4f} avg_sum={st.avg.double().sum().item():.6f}",
      flush=True)
