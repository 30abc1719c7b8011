"""Length-class kernels in isolation: NSEG ragged segments with lengths uniform in [LO, HI]
(16-B aligned runs), timed with and without the fused column reference."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import ops  # noqa: E402


def run(nseg, lo, hi, ncols, reps=5):
    rng = np.random.default_rng(0)
    lens = rng.integers(lo, hi + 1, nseg).astype(np.int64)
    gaps = (lens + 3) // 4 * 4
    off = np.zeros(nseg, np.int64)
    off[1:] = np.cumsum(gaps)[:-1]
    total = int(off[-1] + gaps[-1])
    ns = torch.randint(1000, 2_000_000, (total,), dtype=torch.int32, device="cuda")
    d_off = torch.from_numpy(off).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    out = ops.SegmentStats.empty(nseg, "cuda")
    col = torch.empty(2 * ncols, dtype=torch.int32, device="cuda")
    for cr in (False, True):
        kw = dict(col_ref=col, ncols=ncols) if cr else {}
        ops.segment_stats_ragged(ns, d_off, d_len, max_len=hi, aligned16=True, out=out, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ops.segment_stats_ragged(ns, d_off, d_len, max_len=hi, aligned16=True, out=out, **kw)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"nseg={nseg} len=[{lo},{hi}] colref={cr} ms={ms:.3f} "
              f"GB/s={lens.sum() * 4 / ms / 1e6:.0f} us/seg*waves={ms * 1e3 / nseg * 8192:.1f}")


for lo, hi in [(1, 8), (9, 32), (33, 64), (65, 256), (257, 512), (513, 1024)]:
    run(int(os.environ.get("AB_NSEG", 884736)), lo, hi, 54)
