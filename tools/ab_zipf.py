"""configs[3] pieces timed in one process: records_bucket, then length-classed stats.
AB_R ranks (default 16384) of Zipf record streams; prints ms per phase."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import batch, ops, synth  # noqa: E402

R, K, CAP = int(os.environ.get("AB_R", 16384)), 2048, 8192
counts = synth.zipf_counts(K)
slot, occ = synth.zipf_order(counts)
N = slot.size
t = lambda a: torch.from_numpy(a.view(np.int32)).cuda()  # noqa: E731
recs = synth.synth_records(R, t(slot), t(occ), K, int(counts.max()))
rec_off = torch.arange(R + 1, dtype=torch.int64, device="cuda") * N
rep = batch.MatrixReporter(R, K, cap=CAP)
rep.compute_stats_records(recs, rec_off)
torch.cuda.synchronize()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
b = rep._bucket
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
tb = ts = 0.0
for _ in range(n):
    e[0].record()
    ops.records_bucket(recs, rec_off, K, CAP, out=b)
    e[1].record()
    rep.compute_stats_records(recs, rec_off)  # fused path (bucket + in-block short runs + rest)
    e[2].record()
    torch.cuda.synchronize()
    tb += e[0].elapsed_time(e[1])
    ts += e[1].elapsed_time(e[2])
print(f"R={R} records={R*N} bucket_ms={tb/n:.3f} ({R*N*16/(tb/n)/1e6:.0f} GB/s at 16 B/rec) "
      f"fused_records_stats_ms={ts/n:.3f}")
