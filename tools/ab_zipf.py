"""configs[3] record-stream statistics timed alone: MatrixReporter.compute_stats_records
(bucketing + length-classed statistics) on AB_R ranks (default 16384) of Zipf record
streams; prints ms per call and the NVRX_* environment it ran under (A/B knobs)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AB_PKG: package root to import (a saved copy with another libnvrx_hip.so, e.g. tools/ab_pkg)
sys.path.insert(0, os.environ.get("AB_PKG", os.path.join(ROOT, "nvidia-resiliency-ext-x_amd")))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import batch, synth  # noqa: E402

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
ref = rep.stats.cpu()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ts = 0.0
for _ in range(n):
    e[0].record()
    rep.compute_stats_records(recs, rec_off)
    e[1].record()
    torch.cuda.synchronize()
    ts += e[0].elapsed_time(e[1])
if os.environ.get("AB_DUMP"):  # the statistics of the first call (parity of A/B variants)
    torch.save({f: getattr(ref, f) for f in ("num", "min", "max", "med", "avg", "std")}, os.environ["AB_DUMP"])
env = {k: v for k, v in os.environ.items() if k.startswith("NVRX_")}
print(f"pkg={os.environ.get('AB_PKG', 'tree')} R={R} records={R*N} records_stats_ms={ts/n:.3f} "
      f"({R*N*8/(ts/n)/1e6:.0f} GB/s at 8 B/rec) env={env}")
