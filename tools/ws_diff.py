"""Debug: configs[3]-shaped record streams (AB_R ranks) bucketed + reduced with the shipped kernel
and with NVRX_RB_WS=<split>; prints which statistics differ and where (not part of the library)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import batch, synth  # noqa: E402

R, K, CAP = int(os.environ.get("AB_R", 512)), 2048, 8192
counts = synth.zipf_counts(K)
slot, occ = synth.zipf_order(counts)
N = slot.size
t = lambda a: torch.from_numpy(a.view(np.int32)).cuda()  # noqa: E731
recs = synth.synth_records(R, t(slot), t(occ), K, int(counts.max()))
rec_off = torch.arange(R + 1, dtype=torch.int64, device="cuda") * N
out = {}
for ws in ["0", sys.argv[1] if len(sys.argv) > 1 else "8x8"]:
    os.environ["NVRX_RB_WS"] = ws
    rep = batch.MatrixReporter(R, K, cap=CAP)
    rep.compute_stats_records(recs, rec_off)
    torch.cuda.synchronize()
    out[ws] = {f: getattr(rep.stats, f).cpu().numpy().copy() for f in ("num", "min", "max", "med", "avg", "std")}
    out[ws]["seg_len"] = rep._bucket[1].cpu().numpy().copy()
a, b = out["0"], out[list(out)[1]]
for f in a:
    x, y = a[f].view(np.int32), b[f].view(np.int32)
    bad = np.nonzero(x != y)[0]
    print(f, "differs at", bad.size, "of", x.size, "first", bad[:8].tolist(),
          "stream/slot", [(int(i) // K, int(i) % K) for i in bad[:8]],
          "vals", [(a[f][i], b[f][i]) for i in bad[:4]])
