"""Pipelined reports by launch mode (batch.PipelinedReports: alt = each report on its own stream of
two, side = statistics on one stream and the rest on another, whole = one whole-report graph per
report on one stream), interleaved in one process so the box's clock drift cancels: ROUNDS x (N
reports of each mode), ms per report of each block, then the medians.
Usage: python tools/probe_pipe_streams.py [N] [ROUNDS] [config: c1 | c2 | c3]  (c1 = configs[1]
64 x 2048 x 10000 pushed, c2 = configs[2] 4096 x 2048 x 1024, c3 = configs[3] Zipf records)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# AB_PKG: package root to import (a saved copy with another libnvrx_hip.so, tools/build_variant.sh)
sys.path.insert(0, os.environ.get("AB_PKG", os.path.join(ROOT, "nvidia-resiliency-ext-x_amd")))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import batch, synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
CFG = sys.argv[3] if len(sys.argv) > 3 else "c1"
MODES = os.environ.get("MODES", "alt,side,whole").split(",")
mode_depth = lambda m: (m.rstrip("0123456789"), int(m[len(m.rstrip("0123456789")):] or 2))  # noqa: E731
if CFG == "c3":  # configs[3]: 16,384 Zipf record streams (bench.run_zipf's inputs)
    R, K, CAP = 16384, 2048, 8192
    counts = synth.zipf_counts(K)
    slot, occ = synth.zipf_order(counts)
    t = lambda a: torch.from_numpy(a.view(np.int32)).cuda()  # noqa: E731
    recs = synth.synth_records(R, t(slot), t(occ), K, int(counts.max()))
    rec_off = torch.arange(R + 1, dtype=torch.int64, device="cuda") * slot.size
    rep = batch.MatrixReporter(R, K, cap=CAP, thr_rel=0.8, thr_ind=0.8)
    pipes = {m: rep.pipelined_records(recs, rec_off, mode=mode_depth(m)[0]) for m in MODES}
else:
    R, K, S, CAP = (64, 2048, 10000, 8192) if CFG == "c1" else (4096, 2048, 1024, 8192)
    ns = synth.synth_matrix(R, K, S, device="cuda")
    rep = batch.MatrixReporter(R, K, cap=CAP, thr_rel=0.8, thr_ind=0.8)
    # a mode name may end in the pipeline depth (alt3: three reports in flight on three streams)
    pipes = {m: rep.pipelined(ns, S, mode=mode_depth(m)[0], depth=mode_depth(m)[1]) for m in MODES}


def block(p, n):
    d = p.depth
    for _ in range(d - 1):
        p.submit()
    t0 = time.perf_counter()
    for i in range(n):
        if i + d - 1 < n:
            p.submit()
        p.collect()
    return (time.perf_counter() - t0) / n * 1e3


out = {k: [] for k in pipes}
for k, p in pipes.items():
    block(p, max(4, N // 3))  # warm
for r in range(ROUNDS):
    items = list(pipes.items())
    for k, p in (items if r % 2 == 0 else items[::-1]):
        out[k].append(block(p, N))
        print(k, round(out[k][-1], 4), flush=True)
print("RESULT " + json.dumps({"config": CFG, **{k: dict(median_ms=float(np.median(v)), runs=v)
                                                for k, v in out.items()}}))
