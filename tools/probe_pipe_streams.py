"""configs[1] pipelined reports, two streams (batch.PipelinedReports default) against whole-report
graphs on one stream (NVRX_PIPE_MODE=whole), interleaved in one
process (the box's clock drift cancels): ROUNDS x (N reports of each mode), ms per report of
each block, then the medians.  Usage: python tools/probe_pipe_streams.py [N] [ROUNDS]."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import batch, synth  # noqa: E402

R, K, S, CAP = 64, 2048, 10000, 8192
N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ns = synth.synth_matrix(R, K, S, device="cuda")
rep = batch.MatrixReporter(R, K, cap=CAP, thr_rel=0.8, thr_ind=0.8)
pipes = {}
for name, alt in (("two_streams", True), ("whole", False)):
    batch._PIPE_ALT = alt
    pipes[name] = rep.pipelined(ns, S)


def block(p, n):
    p.submit()
    t0 = time.perf_counter()
    for i in range(n):
        if i + 1 < n:
            p.submit()
        p.collect()
    return (time.perf_counter() - t0) / n * 1e3


out = {k: [] for k in pipes}
for k, p in pipes.items():
    block(p, 100)  # warm
for r in range(ROUNDS):
    for k, p in (list(pipes.items()) if r % 2 == 0 else list(reversed(list(pipes.items())))):
        out[k].append(block(p, N))
        print(k, round(out[k][-1], 4), flush=True)
print("RESULT " + json.dumps({k: dict(median_ms=float(np.median(v)), runs=v) for k, v in out.items()}))
