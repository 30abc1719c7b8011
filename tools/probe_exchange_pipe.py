"""configs[1] reports through the N-GPU scoring branch (RCCL all_gather of the partials) in a world
of one: pipelined on two streams (the bench's N > 1 headline) against one report at a time (graph
phases: statistics | partials | eager all_gather | combine), interleaved blocks of N reports.
Usage: python tools/probe_exchange_pipe.py [N] [ROUNDS]."""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nvidia_resiliency_ext.straggler import batch, synth  # noqa: E402

with socket.socket() as so:
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
torch.cuda.set_device(0)
torch.distributed.init_process_group("nccl", device_id=torch.device("cuda:0"))
R, K, S, CAP = 64, 2048, 10000, 8192
N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ns = synth.synth_matrix(R, K, S, device="cuda")
rep = batch.MatrixReporter(R, K, cap=CAP, thr_rel=0.8, thr_ind=0.8, exchange=True)
pipe = rep.pipelined(ns, S)
g = rep.graph(ns, S)


def piped(n):
    pipe.submit()
    t0 = time.perf_counter()
    for i in range(n):
        if i + 1 < n:
            pipe.submit()
        pipe.collect()
    return (time.perf_counter() - t0) / n * 1e3


def phases(n):
    t0 = time.perf_counter()
    for _ in range(n):
        g.run_stats()
        g.run_rest()
    return (time.perf_counter() - t0) / n * 1e3


out = {"pipelined": [], "graph_phases": []}
piped(50)
phases(50)
for r in range(ROUNDS):
    for k, f in ((("pipelined", piped), ("graph_phases", phases)) if r % 2 == 0 else
                 (("graph_phases", phases), ("pipelined", piped))):
        out[k].append(f(N))
        print(k, round(out[k][-1], 4), flush=True)
torch.distributed.destroy_process_group()
print("RESULT " + json.dumps({k: dict(median_ms=float(np.median(v)), runs=v) for k, v in out.items()}))
