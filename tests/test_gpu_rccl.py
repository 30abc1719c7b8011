"""GPU: the multi-GPU scoring branch of MatrixReporter over RCCL ("nccl" backend) -- score
partials -> device-to-device all_gather_into_tensor -> finalize_kernel -- in a world of one
(a one-GPU box cannot hold two RCCL ranks: RCCL refuses two ranks on one device), against the
fused single-GPU scoring of the same statistics.  The N-rank shard layout itself is covered by
the gloo worlds of test_gpu_batch.py / test_sharding_cpu.py; this runs the RCCL calls."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nvidia-resiliency-ext-x_amd")

CHILD = r"""
import json, os, socket
import numpy as np
import torch
from nvidia_resiliency_ext.straggler import batch, synth
with socket.socket() as so:
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
torch.cuda.set_device(0)
torch.distributed.init_process_group("nccl", device_id=torch.device("cuda:0"))
out = {"backend": str(torch.distributed.get_backend())}

def same(a, b):
    return a.stragglers_relative.tolist() == b.stragglers_relative.tolist() and \
        a.stragglers_individual.tolist() == b.stragglers_individual.tolist() and a.err == b.err == 0

def maxrel(x, y):
    return float(np.max(np.abs(x - y) / np.abs(y)))

# matrix path: two reports (the second exercises the history), eager and graph-replayed
R, K, S, cap = 64, 256, 1000, 512
ns = synth.synth_matrix(R, K, S, device="cuda")
fused = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8, exchange=False)
xchg = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8, exchange=True)
errs, sets = [], []
for t in range(2):
    a, b = fused.report(ns, S), xchg.report(ns, S)
    errs += [maxrel(b.gpu_relative, a.gpu_relative), maxrel(b.gpu_individual, a.gpu_individual)]
    sets.append(same(a, b))
g = xchg.graph(ns, S)  # stats as a graph, the exchange eager
g.run_stats()
b = g.run_rest()
errs.append(maxrel(b.gpu_relative, a.gpu_relative))
sets.append(same(a, b))
# record-stream path (configs[3] shape, 12 ranks)
Kz = 2048
counts = synth.zipf_counts(Kz)
slot, occ = synth.zipf_order(counts)
t32 = lambda x: torch.from_numpy(x.view(np.int32)).cuda()
Rz = 12
recs = synth.synth_records(Rz, t32(slot), t32(occ), Kz, int(counts.max()))
off = torch.arange(Rz + 1, dtype=torch.int64, device="cuda") * slot.size
fz = batch.MatrixReporter(Rz, Kz, cap=8192, thr_rel=0.8, exchange=False).report_records(recs, off)
xz = batch.MatrixReporter(Rz, Kz, cap=8192, thr_rel=0.8, exchange=True).report_records(recs, off)
errs.append(maxrel(xz.gpu_relative, fz.gpu_relative))
sets.append(same(fz, xz))
# ... and as the N-GPU bench leg runs it: statistics, partials and combine as graphs, the
# all_gather eager (MatrixReporter.graph_records)
gz = batch.MatrixReporter(Rz, Kz, cap=8192, thr_rel=0.8, exchange=True).graph_records(recs, off)
for _ in range(2):
    gz.run_stats()
    yz = gz.run_rest()
    errs.append(maxrel(yz.gpu_relative, fz.gpu_relative))
    sets.append(same(fz, yz))
# ... and as the bench runs it: reports two in flight on two streams (PipelinedReports with the
# exchange), the history advancing report by report -- against eager single-GPU reports
ns2 = synth.synth_matrix(R, K, S, seed=77, device="cuda")
ref = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8, exchange=False)
src = [ns, ns, ns2, ns2, ns, ns]  # two reports in flight per input
want = [ref.report(x, S) for x in src]
piped = []
for mode in ("alt", "side"):  # each report on its own stream / statistics | rest on two streams
    xp = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8, exchange=True)
    buf = torch.empty_like(ns)
    pipe = xp.pipelined(buf, S, timing=True, mode=mode, timing_reps=2)  # (the bench's timing graph)
    got = []
    for i in range(0, 6, 2):
        # the input changes only once the reports reading it have been collected
        buf.copy_(src[i])
        pipe.submit()
        pipe.submit(timed=i == 2)  # a timed submit drains the report in flight first
        got += [pipe.collect()[0], pipe.collect()[0]]
    for a, b in zip(want, got):
        errs += [maxrel(b.gpu_relative, a.gpu_relative), maxrel(b.gpu_individual, a.gpu_individual)]
        piped.append(same(a, b))
out.update(errs=errs, sets=sets, piped=piped, nrel=int(xz.stragglers_relative.sum()))
torch.distributed.destroy_process_group()
print("RESULT " + json.dumps(out))
"""


def test_rccl_exchange_matches_fused_scoring():
    e = dict(os.environ)
    r = subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {PKG!r})\n" + CHILD],
                       capture_output=True, text=True, timeout=300, env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1][7:])
    assert out["backend"] == "nccl"
    assert all(out["sets"]), out
    assert len(out["piped"]) == 12 and all(out["piped"]), out
    # one shard: the finalize kernel divides the same two sums the fused kernel does
    assert max(out["errs"]) <= 1e-13, out["errs"]
    assert out["nrel"] > 0  # the injected straggler ranks are flagged through the exchange
