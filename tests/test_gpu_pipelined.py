"""GPU: MatrixReporter.pipelined (two whole-report graphs in flight) gives, report for report,
the results of MatrixReporter.report -- including the individual history, which advances in
submission order -- and its timing events bracket the statistics phase."""
import numpy as np
import pytest
import torch

from nvidia_resiliency_ext.straggler import batch, synth

pytestmark = pytest.mark.gpu


def test_pipelined_matches_sequential_reports():
    R, K, S, cap = 16, 96, 1000, 512
    seqs = [synth.synth_matrix(R, K, S, seed=100 + i, device="cuda") for i in range(2)]
    a = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    b = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    ns = torch.empty_like(seqs[0])
    pipe = b.pipelined(ns, S, timing=True)
    b.reset_history()  # the capture's eager pass ran one report
    want, got = [], []
    ns.copy_(seqs[0])
    for i in range(5):
        want.append(a.report(seqs[i % 2], S))
    # b: the same five reports, two in flight; the input changes only between collections
    for i in range(5):
        ns.copy_(seqs[i % 2])
        pipe.submit(timed=i % 2 == 0)
        res, ms = pipe.collect()
        assert (ms is not None and ms > 0.0) if i % 2 == 0 else ms is None
        got.append(res)
    for w, g in zip(want, got):
        np.testing.assert_array_equal(w.gpu_relative, g.gpu_relative)
        np.testing.assert_array_equal(w.gpu_individual, g.gpu_individual)
        np.testing.assert_array_equal(w.stragglers_relative, g.stragglers_relative)
        np.testing.assert_array_equal(w.stragglers_individual, g.stragglers_individual)


def test_pipelined_two_in_flight():
    R, K, S = 8, 64, 1000
    ns = synth.synth_matrix(R, K, S, device="cuda")
    rep = batch.MatrixReporter(R, K, cap=512, thr_rel=0.8, thr_ind=0.8)
    want = rep.report(ns, S)
    pipe = rep.pipelined(ns, S)
    pipe.submit()
    pipe.submit()
    with pytest.raises(RuntimeError):
        pipe.submit()
    with pytest.raises(RuntimeError):  # timed reports need timing=True
        pipe.collect(), pipe.submit(timed=True)
    pipe2 = rep.pipelined(ns, S, timing=True)
    pipe2.submit()
    pipe2.submit()
    pipe2.collect()
    pipe2.submit(timed=True)  # drains the one in flight first
    outs = [pipe2.collect(), pipe2.collect()]
    assert outs[0][1] is None and outs[1][1] is not None
    for res, _ in outs + [pipe.collect()]:
        np.testing.assert_array_equal(res.stragglers_relative, want.stragglers_relative)
