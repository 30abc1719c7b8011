"""GPU: the batched report (MatrixReporter) vs the oracle, and the kernel-hash sharded
multi-GPU path (gloo world size 2/3 sharing one device) vs the single-GPU report."""
import numpy as np
import pytest
import torch

import oracle as O
from _fastbars import check_avg_std
from _mp import run_world
from nvidia_resiliency_ext.straggler import batch, ops, synth

pytestmark = pytest.mark.gpu


def _oracle_report(R, K, S, cap, thr, hist=None):
    ns = O.gen_matrix(R, K, S)
    st = O.matrix_stats(ns.reshape(-1), R * K, S, 0, S, cap, nthreads=8)
    num, med, avg = (st[f].reshape(R, K) for f in ("num", "med", "avg"))
    gr, gi = O.scores(num, med, avg, hist=hist)
    return gr, gi, O.stragglers(gr, thr).astype(bool), O.stragglers(gi, thr).astype(bool)


@pytest.mark.parametrize("R,K,S,cap", [(8, 64, 1000, 512), (64, 33, 2500, 2048), (3, 5, 10000, 8192),
                                       (130, 7, 1024, 8192)])
def test_matrix_report_matches_oracle(R, K, S, cap):
    ns = synth.synth_matrix(R, K, S, device="cuda")
    rep = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    res = rep.report(ns, S)
    hist = np.full((R, K), np.inf)
    gr, gi, sr, si = _oracle_report(R, K, S, cap, 0.8, hist)
    np.testing.assert_allclose(res.gpu_relative, gr, rtol=1e-6)
    np.testing.assert_allclose(res.gpu_individual, gi, rtol=1e-6)
    assert np.array_equal(res.stragglers_relative, sr) and np.array_equal(res.stragglers_individual, si)
    assert res.err == 0
    # the designated straggler ranks are exactly the ones flagged
    assert np.array_equal(res.stragglers_relative, synth.straggler_ranks(R).astype(bool))
    # second report on the same samples: history == MED -> individual score 1.0
    res2 = rep.report(ns, S)
    np.testing.assert_allclose(res2.gpu_individual, 1.0, rtol=1e-15)
    np.testing.assert_allclose(res2.gpu_relative, res.gpu_relative, rtol=0)


def test_matrix_report_exact_mode_and_f32_gather_rounding():
    R, K, S = 16, 40, 700
    ns = synth.synth_matrix(R, K, S, device="cuda")
    rep = batch.MatrixReporter(R, K, cap=8192, mode=ops.STATS_EXACT, round_f32=True)
    res = rep.report(ns, S)
    gr, gi, _, _ = _oracle_report(R, K, S, 8192, 0.75)
    # EXACT stats are the reference's own; only the score sums' order differs
    np.testing.assert_allclose(res.gpu_relative, gr.astype(np.float32).astype(np.float64), rtol=1.2e-7)
    assert np.all(res.gpu_relative == res.gpu_relative.astype(np.float32).astype(np.float64))


@pytest.mark.parametrize("ws", [2, 3])
def test_sharded_report_matches_single_gpu(ws):
    R, K, S, cap, thr = 12, 96, 800, 512, 0.8
    res = run_world(ws, "_shard_workers", "gpu_sharded_report", R=R, K=K, S=S, cap=cap, thr=thr)
    ns = synth.synth_matrix(R, K, S, device="cuda")
    rep = batch.MatrixReporter(R, K, cap=cap, thr_rel=thr, thr_ind=thr)
    single = [rep.report(ns, S) for _ in range(2)]
    for r in range(ws):
        for t in range(2):
            got = res[r][t]
            np.testing.assert_allclose(got["rel"], single[t].gpu_relative, rtol=1e-13)
            np.testing.assert_allclose(got["ind"], single[t].gpu_individual, rtol=1e-13)
            assert np.array_equal(got["srel"], single[t].stragglers_relative)
            assert np.array_equal(got["sind"], single[t].stragglers_individual)
            assert got["err"] == 0


# ---- configs[3] shape: Zipf record streams (bucket by slot -> length-classed stats)
@pytest.mark.parametrize("R,cap", [(24, 8192), (12, 100), (5, 1)])
def test_zipf_record_streams_match_oracle(R, cap):
    K = 2048
    counts = synth.zipf_counts(K)
    slot, occ = synth.zipf_order(counts)
    N = slot.size
    d_slot = torch.from_numpy(slot.view(np.int32)).cuda()
    d_occ = torch.from_numpy(occ.view(np.int32)).cuda()
    recs = synth.synth_records(R, d_slot, d_occ, K, int(counts.max()))
    rec_off = torch.arange(R + 1, dtype=torch.int64, device="cuda") * N
    rep = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    res = rep.report_records(recs, rec_off)
    # oracle: the same streams, ring retention + computeStats per (rank, slot)
    h = recs.cpu().numpy().view(np.uint32)
    ref = O.records_stats(h, rec_off.cpu().numpy(), K, cap=cap, nthreads=8)
    g = rep.stats.cpu()
    for f in ("num", "min", "max", "med"):
        a, b = getattr(g, f).numpy(), ref[f]
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), f
    xm, xs = O.records_moments(h, rec_off.cpu().numpy(), K, cap=cap, nthreads=8)
    check_avg_std(g.avg.numpy(), g.std.numpy(), ref, xm, xs, f"zipf R={R} cap={cap}")
    num, med, avg = (ref[f].reshape(R, K) for f in ("num", "med", "avg"))
    gr, gi = O.scores(num, med, avg)
    np.testing.assert_allclose(res.gpu_relative, gr, rtol=1e-6)
    np.testing.assert_allclose(res.gpu_individual, gi, rtol=1e-6)
    assert np.array_equal(res.stragglers_relative, O.stragglers(gr, 0.8).astype(bool))
    assert np.array_equal(res.stragglers_relative, synth.straggler_ranks(R).astype(bool))
    assert res.err == 0


def test_zipf_order_is_a_valid_interleaving():
    counts = synth.zipf_counts(2048)
    assert counts.sum() == 47_482 and counts[0] == 8192 and counts[-1] == 1
    slot, occ = synth.zipf_order(counts)
    for k in (0, 1, 7, 100, 2047):
        assert np.array_equal(occ[slot == k], np.arange(counts[k]))  # push order per kernel


def test_graph_replay_matches_eager():
    # MatrixReporter.graph: the same kernels captured once and replayed; four successive
    # reports (history carried) equal the eager reporter's bit for bit, whether replayed as one
    # graph or as the stats / rest halves
    R, K, S, cap = 48, 300, 700, 512
    ns = synth.synth_matrix(R, K, S)
    eager = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    graphed = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    g = graphed.graph(ns, S)
    graphed.reset_history()  # the capture's eager warm pass updated the history once
    for i in range(4):  # the one-graph report and the two-graph (timed) halves alternate
        a = eager.report(ns, S)
        if i % 2 == 0:
            b = g.run()
        else:
            g.run_stats()
            b = g.run_rest()
        assert np.array_equal(a.gpu_relative, b.gpu_relative)
        assert np.array_equal(a.gpu_individual, b.gpu_individual)
        assert np.array_equal(a.stragglers_relative, b.stragglers_relative)
        assert np.array_equal(a.stragglers_individual, b.stragglers_individual)
        assert a.err == b.err == 0
    for f in ("num", "min", "max", "med", "avg", "std"):
        assert torch.equal(getattr(eager.stats, f), getattr(graphed.stats, f)), f
    assert torch.equal(eager.hist, graphed.hist)
