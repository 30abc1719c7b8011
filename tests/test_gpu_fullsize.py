"""GPU: the bench's full-size configurations through size-independent properties:
configs[1] (64 ranks x 2048 kernels x 10,000 pushed, 8192 kept) and configs[2] (4096 x 2048 x
1024) at their real sizes --

  * a sample of whole rank rows bit for bit against the oracle's computeStats restatement;
  * permutation invariance: reversing every retained window leaves NUM/MIN/MAX/MED/AVG bit for
    bit unchanged and STD within the FAST bar (computeStats sorts; the order is free);
  * the straggler set equals the generator's injected set (1.3x ranks, threshold 0.8).
"""
import numpy as np
import pytest
import torch

import oracle as O
from nvidia_resiliency_ext.straggler import batch, synth

pytestmark = pytest.mark.gpu

EXACT_FIELDS = ("num", "min", "max", "med", "avg")


def _stats_host(rep):
    return {f: getattr(rep.stats, f).cpu().numpy() for f in EXACT_FIELDS + ("std",)}


def _check_mean_std(kept, g, idx):
    # FAST mode: AVG / STD are the exact mean / population std of the retained durations
    # rounded once to f32 -- the reference's sequential f32 sums drift ~1e-5
    # from them at n = 8192, so the bar is against the exact values, not the oracle's
    x = kept.astype(np.float64) / 1000.0
    mean = x.mean(axis=1)
    std = np.sqrt(((x - mean[:, None]) ** 2).mean(axis=1))
    np.testing.assert_allclose(g["avg"][idx], mean, rtol=2.5e-7, atol=0)
    np.testing.assert_allclose(g["std"][idx], std, rtol=1e-6, atol=0)


def _check_permutation(R, K, S, cap):
    ns = synth.synth_matrix(R, K, S)
    rep = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    res = rep.report(ns, S)
    a = _stats_host(rep)
    assert np.array_equal(res.stragglers_relative, synth.straggler_ranks(R).astype(bool))
    keep = min(S, cap)
    flat = ns.view(R * K, S)
    rev = torch.cat([flat[:, :S - keep], torch.flip(flat[:, S - keep:], dims=[1])], dim=1)
    del flat
    rep2 = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    res2 = rep2.report(rev.view(R, K, S), S)
    b = _stats_host(rep2)
    for f in EXACT_FIELDS:
        assert np.array_equal(a[f].view(np.uint32), b[f].view(np.uint32)), f
    np.testing.assert_allclose(b["std"], a["std"], rtol=2.5e-7, atol=0)
    np.testing.assert_allclose(res2.gpu_relative, res.gpu_relative, rtol=1e-12)
    return ns, rep


def test_config1_full_size():
    R, K, S, cap = 64, 2048, 10000, 8192
    ns, rep = _check_permutation(R, K, S, cap)
    # 4 whole rank rows (incl. the straggler rank) against the oracle, bit for bit
    rows = sorted({0, int(np.nonzero(synth.straggler_ranks(R))[0][0]), 31, 63})
    host = ns[rows].contiguous().cpu().numpy().view(np.uint32).reshape(-1)
    st = O.matrix_stats(host, len(rows) * K, S, 0, S, cap, nthreads=16)
    g = _stats_host(rep)
    idx = np.concatenate([np.arange(r * K, (r + 1) * K) for r in rows])
    for f in ("num", "min", "max", "med"):
        assert np.array_equal(g[f][idx].view(np.uint32), st[f].view(np.uint32)), f
    _check_mean_std(host.reshape(len(rows) * K, S)[:, S - min(S, cap):], g, idx)


def test_config2_full_size():
    R, K, S, cap = 4096, 2048, 1024, 8192
    ns, rep = _check_permutation(R, K, S, cap)
    rows = [0, 1234, 4095]
    host = ns[rows].contiguous().cpu().numpy().view(np.uint32).reshape(-1)
    st = O.matrix_stats(host, len(rows) * K, S, 0, S, cap, nthreads=16)
    g = _stats_host(rep)
    idx = np.concatenate([np.arange(r * K, (r + 1) * K) for r in rows])
    for f in ("num", "min", "max", "med"):
        assert np.array_equal(g[f][idx].view(np.uint32), st[f].view(np.uint32)), f
    _check_mean_std(host.reshape(len(rows) * K, S), g, idx)
    del ns, rep
    torch.cuda.empty_cache()


def test_config3_full_size():
    # configs[3]: 16,384 Zipf record streams.  A few whole streams against the oracle's
    # ring-push + computeStats restatement; every stream reversed (push order is free when no
    # ring overflows: kernel 1 is pushed exactly cap = 8192 times) gives the same statistics
    R, K, cap = 16384, 2048, 8192
    counts = synth.zipf_counts(K)
    slot, occ = synth.zipf_order(counts)
    N = slot.size
    t = lambda a: torch.from_numpy(a.view(np.int32)).cuda()  # noqa: E731
    recs = synth.synth_records(R, t(slot), t(occ), K, int(counts.max()))
    rec_off = torch.arange(R + 1, dtype=torch.int64, device="cuda") * N
    rep = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    res = rep.report_records(recs, rec_off)
    assert np.array_equal(res.stragglers_relative, synth.straggler_ranks(R).astype(bool))
    a = _stats_host(rep)
    rows = [0, int(np.nonzero(synth.straggler_ranks(R))[0][0]), R - 1]
    for r in rows:
        h = recs[r * N:(r + 1) * N].cpu().numpy().view(np.uint32)
        ref = O.records_stats(h, np.array([0, N], np.int64), K, cap=cap, nthreads=8)
        sl = slice(r * K, (r + 1) * K)
        for f in ("num", "min", "max", "med"):
            assert np.array_equal(a[f][sl].view(np.uint32), ref[f].view(np.uint32)), (r, f)
        short = ref["num"] <= 128  # lane classes: every field bit-exact
        for f in ("avg", "std"):
            assert np.array_equal(a[f][sl][short].view(np.uint32), ref[f][short].view(np.uint32)), (r, f)
    rev = torch.flip(recs.view(R, N, 2), dims=[1]).reshape(R * N, 2)
    del recs
    rep2 = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    res2 = rep2.report_records(rev, rec_off)
    b = _stats_host(rep2)
    for f in ("num", "min", "max", "med"):
        assert np.array_equal(a[f].view(np.uint32), b[f].view(np.uint32)), f
    short = a["num"] <= 128
    for f in ("avg", "std"):
        assert np.array_equal(a[f][short].view(np.uint32), b[f][short].view(np.uint32)), f
        np.testing.assert_allclose(b[f], a[f], rtol=2.5e-7, atol=0)
    np.testing.assert_allclose(res2.gpu_relative, res.gpu_relative, rtol=1e-12)
    del rev, rep, rep2
    torch.cuda.empty_cache()
