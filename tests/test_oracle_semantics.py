"""CPU: the oracle's scoring and retention semantics, restated from the reference's own
known-answer tests and its source, so that the checker the GPU parity tests
lean on is pinned case by case, not only through the golden report fixtures.

Reference anchors:
  relative scores 1/(rank+1)          test_relative_gpu_scores.py:97-139, reporting.py:219-253
  partially / not common kernels      test_relative_gpu_scores.py:210-242, :281-356;
                                      reporting.py:255-296 (any rank missing -> NaN reference)
  individual history 1 -> 0.8 -> ...  test_individual_gpu_scores.py:46-121; reporting.py:298-314,470
  ncclDev filter                      reporting.py:330-336
  stragglers: score < thr (strict)    reporting.py:84-151
  ring keeps the last cap pushes      CircularBuffer.h:53-69
  section stats: lower median,        straggler.py:171-197
  unbiased std, NaN for n == 1
"""
import math

import numpy as np
import pytest
import torch

import oracle as O
import oracle_report as OR


def _uniform(R, K, med):
    num = np.full((R, K), 10, np.int32)
    avg = np.asarray(med, np.float32)
    return num, np.asarray(med, np.float32), avg


@pytest.mark.parametrize("R,K", [(1, 1), (4, 3), (8, 200)])
def test_relative_scores_are_one_over_rank_plus_one(R, K):
    base = np.arange(1, K + 1, dtype=np.float32) * 3.0
    med = np.stack([base * (r + 1) for r in range(R)])
    num, med, avg = _uniform(R, K, med)
    gr, gi = O.scores(num, med, avg)
    np.testing.assert_allclose(gr, [1.0 / (r + 1) for r in range(R)], rtol=1e-15)
    assert np.all(gi == 1.0)  # first report: the history is the median itself


def test_relative_partially_common_kernels_use_only_the_common_ones():
    # kernel 0 missing on rank 1: its reference is NaN for every rank (MIN all-reduce of -1)
    R, K = 3, 3
    med = np.array([[1.0, 2.0, 4.0], [9.0, 4.0, 8.0], [1.0, 8.0, 16.0]], np.float32)
    num = np.full((R, K), 5, np.int32)
    num[1, 0] = 0
    avg = med.copy()
    ref = O.kernel_ref(num, med)
    assert math.isnan(ref[0]) and ref[1] == 2.0 and ref[2] == 4.0
    gr, _ = O.scores(num, med, avg)
    # only kernels 1 and 2; weights num * avg
    for r in range(R):
        w = num[r, 1:] * avg[r, 1:].astype(np.float64)
        s = np.array([2.0, 4.0]) / med[r, 1:].astype(np.float64)
        assert gr[r] == pytest.approx(float((s * w).sum() / w.sum()), rel=1e-15)


def test_relative_no_common_kernel_is_nan_for_every_rank():
    R, K = 2, 2
    med = np.ones((R, K), np.float32)
    num = np.array([[1, 0], [0, 1]], np.int32)
    gr, gi = O.scores(num, med, med.copy())
    assert np.all(np.isnan(gr))
    assert np.all(gi == 1.0)  # the individual score does not need other ranks


def test_individual_history_sequence():
    # one rank, medians over successive reports; the history is the running minimum,
    # updated before scoring, so the score is <= 1 and 1 on first sight
    hist = np.full((1, 2), np.inf)
    seq = []

    def report(meds, present):
        med = np.array([meds], np.float32)
        num = np.array([present], np.int32)
        _, gi = O.scores(num, med, med.copy(), hist=hist, rel=False)
        seq.append(gi[0])

    for m in (1.0, 1.25, 2.0, 3.0, 4.0, 5.0):
        report([m, 1.0], [1, 0])
    report([1.0, 1.0], [0, 0])      # no kernels at all -> NaN
    report([9.0, 2.0], [0, 1])      # a new kernel -> 1.0
    report([9.0, 1.0], [0, 1])      # a new minimum -> 1.0
    report([9.0, 2.0], [0, 1])      # twice the minimum -> 0.5
    want = [1.0, 0.8, 0.5, 1 / 3, 0.25, 0.2, float("nan"), 1.0, 1.0, 0.5]
    for got, exp in zip(seq, want):
        if math.isnan(exp):
            assert math.isnan(got)
        else:
            assert got == pytest.approx(exp, rel=1e-15)


def test_filtered_columns_are_ignored_like_nccl_kernels():
    # col_valid = 0 drops a column for both scores (the "ncclDev" name filter)
    R, K = 2, 2
    med = np.array([[1.0, 1.0], [2.0, 100.0]], np.float32)
    num = np.ones((R, K), np.int32)
    gr, _ = O.scores(num, med, med.copy(), col_valid=np.array([1, 0], np.uint8))
    np.testing.assert_allclose(gr, [1.0, 0.5], rtol=1e-15)


def test_stragglers_strict_threshold_and_nan():
    score = np.array([0.5, 0.8, 0.8000000001, float("nan"), 0.79999999])
    assert O.stragglers(score, 0.8).tolist() == [1, 0, 0, 0, 1]


def test_ring_keeps_the_last_cap_pushes_in_order():
    pushed = np.arange(1, 22, dtype=np.float32)  # 21 pushes into a cap-7 ring
    assert O.ring_linearize(pushed, 7).tolist() == list(range(15, 22))
    assert O.ring_linearize(pushed[:5], 7).tolist() == [1, 2, 3, 4, 5]


def test_matrix_stats_equals_per_segment_restatement():
    rng = np.random.default_rng(7)
    nseg, stride, begin, length, cap = 23, 50, 3, 40, 16
    ns = rng.integers(1, 3_000_000, size=nseg * stride, dtype=np.uint32)
    st = O.matrix_stats(ns, nseg, stride, begin, length, cap, nthreads=3)
    for s in range(nseg):
        seg = ns[s * stride + begin: s * stride + begin + length]
        k = O.compute_stats(O.ring_linearize(O.ns_to_us(seg), cap))
        assert st["num"][s] == k.num_calls == cap
        for f, v in (("min", k.min), ("max", k.max), ("med", k.median), ("avg", k.avg), ("std", k.stddev)):
            assert np.float32(st[f][s]).view(np.uint32) == np.float32(v).view(np.uint32), (s, f)


def test_records_stats_equals_ring_pushes_per_slot():
    rng = np.random.default_rng(11)
    nslots, cap = 9, 5
    streams, off = [], [0]
    for n in (0, 17, 60, 3):
        slot = rng.integers(0, nslots + 1, size=n, dtype=np.uint32)  # nslots: out of range, dropped
        ns = rng.integers(1000, 4_000_000, size=n, dtype=np.uint32)
        streams.append(np.stack([slot, ns], axis=1).reshape(-1, 2))
        off.append(off[-1] + n)
    recs = np.concatenate(streams)
    off = np.array(off, np.int64)
    st = O.records_stats(recs, off, nslots, cap=cap)
    for t in range(len(off) - 1):
        stream = recs[off[t]:off[t + 1]]
        for s in range(nslots):
            pushed = stream[stream[:, 0] == s, 1]
            g = t * nslots + s
            if pushed.size == 0:
                assert st["num"][g] == 0 and math.isnan(st["med"][g])
                continue
            k = O.compute_stats(O.ring_linearize(O.ns_to_us(pushed), cap))
            assert st["num"][g] == k.num_calls == min(cap, pushed.size)
            assert np.float32(st["med"][g]) == np.float32(k.median)
            assert np.float32(st["avg"][g]).view(np.uint32) == np.float32(k.avg).view(np.uint32)


@pytest.mark.parametrize("vals", [[3.5], [2.0, 1.0], [5.0, 1.0, 3.0, 2.0], list(np.linspace(0.1, 9.0, 17))])
def test_section_summary_matches_torch_semantics(vals):
    got = OR.section_summary_torch_semantics(vals)
    t = torch.tensor(vals, dtype=torch.float64)
    assert got[OR.MED] == float(torch.median(t))          # the lower median
    assert got[OR.MIN] == float(t.min()) and got[OR.MAX] == float(t.max())
    assert got[OR.NUM] == len(vals)
    if len(vals) == 1:
        assert math.isnan(got[OR.STD])                    # unbiased std of one sample
    else:
        assert got[OR.STD] == pytest.approx(float(torch.std(t)), rel=1e-15)


# ---- the oracle's three routes to computeStats give identical statistics: the radix-sorted
# integer keys (checker), a comparison sort of the converted floats (computeStats' own route),
# and the std::sort ring-push port that bench.py times as the host-CPU Reporter
@pytest.mark.parametrize("cap", [8192, 100, 7, 1])
def test_matrix_stats_routes_agree(cap):
    rng = np.random.default_rng(cap)
    parts = [O.gen_matrix(4, 40, 900).reshape(160, 900),
             rng.integers(0, 2**32, size=(64, 900), dtype=np.uint64).astype(np.uint32),
             rng.integers(2**24 - 8, 2**24 + 8, size=(32, 900)).astype(np.uint32),  # f32 ties
             np.full((8, 900), 12345, np.uint32)]
    ns = np.ascontiguousarray(np.concatenate(parts))
    r = [O.matrix_stats(ns.reshape(-1), ns.shape[0], 900, 0, 900, cap, nthreads=3, route=x)
         for x in ("radix", "qsort", "baseline")]
    for f in r[0]:
        for other in r[1:]:
            assert np.array_equal(r[0][f].view(np.uint32), other[f].view(np.uint32)), f


@pytest.mark.parametrize("cap", [8192, 5, 1])
def test_records_stats_routes_agree(cap):
    rng = np.random.default_rng(11 + cap)
    R, K, N = 5, 40, 2500
    slot = rng.integers(0, K + 2, size=R * N).astype(np.uint32)  # a few out-of-range slots
    ns = rng.integers(1, 2**32, size=R * N, dtype=np.uint64).astype(np.uint32)
    recs = np.ascontiguousarray(np.stack([slot, ns], 1))
    off = np.arange(R + 1, dtype=np.int64) * N
    a = O.records_stats(recs, off, K, cap=cap, nthreads=2)
    b = O.records_stats(recs, off, K, cap=cap, nthreads=2, route="baseline")
    for f in a:
        assert np.array_equal(a[f].view(np.uint32), b[f].view(np.uint32)), f
