"""GPU parity: per-kernel statistics (HIP segment_stats) vs the oracle computeStats.

Bar (north_star): NUM / MIN / MAX / MED bit-exact on integer-ns inputs, in both modes;
EXACT mode also AVG / STD bit-exact; FAST mode AVG / STD are the exact f64 mean /
population std of the retained samples rounded once to f32, checked (a) against an f64
numpy reference within 2 f32 ulps and (b) against the oracle's sequential-f32 values
within rtol 1e-4 (the reference's own accumulation error at n <= 8192).
"""
import numpy as np
import pytest
import torch

import oracle as O
from _fastbars import key_values
from nvidia_resiliency_ext.straggler import ops, synth

pytestmark = pytest.mark.gpu
DEV = "cuda"
FIELDS = ("num", "min", "max", "med")


def _oracle_segments(host_ns, nseg, stride, begin, length, cap):
    return O.matrix_stats(host_ns, nseg, stride, begin, length, cap, nthreads=8)


def _exact_avg_std(host_ns, nseg, stride, begin, length, cap):
    keep = min(length, cap) if cap > 0 else length
    avg = np.empty(nseg)
    std = np.empty(nseg)
    for s in range(nseg):
        seg = key_values(host_ns[s * stride + begin + length - keep: s * stride + begin + length])
        avg[s] = seg.mean() / 1000.0
        std[s] = seg.std() / 1000.0
    return avg, std


def _check(gpu, ref, exact_fields=FIELDS, avg_std=None):
    g = gpu.cpu()
    for f in exact_fields:
        a = getattr(g, f).numpy()
        b = ref[f]
        if a.dtype.kind == "f":
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (f, a[:8], b[:8])
        else:
            assert np.array_equal(a, b), (f, a[:8], b[:8])
    if avg_std is not None:
        # FAST: exact mean/std rounded once to f32.  A segment that does not fit a fast
        # wave (>8192 slots incl. 16-B misalignment) runs the EXACT kernel instead, whose
        # AVG/STD are the reference's own (bit-exact with the oracle): accept either.
        avg, std = avg_std
        ga, gs = g.avg.numpy(), g.std.numpy()
        exact_ref = (ga.view(np.uint32) == ref["avg"].view(np.uint32)) & \
                    (gs.view(np.uint32) == ref["std"].view(np.uint32))
        fast_ok = (np.abs(ga - avg) <= 2.5e-7 * np.abs(avg)) & \
                  (np.abs(gs - std) <= 1e-6 * np.abs(std) + 1e-6)
        assert np.all(exact_ref | fast_ok), (ga, avg, ref["avg"])
        np.testing.assert_allclose(ga, ref["avg"], rtol=1e-4)


def test_synth_matrix_matches_oracle_generator():
    R, K, S = 3, 7, 37
    strag = synth.straggler_ranks(R)
    g = synth.synth_matrix(R, K, S, device=DEV).cpu().numpy().view(np.uint32)
    h = O.gen_matrix(R, K, S, straggler=strag)
    assert np.array_equal(g, h)
    # sharded columns: local column kk holds global kernel kmap[kk]
    kmap = np.array([5, 1, 6], dtype=np.int64)
    g2 = synth.synth_matrix(R, 3, S, K_global=K, kmap=torch.from_numpy(kmap).to(DEV),
                            device=DEV).cpu().numpy().view(np.uint32)
    assert np.array_equal(g2, h[:, kmap, :])


@pytest.mark.parametrize("mode", [ops.STATS_FAST, ops.STATS_EXACT])
def test_matrix_config_small(mode):
    # config-2 shape scaled down: S_push 10000 pushed, last 8192 retained
    R, K, S = 2, 12, 10000
    ns = synth.synth_matrix(R, K, S, device=DEV)
    st = ops.segment_stats_strided(ns.view(-1), R * K, S, 0, S, cap=8192, mode=mode)
    host = ns.cpu().numpy().view(np.uint32).reshape(-1)
    ref = _oracle_segments(host, R * K, S, 0, S, 8192)
    if mode == ops.STATS_EXACT:
        _check(st, ref, exact_fields=FIELDS + ("avg", "std"))
    else:
        _check(st, ref, avg_std=_exact_avg_std(host, R * K, S, 0, S, 8192))


LENGTHS = [1, 2, 3, 4, 5, 7, 8, 63, 64, 65, 255, 256, 257, 511, 512, 1000, 1023, 1024, 1025,
           2047, 2048, 2049, 4095, 4096, 4097, 8191, 8192]


@pytest.mark.parametrize("mode", [ops.STATS_FAST, ops.STATS_EXACT])
@pytest.mark.parametrize("length", LENGTHS)
def test_lengths_and_alignment(mode, length):
    rng = np.random.default_rng(length)
    nseg = 6
    for begin in (0, 1, 2, 3):
        stride = length + begin + (rng.integers(0, 5) if begin else 0)
        host = rng.integers(1000, 3_000_000, size=nseg * stride, dtype=np.uint32)
        ns = torch.from_numpy(host.view(np.int32)).to(DEV)
        st = ops.segment_stats_strided(ns, nseg, stride, begin, length, cap=0, mode=mode)
        ref = _oracle_segments(host, nseg, stride, begin, length, 0)
        if mode == ops.STATS_EXACT:
            _check(st, ref, exact_fields=FIELDS + ("avg", "std"))
        else:
            _check(st, ref, avg_std=_exact_avg_std(host, nseg, stride, begin, length, 0))


def _edge_segments(n):
    rng = np.random.default_rng(7)
    segs = [
        np.full(n, 12345, np.uint32),                                   # all equal
        np.where(rng.random(n) < 0.5, 10, 20).astype(np.uint32),       # two values
        rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32),  # full 32-bit range
        (2**24 + rng.integers(-3, 4, size=n)).astype(np.uint32),       # u32->f32 rounding edge
        np.sort(rng.integers(100, 200, size=n).astype(np.uint32)),     # sorted, narrow
        np.sort(rng.integers(100, 2**31, size=n).astype(np.uint32))[::-1].copy(),  # reverse
        # one huge bucket: most values clustered, few outliers (forces deeper levels)
        np.concatenate([np.full(n - min(n, 3), 1_000_000, np.uint32) +
                        rng.integers(0, 7, size=n - min(n, 3)).astype(np.uint32),
                        np.array([1, 4_000_000_000, 7][:min(n, 3)], np.uint32)]),
        (rng.integers(0, 2**20, size=n) * 4096 + 5).astype(np.uint32),  # sparse keys
        np.zeros(n, np.uint32),                                          # 0-ns durations
        # tight cluster + one low outlier: variance far below mean^2 (cancellation-prone)
        np.where(np.arange(n) == n - 1, 10, 100_000 + rng.integers(0, 20, size=n)).astype(np.uint32),
    ]
    return segs


@pytest.mark.parametrize("mode", [ops.STATS_FAST, ops.STATS_EXACT])
@pytest.mark.parametrize("n", [1, 2, 5, 64, 100, 1024, 3000, 8192])
def test_edge_distributions(mode, n):
    segs = _edge_segments(n)
    host = np.concatenate(segs)
    ns = torch.from_numpy(host.view(np.int32)).to(DEV)
    st = ops.segment_stats_strided(ns, len(segs), n, 0, n, cap=0, mode=mode)
    ref = _oracle_segments(host, len(segs), n, 0, n, 0)
    if mode == ops.STATS_EXACT:
        _check(st, ref, exact_fields=FIELDS + ("avg", "std"))
    else:
        _check(st, ref)
        avg, std = _exact_avg_std(host, len(segs), n, 0, n, 0)
        g = st.cpu()
        np.testing.assert_allclose(g.avg.numpy(), avg, rtol=2.5e-7, atol=1e-30)
        np.testing.assert_allclose(g.std.numpy(), std, rtol=1e-6, atol=1e-6 * avg.max())


@pytest.mark.parametrize("mode", [ops.STATS_FAST, ops.STATS_EXACT])
def test_ragged_segments(mode):
    rng = np.random.default_rng(11)
    lens = np.array([0, 1, 3, 17, 64, 257, 1000, 4096, 8192, 9000, 20000, 5, 2], np.int64)
    cap = 8192
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    host = rng.integers(2000, 2_200_000, size=int(off[-1]), dtype=np.uint32)
    ns = torch.from_numpy(host.view(np.int32)).to(DEV)
    st = ops.segment_stats_ragged(ns, torch.from_numpy(off).to(DEV), None,
                                  max_len=int(lens.max()), cap=cap, mode=mode)
    g = st.cpu()
    for s, L in enumerate(lens):
        seg = host[off[s]:off[s + 1]]
        if L == 0:
            assert g.num[s].item() == 0 and np.isnan(g.med[s].item())
            continue
        r = O.compute_stats(O.ns_to_us(seg[-min(L, cap):]))
        assert g.num[s].item() == r.num_calls
        for f, rf in (("min", "min"), ("max", "max"), ("med", "median")):
            assert np.float32(getattr(g, f)[s].item()) == np.float32(getattr(r, rf)), (s, f)
        if mode == ops.STATS_EXACT:
            assert np.float32(g.avg[s].item()) == np.float32(r.avg)
            assert np.float32(g.std[s].item()) == np.float32(r.stddev)
        else:
            assert abs(g.avg[s].item() - r.avg) <= 1e-4 * r.avg


def test_ring_cap_seven():
    # test_cupti_ext.py:107-127: statsMaxLenPerKernel=7, 21 pushes -> num_calls == 7
    host = np.arange(1, 22, dtype=np.uint32) * 1000
    ns = torch.from_numpy(host.view(np.int32)).to(DEV)
    for mode in (ops.STATS_FAST, ops.STATS_EXACT):
        g = ops.segment_stats_strided(ns, 1, 21, 0, 21, cap=7, mode=mode).cpu()
        assert g.num[0].item() == 7
        assert g.min[0].item() == 15.0 and g.max[0].item() == 21.0 and g.med[0].item() == 18.0


def test_shape_errors_raise():
    ns = torch.zeros(100, dtype=torch.int32, device=DEV)
    with pytest.raises(ValueError):
        ops.segment_stats_strided(ns, 2, 60, 0, 60)
    with pytest.raises(RuntimeError):
        ops.segment_stats_strided(ns, 1, 100, 0, 100, cap=0, mode=7)


# ---- short strided segments: every length class up to 1024 kept, all four 16-B phases
@pytest.mark.parametrize("length", [1, 2, 3, 5, 16, 63, 64, 65, 100, 127, 128, 129, 255, 256, 257,
                                    511, 512, 513, 1000, 1021, 1024])
@pytest.mark.parametrize("nseg", [4, 5, 7, 33])
def test_short_segments_parity(length, nseg):
    rng = np.random.default_rng(length * 100 + nseg)
    for begin in (0, 1, 2, 3):
        stride = (length + begin + 3) // 4 * 4 + 4 * int(rng.integers(0, 3))
        host = rng.integers(1000, 3_000_000, size=nseg * stride, dtype=np.uint32)
        ns = torch.from_numpy(host.view(np.int32)).to(DEV)
        st = ops.segment_stats_strided(ns, nseg, stride, begin, length, cap=0, mode=ops.STATS_FAST)
        ref = _oracle_segments(host, nseg, stride, begin, length, 0)
        _check(st, ref, avg_std=_exact_avg_std(host, nseg, stride, begin, length, 0))


@pytest.mark.parametrize("n", [1, 2, 5, 64, 100, 1024])
def test_short_segments_edge_distributions(n):
    segs = _edge_segments(n)
    stride = (n + 3) // 4 * 4
    host = np.zeros(len(segs) * stride, np.uint32)
    for i, sgm in enumerate(segs):
        host[i * stride:i * stride + n] = sgm
    ns = torch.from_numpy(host.view(np.int32)).to(DEV)
    st = ops.segment_stats_strided(ns, len(segs), stride, 0, n, cap=0, mode=ops.STATS_FAST)
    _check(st, _oracle_segments(host, len(segs), stride, 0, n, 0))


def test_config3_shape_with_colref():
    # configs[2] shape scaled down: S=1024 per (rank, kernel), and a pushed-1500 / cap-1024 ring
    for S, cap in ((1024, 8192), (1500, 1024)):
        R, K = 9, 24
        ns = synth.synth_matrix(R, K, S, device=DEV)
        col = torch.empty(2 * K, dtype=torch.int32, device=DEV)
        st = ops.segment_stats_strided(ns.view(-1), R * K, S, 0, S, cap=cap, col_ref=col, ncols=K)
        host = ns.cpu().numpy().view(np.uint32).reshape(-1)
        ref = _oracle_segments(host, R * K, S, 0, S, cap)
        _check(st, ref, avg_std=_exact_avg_std(host, R * K, S, 0, S, cap))
        want = O.kernel_ref(ref["num"].reshape(R, K), ref["med"].reshape(R, K))
        got = col.cpu().numpy()
        assert np.array_equal(got[:K].view(np.float32), want) and not got[K:].any()


# ---- classified ragged path (segment_ragged.hip): >= 4096 segments, lengths mixed
def _mixed_lengths(rng, nseg, longest):
    u = rng.random(nseg)
    lens = np.where(u < 0.10, 0,
           np.where(u < 0.50, rng.integers(1, 9, nseg),
           np.where(u < 0.70, rng.integers(9, 33, nseg),
           np.where(u < 0.80, rng.integers(33, 65, nseg),
           np.where(u < 0.90, rng.integers(65, 1001, nseg),
           np.where(u < 0.995, rng.integers(1001, 8193, nseg),
                    rng.integers(8193, longest + 1, nseg)))))))
    return lens.astype(np.int64)


@pytest.mark.parametrize("mode", [ops.STATS_FAST, ops.STATS_EXACT])
@pytest.mark.parametrize("aligned16", [False, True])
@pytest.mark.parametrize("cap", [0, 8192, 40])
def test_ragged_length_classes(mode, aligned16, cap):
    rng = np.random.default_rng(7 + cap + 2 * aligned16 + 5 * mode)
    rows, ncols = 60, 80
    nseg = rows * ncols
    lens = _mixed_lengths(rng, nseg, 20000)
    # retained runs start 16-B aligned (aligned16: the promise is about the retained
    # run, last min(len, cap) samples) or at arbitrary 4-B offsets
    keeps = np.minimum(lens, cap) if cap > 0 else lens
    off = np.zeros(nseg, np.int64)
    pos = 0
    for s in range(nseg):
        if aligned16:
            pos += (-(pos + lens[s] - keeps[s])) % 4
        else:
            pos += int(rng.integers(0, 3))
        off[s] = pos
        pos += int(lens[s])
    total = pos + 8
    host = rng.integers(1000, 5_000_000, size=total, dtype=np.uint32)
    # a few tightly clustered / duplicate-heavy segments
    for s in rng.choice(nseg, 50, replace=False):
        host[off[s]:off[s] + lens[s]] = 777_000 + rng.integers(0, 3, lens[s])
    ns = torch.from_numpy(host.view(np.int32)).to(DEV)
    col = torch.empty(2 * ncols, dtype=torch.int32, device=DEV)
    st = ops.segment_stats_ragged(ns, torch.from_numpy(off).to(DEV),
                                  torch.from_numpy(lens.astype(np.int32)).to(DEV),
                                  max_len=int(lens.max()), cap=cap, mode=mode,
                                  aligned16=aligned16, col_ref=col, ncols=ncols)
    g = st.cpu()
    num = np.empty(nseg, np.int32)
    med = np.empty(nseg, np.float32)
    for s in range(nseg):
        L = int(lens[s])
        seg = host[off[s]:off[s] + L]
        keep = min(L, cap) if cap > 0 else L
        r = O.compute_stats(O.ns_to_us(seg[L - keep:]))
        num[s], med[s] = r.num_calls, r.median
        if keep == 0:
            assert g.num[s].item() == 0 and np.isnan(g.med[s].item()) and np.isnan(g.std[s].item())
            continue
        got = [np.float32(getattr(g, f)[s].item()) for f in ("min", "max", "med", "avg", "std")]
        want = [np.float32(x) for x in (r.min, r.max, r.median, r.avg, r.stddev)]
        assert g.num[s].item() == r.num_calls, s
        assert got[:3] == want[:3], (s, keep, got, want)
        if mode == ops.STATS_EXACT or keep <= 128:  # lane / workgroup classes: every field
            assert got[3:] == want[3:], (s, keep, got, want)
        else:
            v = seg[L - keep:].astype(np.float64)
            assert abs(got[3] - v.mean() / 1000) <= 2.5e-7 * v.mean() / 1000 or got[3] == want[3], s
            assert abs(got[4] - v.std() / 1000) <= 1e-6 * v.std() / 1000 + 1e-6 or got[4] == want[4], s
    want_ref = O.kernel_ref(num.reshape(rows, ncols), med.reshape(rows, ncols))
    c = col.cpu().numpy()
    missing = c[ncols:] != 0
    assert np.array_equal(missing, (num.reshape(rows, ncols) == 0).any(axis=0))
    ok = ~missing
    assert np.array_equal(c[:ncols].view(np.float32)[ok], want_ref[ok])


@pytest.mark.parametrize("mode", [ops.STATS_FAST, ops.STATS_EXACT])
@pytest.mark.parametrize("aligned16", [False, True])
def test_ragged_class_boundaries(mode, aligned16):
    # every length of the lane classes (1..129: the sorting networks, the class-restricted
    # masks and the multiplexer selects of s[n-1], s[n/2], s[n/2-1] at both edges of each
    # class) and the wave-class edges, 6 segments each, with ties and a wide-range segment;
    # lane classes are bit-exact in every field in both modes
    rng = np.random.default_rng(20261017)
    lens = list(range(1, 130)) + [255, 256, 257, 258, 511, 512, 513, 1023, 1024, 1025, 4096, 4097, 8192]
    lens = np.repeat(np.array(lens, np.int64), 6)
    if aligned16:
        lens = (lens + 3) // 4 * 4  # 16-byte aligned starts
    off = np.zeros(len(lens) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    host = rng.integers(2000, 2_200_000, size=int(off[-1]), dtype=np.uint32)
    host[off[6]:off[7]] = 5000  # all ties
    host[off[-2]:off[-1]:3] = rng.integers(1 << 30, 1 << 32, size=len(host[off[-2]:off[-1]:3]), dtype=np.uint32)
    ns = torch.from_numpy(host.view(np.int32)).to(DEV)
    st = ops.segment_stats_ragged(ns, torch.from_numpy(off).to(DEV), None, max_len=int(lens.max()),
                                  cap=8192, mode=mode)
    g = st.cpu()
    for s, L in enumerate(lens):
        r = O.compute_stats(O.key_to_us(host[off[s]:off[s + 1]]))  # u32 duration keys
        got = [np.float32(getattr(g, f)[s].item()) for f in ("min", "max", "med", "avg", "std")]
        want = [np.float32(x) for x in (r.min, r.max, r.median, r.avg, r.stddev)]
        assert g.num[s].item() == r.num_calls == L, s
        assert got[:3] == want[:3], (s, L, got, want)
        if mode == ops.STATS_EXACT or L <= 128:
            assert got[3:] == want[3:], (s, L, got, want)
        else:  # FAST: exact mean / std rounded once, or (a segment too long for a misaligned
            # wave, sent to the workgroup kernel) the reference's own values
            v = key_values(host[off[s]:off[s + 1]])
            assert abs(got[3] - v.mean() / 1000) <= 2.5e-7 * v.mean() / 1000 or got[3] == want[3], (s, L)
            assert abs(got[4] - v.std() / 1000) <= 1e-6 * v.std() / 1000 + 1e-6 or got[4] == want[4], (s, L)


@pytest.mark.parametrize("n,mult", [(256, 3601), (512, 3601), (1024, 3550), (256, 7087)])
def test_grouped_full_segments(n, mult):
    """Full segments of <= 1024 samples run the group kernel (several segments per wave, the
    epilogue once per group, lane-parallel): enough segments for groups of > 1 (nseg / 32768),
    a partial last group, the edge distributions (full 32-bit range = wide keys, clusters,
    zeros) at the first, last and middle positions of groups, and the fused column reference."""
    rng = np.random.default_rng(n)
    K = 37
    nseg = K * mult
    group = min(8, max(1, nseg // 32768))  # segment_kernels.h lean_group
    assert group > 1 and nseg % group  # groups of 4 or 8 and a partial last group
    host = rng.integers(2000, 2_200_000, size=nseg * n, dtype=np.uint32)
    edges = _edge_segments(n)
    where = [0, group - 1, group, 5 * group + group // 2, nseg - 1, nseg - group, 3 * group - 1,
             nseg // 2, 7 * group + 1, 11 * group - 1]
    for w, seg in zip(where, edges):
        host[w * n:(w + 1) * n] = seg
    ns = torch.from_numpy(host.view(np.int32)).to(DEV)
    col = torch.empty(2 * K, dtype=torch.int32, device=DEV)
    st = ops.segment_stats_strided(ns, nseg, n, 0, n, cap=0, mode=ops.STATS_FAST, col_ref=col, ncols=K)
    ref = _oracle_segments(host, nseg, n, 0, n, 0)
    _check(st, ref)
    # FAST AVG / STD against the exact moments (vectorised: segments of the random bulk are
    # below the wide-key threshold; the edge segments take key_values)
    g = st.cpu()
    x = host.reshape(nseg, n).astype(np.float64)
    avg, std = x.mean(axis=1) / 1000.0, x.std(axis=1) / 1000.0
    for w in where:
        v = key_values(host[w * n:(w + 1) * n])
        avg[w], std[w] = v.mean() / 1000.0, v.std() / 1000.0
    np.testing.assert_allclose(g.avg.numpy(), avg, rtol=2.5e-7, atol=1e-30)
    np.testing.assert_allclose(g.std.numpy(), std, rtol=1e-6, atol=1e-6 * avg.max())
    want = O.kernel_ref(ref["num"].reshape(-1, K), ref["med"].reshape(-1, K))
    got = col.cpu().numpy()
    assert np.array_equal(got[:K].view(np.float32), want) and not got[K:].any()


@pytest.mark.parametrize("keep,nfull", [(1024, 4 * 8300 + 3), (2048, 4 * 40 + 1), (4096, 4 * 25 + 2),
                                        (8192, 4 * 30 + 3)])
def test_full_class_segments(keep, nfull):
    """The FULL classes (FAST, 16-B aligned retained runs of exactly keep = 64 * PL samples,
    PL 16..128: seg_stats_list_full_kernel, four list entries per wave, one lane-parallel
    epilogue): rings at capacity (length == keep) and overflowed ones (length > keep, the last
    keep retained) mixed with the neighbouring list / lane classes; the edge distributions
    (wide keys take the decoded moments) at the first, last and a middle entry of a group and in
    a partial last group; for keep 1024 more entries than one sweep of the grid covers."""
    rng = np.random.default_rng(keep + nfull)
    nother = 300
    lens = np.concatenate([np.where(rng.random(nfull) < 0.5, keep, keep + rng.integers(1, keep, nfull)),
                           rng.choice([keep - 1, keep - 4, keep // 2 + 3, 100, 9], nother)]).astype(np.int64)
    perm = rng.permutation(lens.size)
    lens = lens[perm]
    off = np.zeros(lens.size, np.int64)
    pos = 0
    for s, L in enumerate(lens):
        keep_s = min(int(L), keep)
        pos += (-(pos + int(L) - keep_s)) % 4  # the retained run starts 16-B aligned
        off[s] = pos
        pos += int(L)
    host = rng.integers(2000, 2_200_000, size=pos + 8, dtype=np.uint32)
    full = np.flatnonzero(lens >= keep)
    assert full.size == nfull
    edges = _edge_segments(keep)
    # list positions of the FULL class follow segment order: entries 0, 3, 4, 5, the middle and
    # the last three (the partial last group)
    at = [0, 3, 4, 5, nfull // 2, nfull - 1, nfull - 2, nfull - 3, 9, 14]
    for a, seg in zip(at, edges):
        s = full[a]
        host[off[s] + lens[s] - keep: off[s] + lens[s]] = seg
    ns = torch.from_numpy(host.view(np.int32)).to(DEV)
    st = ops.segment_stats_ragged(ns, torch.from_numpy(off).to(DEV),
                                  torch.from_numpy(lens.astype(np.int32)).to(DEV),
                                  max_len=int(lens.max()), cap=keep, mode=ops.STATS_FAST, aligned16=True)
    g = st.cpu()
    # the retained windows of the FULL segments as a matrix: the oracle's threaded matrix path
    idx = (off[full] + lens[full] - keep)[:, None] + np.arange(keep)[None, :]
    win = np.ascontiguousarray(host[idx]).reshape(-1)
    ref = _oracle_segments(win, nfull, keep, 0, keep, 0)
    for f in FIELDS:
        a = getattr(g, f).numpy()[full]
        b = ref[f]
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (f, keep)
    x = host[idx].astype(np.float64)
    avg, std = x.mean(axis=1) / 1000.0, x.std(axis=1) / 1000.0
    for a, _ in zip(at, edges):
        v = key_values(host[idx[a]])
        avg[a], std[a] = v.mean() / 1000.0, v.std() / 1000.0
    np.testing.assert_allclose(g.avg.numpy()[full], avg, rtol=2.5e-7, atol=1e-30)
    np.testing.assert_allclose(g.std.numpy()[full], std, rtol=1e-6, atol=1e-6 * avg.max())
    for s in np.flatnonzero(lens < keep):  # the other classes, against computeStats
        L = int(lens[s])
        r = O.compute_stats(O.key_to_us(host[off[s]:off[s] + L]))
        assert g.num[s].item() == r.num_calls == L
        got = [np.float32(getattr(g, f)[s].item()) for f in ("min", "max", "med")]
        assert got == [np.float32(x) for x in (r.min, r.max, r.median)], (s, L)
