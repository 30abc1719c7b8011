"""GPU: the device-resident record log + ring retention (records.hip) and the profiler
handle that replaces nvrx_cupti_module.CuptiProfiler (test_cupti_ext.py / test_cupti_manager.py
semantics restated)."""
import numpy as np
import pytest
import torch

import oracle as O
from _fastbars import check_avg_std
from nvidia_resiliency_ext.straggler import cupti, ops

pytestmark = pytest.mark.gpu


def _oracle_slot_stats(durations, cap):
    st = O.compute_stats(O.ring_linearize(O.ns_to_us(np.asarray(durations, np.uint32)), cap))
    return (st.num_calls, np.float32(st.min), np.float32(st.max), np.float32(st.median),
            np.float32(st.avg), np.float32(st.stddev))


def _streams(rng, nstreams, nslots, lo, hi):
    """push-ordered record streams {slot, ns} with per-slot counts in [lo, hi]"""
    recs, off = [], [0]
    for _ in range(nstreams):
        counts = rng.integers(lo, hi + 1, size=nslots)
        slots = np.repeat(np.arange(nslots, dtype=np.uint32), counts)
        rng.shuffle(slots)
        ns = rng.integers(1000, 5_000_000, size=slots.size, dtype=np.uint32)
        recs.append(np.stack([slots, ns], axis=1))
        off.append(off[-1] + slots.size)
    return np.concatenate(recs), np.array(off, np.int64)


# (8192, 500, 2000) / (1000, 500, 2000): ~46k records per stream, longer than the LDS stash of a
# wave's chunk head (records.hip), so pass 2 reads both the stash and the memory side
@pytest.mark.parametrize("cap,lo,hi", [(8192, 0, 40), (7, 0, 30), (16, 10, 100), (3, 0, 5),
                                       (8192, 500, 2000), (1000, 500, 2000)])
def test_records_bucket_keeps_last_cap_per_slot(cap, lo, hi):
    rng = np.random.default_rng(cap * 7 + hi)
    nstreams, nslots = 5, 37
    recs, off = _streams(rng, nstreams, nslots, lo, hi)
    d_recs = torch.from_numpy(recs.view(np.int32)).cuda()
    seg_off, seg_len, out_ns, counts = ops.records_bucket(d_recs, torch.from_numpy(off).cuda(),
                                                          nslots, cap)
    seg_off, seg_len, out_ns, counts = (t.cpu().numpy() for t in (seg_off, seg_len, out_ns, counts))
    for t in range(nstreams):
        stream = recs[off[t]:off[t + 1]]
        for s in range(nslots):
            pushed = stream[stream[:, 0] == s, 1]
            g = t * nslots + s
            assert counts[g] == pushed.size
            kept = pushed[-cap:] if cap > 0 else pushed
            assert seg_len[g] == kept.size
            assert seg_off[g] % 4 == 0  # 16-byte aligned runs
            got = out_ns[seg_off[g]:seg_off[g] + seg_len[g]].view(np.uint32)
            if pushed.size > cap:  # overflowed rings are written in push order
                assert np.array_equal(got, kept)
            else:
                assert np.array_equal(np.sort(got), np.sort(kept))
    # the buckets feed the segment-stats kernel directly (aligned runs)
    st = ops.segment_stats_ragged(torch.from_numpy(out_ns).cuda(), torch.from_numpy(seg_off).cuda(),
                                  torch.from_numpy(seg_len).cuda(), max_len=max(1, int(seg_len.max())),
                                  cap=cap, mode=ops.STATS_EXACT, aligned16=True).cpu()
    for t in range(nstreams):
        stream = recs[off[t]:off[t + 1]]
        for s in range(nslots):
            g = t * nslots + s
            pushed = stream[stream[:, 0] == s, 1]
            if pushed.size == 0:
                assert st.num[g].item() == 0
                continue
            r = _oracle_slot_stats(pushed, cap)
            got = (st.num[g].item(), np.float32(st.min[g]), np.float32(st.max[g]),
                   np.float32(st.med[g]), np.float32(st.avg[g]), np.float32(st.std[g]))
            assert got == r, (t, s)


@pytest.fixture
def profiler():
    p = cupti.KernelProfiler(statsMaxLenPerKernel=8192)
    yield p
    p.close()


def test_profiler_singleton(profiler):
    with pytest.raises(RuntimeError):
        cupti.KernelProfiler()


def test_profiler_stats_bit_exact_and_name_sorted(profiler):
    rng = np.random.default_rng(3)
    profiler.initialize()
    profiler.start()
    pushed = {}
    for name in ["zeta_kernel_blk_64_1_1_grid_8_1_1", "alpha_blk_256_1_1_grid_1_1_1", "mid_k"]:
        d = rng.integers(1000, 900_000, size=int(rng.integers(1, 3000)), dtype=np.uint32)
        profiler.push(name, d)
        pushed[name] = d
    stats = profiler.get_stats()
    assert list(stats) == sorted(pushed)
    for name, d in pushed.items():
        s = stats[name]
        r = _oracle_slot_stats(d, 8192)
        assert (s.num_calls, np.float32(s.min), np.float32(s.max), np.float32(s.median),
                np.float32(s.avg), np.float32(s.stddev)) == r, name
    profiler.stop()
    profiler.push("ignored_while_stopped", [5, 6, 7])  # activity disabled: not captured
    assert "ignored_while_stopped" not in profiler.get_stats()
    profiler.reset()
    assert profiler.get_stats() == {}


def test_profiler_ring_cap_seven():
    # test_cupti_ext.py:107-127: statsMaxLenPerKernel=7, 21 executions -> num_calls == 7
    p = cupti.KernelProfiler(statsMaxLenPerKernel=7)
    try:
        p.initialize()
        p.start()
        p.push("mm_kernel", [1000 * (i + 1) for i in range(21)])
        s = p.get_stats()["mm_kernel"]
        assert s.num_calls == 7 and s.min == 15.0 and s.max == 21.0 and s.median == 18.0
        # results survive stop; a later start keeps accumulating (test_cupti_ext.py:23-105)
        p.stop()
        p.start()
        p.push("mm_kernel", [50_000])
        s = p.get_stats()["mm_kernel"]
        assert s.num_calls == 7 and s.max == 50.0 and s.min == 16.0
    finally:
        p.close()


def test_profiler_compaction_keeps_retention_semantics():
    cap = 5
    p = cupti.KernelProfiler(statsMaxLenPerKernel=cap)
    try:
        p.initialize()
        p.start()
        rng = np.random.default_rng(9)
        n = (1 << 22) + 4096  # past the compaction threshold
        slots = rng.integers(0, 3, size=n).astype(np.uint32)
        ns = rng.integers(1000, 2_000_000, size=n, dtype=np.uint32)
        for name in ("k0", "k1", "k2"):
            p.register_kernel(name)
        p.push_slots(slots, ns)
        p.get_stats()  # flush -> compaction (log >> retained records)
        p.push_slots(np.array([1, 1], np.uint32), np.array([7, 9], np.uint32))
        st = p.get_stats()
        for s, name in enumerate(("k0", "k1", "k2")):
            d = ns[slots == s]
            if s == 1:
                d = np.concatenate([d, [7, 9]]).astype(np.uint32)
            r = _oracle_slot_stats(d, cap)
            got = st[name]
            assert (got.num_calls, np.float32(got.min), np.float32(got.max),
                    np.float32(got.median)) == r[:4], name
    finally:
        p.close()


def test_cupti_manager_refcount():
    # test_cupti_manager.py:23-87
    m = cupti.CuptiManager(statsMaxLenPerKernel=64)
    try:
        with pytest.raises(RuntimeError):
            m.start_profiling()  # not initialized
        m.initialize()
        m.start_profiling()
        m.start_profiling()
        m.push("k", [1000, 2000])
        m.stop_profiling()
        m.push("k", [3000])           # still started (refcount 1)
        m.stop_profiling()
        m.push("k", [4000])           # stopped: dropped
        assert m.get_results()["k"].num_calls == 3
        with pytest.raises(RuntimeError):
            m.stop_profiling()
        m.reset_results()
        assert m.get_results() == {}
    finally:
        m.shutdown()


# records_bucket (records.hip) + the length-classed ragged kernels.  (52, 8192, 900, 1100): ~52k
# records per stream, past the 16,384 pairs a workgroup holds in VGPRs and its LDS stash, so
# pass 2 re-reads from memory; (500, 100, ...): overflowed rings; (6000, 100, ...) / (9000, 8192,
# ...): large slot tables, whose buckets do not all fit the LDS stage; (20, 1024, ...), (6, 2048,
# ...), (3, 4096, ...): rings at and past a capacity of 64 * PL samples (the FULL classes)
@pytest.mark.parametrize("nslots,cap,lo,hi", [(37, 8192, 0, 40), (37, 5, 0, 30), (3000, 0, 0, 3),
                                              (500, 100, 0, 150), (64, 8192, 60, 70),
                                              (52, 8192, 900, 1100), (6000, 100, 0, 6),
                                              (9000, 8192, 0, 3), (20, 1024, 900, 1300),
                                              (6, 2048, 1900, 2300), (3, 4096, 4000, 4300)])
def test_records_stats_fused_matches_oracle(nslots, cap, lo, hi):
    # every field vs the oracle's ring-push + computeStats restatement
    rng = np.random.default_rng(nslots + cap + hi)
    nstreams = 6
    recs, off = _streams(rng, nstreams, nslots, lo, hi)
    # an empty stream in the middle
    recs = np.concatenate([recs[:off[2]], recs[off[3]:]])
    off = np.concatenate([off[:3], off[3:] - (off[3] - off[2])])
    off = np.concatenate([off[:3], [off[2]], off[3:]])[:nstreams + 1]
    recs = recs[:off[-1]]
    d_recs = torch.from_numpy(np.ascontiguousarray(recs).view(np.int32)).cuda()
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    max_len = int(np.diff(off).max())
    col = torch.empty(2 * nslots, dtype=torch.int32, device="cuda")
    st = ops.records_stats(d_recs, d_off, nslots, cap, max(1, min(max_len, cap) if cap else max_len),
                           mode=ops.STATS_FAST, col_ref=col).cpu()
    ref = O.records_stats(recs, off.astype(np.int64), nslots, cap=cap, nthreads=4)
    for f in ("num", "min", "max", "med"):
        assert np.array_equal(getattr(st, f).numpy().view(np.int32), ref[f].view(np.int32)), f
    # AVG / STD: bit-exact for <= 128 records (lane classes), else bit-exact or within the FAST
    # bars of the exact moments (2.5e-7 / 1e-6)
    xm, xs = O.records_moments(recs, off.astype(np.int64), nslots, cap=cap, nthreads=4)
    check_avg_std(st.avg.numpy(), st.std.numpy(), ref, xm, xs, f"nslots={nslots} cap={cap}")
    num = ref["num"].reshape(nstreams, nslots)
    want = O.kernel_ref(num, ref["med"].reshape(nstreams, nslots))
    c = col.cpu().numpy()
    miss = c[nslots:] != 0
    assert np.array_equal(miss, (num == 0).any(axis=0))
    assert np.array_equal(c[:nslots].view(np.float32)[~miss], want[~miss])


def test_reset_renumbers_slots_across_intervals():
    # a job that sees more distinct composite keys than nvrx_records_max_slots()
    # over its lifetime (dynamic shapes) keeps reporting: reset forgets the kernels, as the
    # reference's reset clears its map (CuptiProfiler.cpp:148-152)
    maxs = int(cupti.N.lib().nvrx_records_max_slots())
    per = maxs // 2 + 7
    p = cupti.KernelProfiler(statsMaxLenPerKernel=64)
    try:
        p.initialize()
        p.start()
        for window in range(3):  # 3 * per > maxs distinct names in all
            names = [f"w{window}_k{i:05d}_blk_64_1_1_grid_{i % 13 + 1}_1_1" for i in range(per)]
            slots = np.array([p.register_kernel(n) for n in names], np.uint32)
            assert slots.min() == 0 and slots.max() == per - 1  # renumbered every interval
            ns = (np.arange(per, dtype=np.uint32) + 1) * 1000
            p.push_slots(np.repeat(slots, 2), np.repeat(ns, 2))
            st = p.get_stats_columns()
            assert st.names == sorted(names)
            assert np.all(st.num == 2)
            order = np.argsort(names)
            np.testing.assert_array_equal(st.med, (ns[order] / 1000).astype(np.float32))
            p.reset()
            assert p.get_stats() == {}
    finally:
        p.close()


def test_profiler_ingest_device_records():
    # the device-side entry (SURVEY 8(b) nvrx_ingest_records): device {slot, ns} records land
    # in the device log in push order after the host records staged before them
    rng = np.random.default_rng(21)
    p = cupti.KernelProfiler(statsMaxLenPerKernel=100)
    try:
        p.initialize()
        names = ["a_blk_1_1_1_grid_1_1_1", "b_blk_1_1_1_grid_1_1_1", "c_blk_1_1_1_grid_1_1_1"]
        slots = [p.register_kernel(n) for n in names]
        dev = torch.from_numpy(np.stack([np.full(5, slots[0], np.uint32),
                                         np.arange(5, dtype=np.uint32) + 1], 1).view(np.int32)).cuda()
        p.ingest(dev, generation=p.generation)  # stopped: ignored
        p.start()
        host_ns = rng.integers(1000, 90_000, size=80, dtype=np.uint32)
        p.push(names[0], host_ns)
        ing = np.stack([rng.integers(0, 3, size=300).astype(np.uint32),
                        rng.integers(1000, 90_000, size=300, dtype=np.uint32)], 1)
        ing[7, 0] = 3  # not a registered slot: not counted
        p.ingest(torch.from_numpy(np.ascontiguousarray(ing).view(np.int32)).cuda(), generation=p.generation)
        st = p.get_stats()
        for s, name in zip(slots, names):
            d = ing[(ing[:, 0] == s), 1]
            if s == slots[0]:
                d = np.concatenate([host_ns, d])  # host records first: ring keeps the last 100
            r = _oracle_slot_stats(d, 100)
            got = st[name]
            assert (got.num_calls, np.float32(got.min), np.float32(got.max), np.float32(got.median),
                    np.float32(got.avg), np.float32(got.stddev)) == r, name
        assert len(st) == 3
    finally:
        p.close()


def test_profiler_ingest_rejects_slots_from_before_a_reset():
    # slots are renumbered by reset; records built from a slot of the previous
    # interval must not be counted under whichever kernel took that number afterwards, and a
    # record of a slot registered only after the ingest call is never counted
    p = cupti.KernelProfiler(statsMaxLenPerKernel=64)
    try:
        p.initialize()
        p.start()
        old = p.register_kernel("old_blk_1_1_1_grid_1_1_1")
        g_old = p.generation
        rec = lambda s, ns: torch.from_numpy(  # noqa: E731
            np.array([[s, ns]] * 4, np.uint32).view(np.int32)).cuda()
        p.reset()
        assert p.generation == g_old + 1
        new = p.register_kernel("new_blk_1_1_1_grid_1_1_1")
        assert new == old == 0  # the same number, another kernel
        with pytest.raises(RuntimeError, match="generation"):
            p.ingest(rec(old, 7000), generation=g_old)
        p.ingest(rec(new, 3000), generation=p.generation)
        p.ingest(rec(1, 5000), generation=p.generation)  # slot 1 is not registered yet: dropped
        later = p.register_kernel("later_blk_1_1_1_grid_1_1_1")
        assert later == 1
        st = p.get_stats()
        assert set(st) == {"new_blk_1_1_1_grid_1_1_1"}
        assert st["new_blk_1_1_1_grid_1_1_1"].num_calls == 4
        assert st["new_blk_1_1_1_grid_1_1_1"].median == np.float32(3.0)
    finally:
        p.close()


def test_profiler_drains_staged_records_at_the_watermark():
    # bufferSize 8 KiB = 1024 records: pushes beyond it go to the device log right away
    # (host memory bounded); the statistics are those of every record
    p = cupti.KernelProfiler(bufferSize=8 * 1024, statsMaxLenPerKernel=8192)
    try:
        p.initialize()
        p.start()
        rng = np.random.default_rng(5)
        all_ns = []
        for _ in range(9):
            d = rng.integers(1000, 500_000, size=700, dtype=np.uint32)
            p.push("k_blk_1_1_1_grid_1_1_1", d)
            all_ns.append(d)
        slots, ns = p.get_records()
        assert np.array_equal(ns, np.concatenate(all_ns))
        r = _oracle_slot_stats(np.concatenate(all_ns), 8192)
        s = p.get_stats()["k_blk_1_1_1_grid_1_1_1"]
        assert (s.num_calls, np.float32(s.median), np.float32(s.avg)) == (r[0], r[3], r[4])
    finally:
        p.close()


@pytest.mark.parametrize("exact", [True, False])
def test_profiler_durations_of_any_length(exact):
    # a hung kernel's magnitude must reach MAX / MED.  The reference keeps
    # (end - start) / 1000.0f (CuptiProfiler.cpp:187) of the u64 difference; duration keys carry
    # f32(ns) exactly, so 6 s, 5000 s and 2^64-1 ns come out as the reference's floats, bit for
    # bit (EXACT: every field; FAST: NUM/MIN/MAX/MED, AVG/STD within the FAST bars)
    ns = np.array([6_000_000_000, 1000, 5_000_000_000_000, 3_758_096_383, 3_758_096_384,
                   2**64 - 1, 250_000, 4_294_967_296], np.uint64)
    p = cupti.KernelProfiler(statsMaxLenPerKernel=64, exact=exact)
    try:
        p.initialize()
        p.start()
        name = "hung_blk_1_1_1_grid_1_1_1"
        p.push(name, ns)
        p.push("one_blk_1_1_1_grid_1_1_1", [7_000_000_000])
        st = p.get_stats()
        ref = O.compute_stats(O.ns_to_us(ns))  # the reference's floats of the raw u64 ns
        s = st[name]
        assert s.num_calls == ns.size
        assert (np.float32(s.min), np.float32(s.max), np.float32(s.median)) == \
            (np.float32(ref.min), np.float32(ref.max), np.float32(ref.median))
        assert np.float32(s.max) == np.float32(np.float32(2.0**64) / np.float32(1000.0))
        if exact:
            assert (np.float32(s.avg), np.float32(s.stddev)) == (np.float32(ref.avg), np.float32(ref.stddev))
        else:
            v = O.key_to_f32(O.duration_key(ns)).astype(np.float64)
            np.testing.assert_allclose(s.avg, v.mean() / 1000, rtol=2.5e-7)
            np.testing.assert_allclose(s.stddev, v.std() / 1000, rtol=1e-6)
        one = st["one_blk_1_1_1_grid_1_1_1"]
        assert one.max == one.median == np.float32(np.float32(7e9) / np.float32(1000.0))
        assert p.saturated() == 6  # durations of >= 3.76 s (wide keys), counted
    finally:
        p.close()


@pytest.mark.parametrize("n", [5, 40, 3000])
def test_records_stats_wide_keys(n):
    # FAST record statistics (records_bucket + ragged classes: lane classes <= 128 records, wave
    # classes above) over buckets mixing narrow and wide duration keys: MIN/MAX/MED bit-exact with the
    # reference's floats, AVG/STD within the FAST bars of the decoded values' moments
    rng = np.random.default_rng(n)
    nslots, nstreams = 3, 2
    d = []
    for t in range(nstreams):
        for s in range(nslots):
            ns = rng.integers(1000, 9_000_000_000 if s != 1 else 5_000_000, size=n, dtype=np.uint64)
            if s == 2:
                ns[rng.integers(0, n)] = 2**63 + 12345
            d.append((s, ns))
    slots = np.concatenate([np.full(x.size, s, np.uint32) for s, x in d])
    keys = np.concatenate([O.duration_key(x) for _, x in d])
    recs = np.ascontiguousarray(np.stack([slots, keys], 1))
    off = np.arange(nstreams + 1, dtype=np.int64) * (nslots * n)
    st = ops.records_stats(torch.from_numpy(recs.view(np.int32)).cuda(), torch.from_numpy(off).cuda(),
                           nslots, 8192, n, mode=ops.STATS_FAST).cpu()
    for g, (s, ns) in enumerate(d):
        ref = O.compute_stats(O.ns_to_us(ns))
        assert st.num[g].item() == n
        got = [np.float32(getattr(st, f)[g].item()) for f in ("min", "max", "med")]
        assert got == [np.float32(ref.min), np.float32(ref.max), np.float32(ref.median)], (g, s)
        if n <= 128:  # lane classes: computeStats' own sequential f32 sums
            assert (np.float32(st.avg[g].item()), np.float32(st.std[g].item())) == \
                (np.float32(ref.avg), np.float32(ref.stddev))
        else:
            v = O.key_to_f32(O.duration_key(ns)).astype(np.float64) if s != 1 else ns.astype(np.float64)
            np.testing.assert_allclose(st.avg[g].item(), v.mean() / 1000, rtol=2.5e-7)
            np.testing.assert_allclose(st.std[g].item(), v.std() / 1000, rtol=1e-6)


def test_profiler_more_kernels_than_one_bucketing_pass():
    # the reference's per-kernel map is unbounded (CuptiProfiler.cpp:189-198);
    # ~20,000 distinct composite keys in ONE report interval (past the 12,288 slots one bucketing
    # pass counts in LDS) are bucketed in passes over slot ranges and reduced like any other
    maxs = int(cupti.N.lib().nvrx_records_max_slots())
    nk = maxs + 7_700
    rng = np.random.default_rng(20_000)
    p = cupti.KernelProfiler(statsMaxLenPerKernel=16)
    try:
        p.initialize()
        p.start()
        names = [f"dyn_{i:06d}_blk_128_1_1_grid_{i % 31 + 1}_1_1" for i in range(nk)]
        slots = np.array([p.register_kernel(n) for n in names], np.uint32)
        cnt = rng.integers(1, 24, size=nk)                   # some rings overflow (cap 16)
        sl = np.repeat(slots, cnt)
        ns = rng.integers(1000, 3_000_000, size=sl.size, dtype=np.uint64)
        order = rng.permutation(sl.size)
        p.push_slots(sl[order], ns[order])
        st = p.get_stats_columns()
        assert len(st.names) == nk and st.names == sorted(names)
        pos = {n: i for i, n in enumerate(st.names)}
        for k in list(range(0, nk, 997)) + [maxs - 1, maxs, maxs + 1, nk - 1]:
            d = ns[order][sl[order] == slots[k]]
            r = _oracle_slot_stats(d, 16)
            i = pos[names[k]]
            got = (int(st.num[i]), np.float32(st.min[i]), np.float32(st.max[i]), np.float32(st.med[i]),
                   np.float32(st.avg[i]), np.float32(st.std[i]))
            assert got == r, names[k]
    finally:
        p.close()


@pytest.mark.parametrize("nslots,cap", [(30_000, 8192), (25_001, 3)])
def test_records_stats_slot_tables_past_one_pass(nslots, cap):
    # nvrx_records_stats / nvrx_records_bucket with more slots than one pass's LDS counters:
    # three passes over slot ranges, every statistic against the oracle
    rng = np.random.default_rng(nslots)
    recs, off = _streams(rng, 3, nslots, 0, 4)
    d_recs = torch.from_numpy(np.ascontiguousarray(recs).view(np.int32)).cuda()
    d_off = torch.from_numpy(off).cuda()
    st = ops.records_stats(d_recs, d_off, nslots, cap, min(cap, 4), mode=ops.STATS_FAST).cpu()
    ref = O.records_stats(recs, off, nslots, cap=cap, nthreads=4)
    for f in ("num", "min", "max", "med", "avg", "std"):  # <= 4 records: bit-exact in every field
        assert np.array_equal(getattr(st, f).numpy().view(np.int32), ref[f].view(np.int32)), f
    seg_off, seg_len, out_ns, counts = (t.cpu().numpy() for t in ops.records_bucket(d_recs, d_off, nslots, cap))
    for t in range(3):
        stream = recs[off[t]:off[t + 1]]
        for s in list(range(0, nslots, 1777)) + [12287, 12288, 24575, 24576, nslots - 1]:
            pushed = stream[stream[:, 0] == s, 1]
            g = t * nslots + s
            assert counts[g] == pushed.size and seg_len[g] == min(pushed.size, cap)
            got = out_ns[seg_off[g]:seg_off[g] + seg_len[g]].view(np.uint32)
            assert np.array_equal(np.sort(got), np.sort(pushed[-cap:]))


@pytest.mark.parametrize("cap", [8192, 700])
def test_records_streams_around_the_register_head(cap):
    # the bucketing kernel holds the first 16 x 64 x 16 = 16,384 record pairs of a stream in
    # registers (read by its 16 waves together) and splits the rest into per-wave chunks: streams
    # of exactly that many records, one more, one fewer, odd lengths, a rest shorter than one
    # chunk per wave, and unaligned stream starts (after an odd-length stream); rings that
    # overflow take the ordered walk.  Every field against the oracle.
    rng = np.random.default_rng(cap + 17)
    nslots = 97
    head = 16 * 64 * 16 * 2  # records
    lens = [head, head + 1, head - 1, head + 2, head + 31, head + 16 * 64 * 2 + 3, 2 * head + 5, 7, 0]
    recs, off = [], [0]
    for n in lens:
        slot = (rng.zipf(1.3, n) - 1) % nslots
        ns = rng.integers(1000, 3_000_000, n)
        recs.append(np.stack([slot, ns], 1).astype(np.uint32))
        off.append(off[-1] + n)
    recs = np.concatenate(recs)
    off = np.array(off, np.int64)
    d_recs = torch.from_numpy(np.ascontiguousarray(recs).view(np.int32)).cuda()
    d_off = torch.from_numpy(off).cuda()
    max_len = int(np.diff(off).max())
    st = ops.records_stats(d_recs, d_off, nslots, cap, max(1, min(max_len, cap) if cap else max_len),
                           mode=ops.STATS_FAST).cpu()
    ref = O.records_stats(recs, off, nslots, cap=cap, nthreads=4)
    for f in ("num", "min", "max", "med"):
        assert np.array_equal(getattr(st, f).numpy().view(np.int32), ref[f].view(np.int32)), f
    xm, xs = O.records_moments(recs, off, nslots, cap=cap, nthreads=4)
    check_avg_std(st.avg.numpy(), st.std.numpy(), ref, xm, xs, f"register head cap={cap}")


def _wide_kat():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "compute_stats_wide_kat.json")) as f:
        return json.load(f)


def _bits(x):
    return int(np.float32(x).view(np.uint32))


@pytest.mark.parametrize("exact", [True, False])
def test_wide_duration_kat_through_profiler(exact):
    """u64 durations of 2^32 ns and more, against the REFERENCE-generated
    fixture (compute_stats_wide_kat.json: ref_ns_to_us + computeStats of the reference build).
    EXACT: every field bit-exact.  FAST: NUM/MIN/MAX/MED bit-exact, AVG/STD bit-exact for rings
    of <= 128 (lane classes), else within the FAST bars of the decoded values' exact moments."""
    kat = _wide_kat()
    for cap in sorted({c["cap"] for c in kat["cases"]}):
        cases = [c for c in kat["cases"] if c["cap"] == cap]
        p = cupti.KernelProfiler(statsMaxLenPerKernel=cap, exact=exact)
        try:
            p.initialize()
            p.start()
            for c in cases:
                p.push(c["name"] + "_blk_1_1_1_grid_1_1_1", np.array(c["ns"], np.uint64))
            st = p.get_stats()
            for c in cases:
                s = st[c["name"] + "_blk_1_1_1_grid_1_1_1"]
                got = [s.num_calls] + [_bits(v) for v in (s.min, s.max, s.median, s.avg, s.stddev)]
                e = c["expect"]
                if exact or e[0] <= 128:
                    assert got == e, c["name"]
                else:
                    assert got[:4] == e[:4], c["name"]
                    v = O.key_to_f32(O.duration_key(np.array(c["ns"], np.uint64)[-cap:])).astype(np.float64)
                    np.testing.assert_allclose(s.avg, v.mean() / 1000, rtol=2.5e-7)
                    np.testing.assert_allclose(s.stddev, v.std() / 1000, rtol=1e-6)
        finally:
            p.close()


@pytest.mark.parametrize("mode", [ops.STATS_EXACT, ops.STATS_FAST])
def test_wide_duration_kat_through_matrix_segments(mode):
    """The same fixture through segment_stats_ragged on duration keys (one segment per case of
    cap 8192; the ring retention of a segment is its last `cap` keys)."""
    kat = _wide_kat()
    cases = [c for c in kat["cases"] if c["cap"] == 8192]
    keys = [O.duration_key(np.array(c["ns"], np.uint64)) for c in cases]
    off = np.zeros(len(keys) + 1, np.int64)
    off[1:] = np.cumsum([k.size for k in keys])
    d = torch.from_numpy(np.concatenate(keys).view(np.int32)).cuda()
    st = ops.segment_stats_ragged(d, torch.from_numpy(off).cuda(), None, int(max(k.size for k in keys)),
                                  cap=8192, mode=mode).cpu()
    for i, c in enumerate(cases):
        got = [int(st.num[i])] + [_bits(getattr(st, f)[i].item()) for f in ("min", "max", "med", "avg", "std")]
        e = c["expect"]
        if mode == ops.STATS_EXACT or e[0] <= 128:
            assert got == e, c["name"]
        else:
            assert got[:4] == e[:4], c["name"]
            v = O.key_to_f32(keys[i]).astype(np.float64)
            np.testing.assert_allclose(st.avg[i].item(), v.mean() / 1000, rtol=2.5e-7)
            np.testing.assert_allclose(st.std[i].item(), v.std() / 1000, rtol=1e-6)


def test_raw_u32_ns_need_encoding():
    """a raw u32 ns of 3.76 s or more is not a duration key.  encode_ns_u32_ turns raw
    ns into keys on the device, after which the reference's f32(ns) / 1000 of a 4.0 s kernel
    comes out bit for bit."""
    raw = np.array([1000, 2000, 4_000_000_000, 3_900_000_123, 4_294_967_295, 3_758_096_384, 7],
                   np.uint32)
    t = torch.from_numpy(raw.view(np.int32).copy()).cuda()
    ops.encode_ns_u32_(t)
    enc = t.cpu().numpy().view(np.uint32)
    assert np.array_equal(enc, O.duration_key(raw.astype(np.uint64)))
    for mode in (ops.STATS_FAST, ops.STATS_EXACT):
        st = ops.segment_stats_strided(t, 1, raw.size, 0, raw.size, mode=mode).cpu()
        ref = O.compute_stats(O.ns_to_us(raw.astype(np.uint64)))
        assert [_bits(getattr(st, f)[0].item()) for f in ("min", "max", "med")] == \
            [_bits(ref.min), _bits(ref.max), _bits(ref.median)]
        assert np.float32(st.max[0].item()) == np.float32(np.float32(4_294_967_295) / np.float32(1000))
    # a larger encoded array: the grid-stride loop, every element
    big = np.random.default_rng(3).integers(0, 2**32, size=1_000_003, dtype=np.uint64).astype(np.uint32)
    tb = torch.from_numpy(big.view(np.int32).copy()).cuda()
    assert np.array_equal(ops.encode_ns_u32_(tb).cpu().numpy().view(np.uint32),
                          O.duration_key(big.astype(np.uint64)))
    # without encoding, a raw 4.0 s reads as a key: the f32 bits of a far longer duration
    raw4 = torch.tensor(np.array([4_000_000_000, 1000], np.uint32).view(np.int32)).cuda()
    st = ops.segment_stats_strided(raw4, 1, 2, 0, 2).cpu()
    assert np.float32(st.max[0].item()) > np.float32(1e15)
    st = ops.segment_stats_strided(ops.encode_ns_u32_(raw4), 1, 2, 0, 2).cpu()
    assert np.float32(st.max[0].item()) == np.float32(np.float32(4e9) / np.float32(1000))
    # the largest key of a u64 duration: f32(2^64) / 1000
    ok = torch.tensor(np.array([5000, 0xF0200000, 3000], np.uint32).view(np.int32)).cuda()
    st = ops.segment_stats_strided(ok, 1, 3, 0, 3, mode=ops.STATS_FAST).cpu()
    assert np.float32(st.max[0].item()) == np.float32(np.float32(2.0**64) / np.float32(1000))


@pytest.mark.parametrize("exact", [True, False])
def test_ring_capacity_beyond_32768(exact):
    """statsMaxLenPerKernel above 32,768 (the reference's ring takes any
    capacity, CuptiProfiler.h:49-51; CircularBuffer.h:23-70).  70,000 pushes of one key into a
    65,536 ring, 40,000 of another and 20 of a third: the oracle's statistics, every field bit
    for bit (rings this long sort in device scratch in both modes)."""
    rng = np.random.default_rng(65536)
    p = cupti.KernelProfiler(statsMaxLenPerKernel=65536, exact=exact)
    try:
        p.initialize()
        p.start()
        pushed = {"long_blk_1_1_1_grid_1_1_1": rng.integers(1000, 3_000_000, size=70_000, dtype=np.uint32),
                  "mid_blk_1_1_1_grid_1_1_1": rng.integers(1000, 30_000, size=40_000, dtype=np.uint32),
                  "short_blk_1_1_1_grid_1_1_1": rng.integers(1000, 30_000, size=20, dtype=np.uint32)}
        pushed["mid_blk_1_1_1_grid_1_1_1"][::7] = 12345  # ties
        for i in range(0, 70_000, 10_000):  # interleaved pushes
            for k, v in pushed.items():
                p.push(k, v[i:i + 10_000])
        st = p.get_stats()
        for k, v in pushed.items():
            r = _oracle_slot_stats(v, 65536)
            s = st[k]
            got = (s.num_calls, np.float32(s.min), np.float32(s.max), np.float32(s.median),
                   np.float32(s.avg), np.float32(s.stddev))
            assert [np.float32(x).view(np.uint32) if i else x for i, x in enumerate(got)] == \
                [np.float32(x).view(np.uint32) if i else x for i, x in enumerate(r)], k
        assert st["long_blk_1_1_1_grid_1_1_1"].num_calls == 65536
    finally:
        p.close()


@pytest.mark.parametrize("mode", [ops.STATS_EXACT, ops.STATS_FAST])
def test_segments_beyond_32768_strided_and_ragged(mode):
    """The statistics entry points take retained segments of any length: strided segments of
    50,000 kept of 60,000, and ragged ones of 33,000 / 100,000 / 5 next to each other."""
    rng = np.random.default_rng(7)
    m = rng.integers(1000, 5_000_000, size=(3, 60_000), dtype=np.uint32)
    d = torch.from_numpy(m.view(np.int32)).cuda()
    st = ops.segment_stats_strided(d, 3, 60_000, 0, 60_000, cap=50_000, mode=mode).cpu()
    for s in range(3):
        r = _oracle_slot_stats(m[s], 50_000)
        got = (int(st.num[s]),) + tuple(np.float32(getattr(st, f)[s].item()) for f in ("min", "max", "med", "avg", "std"))
        assert got == r, s
    lens = [33_000, 100_000, 5]
    vals = [rng.integers(1000, 5_000_000, size=n, dtype=np.uint32) for n in lens]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    d = torch.from_numpy(np.concatenate(vals).view(np.int32)).cuda()
    st = ops.segment_stats_ragged(d, torch.from_numpy(off).cuda(), None, max(lens), cap=0, mode=mode).cpu()
    for s, v in enumerate(vals):
        r = _oracle_slot_stats(v, len(v))
        got = (int(st.num[s]),) + tuple(np.float32(getattr(st, f)[s].item()) for f in ("min", "max", "med", "avg", "std"))
        assert got == r, s
