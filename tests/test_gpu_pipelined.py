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
    # (timing_reps: a timed report's statistics phase runs three times back to back: same results)
    pipe = b.pipelined(ns, S, timing=True, timing_reps=3)
    # (no reset_history: the warm-up pass of the capture leaves the individual history as it
    # was, ADVICE r03 -- ns holds uninitialised memory here)
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


@pytest.mark.parametrize("R", [8, 300])
def test_error_flags_per_report_and_column_reference_reset(R):
    """The scores epilogue (nvrx_score_args.done, R <= 256) stores each report's error bits and
    re-initialises the column reference itself: a report whose MED is 0 (ZeroDivisionError in
    the reference) sets err bit 1, the next clean report reads 0 again, and its reference (hence
    its relative scores) is that of its own input alone -- eager, graph-replayed and pipelined.
    R = 300 takes the column-reduction path (no epilogue; err zeroed per report)."""
    K, S = 64, 200
    good = synth.synth_matrix(R, K, S, seed=7, device="cuda")
    bad = good.clone()
    bad[1, 3, :] = 0  # kernel 3 of rank 1: every retained duration 0 ns -> MED 0
    fast = good.clone().view(R, K, S)
    fast[:, :, :] //= 2  # halved durations: a different per-kernel reference
    fresh = batch.MatrixReporter(R, K, cap=512, thr_rel=0.8, thr_ind=0.8)
    want_fast = fresh.report(fast, S)
    rep = batch.MatrixReporter(R, K, cap=512, thr_rel=0.8, thr_ind=0.8)
    assert rep.report(bad, S).err & 1
    assert rep.report(good, S).err == 0
    rep.reset_history()
    np.testing.assert_array_equal(rep.report(fast, S).gpu_relative, want_fast.gpu_relative)
    g = rep.graph(good, S)
    good_copy = good.clone()
    assert g.run().err == 0
    good.copy_(bad)
    assert g.run().err & 1
    good.copy_(good_copy)
    assert g.run().err == 0
    pipe = rep.pipelined(good, S)
    for src, want in ((bad, 1), (good_copy, 0), (bad, 1)):
        good.copy_(src)
        pipe.submit()
        res, _ = pipe.collect()
        assert (res.err & 1) == want


@pytest.mark.parametrize("R", [64, 300])
def test_pipelined_records_matches_eager_reports(R):
    """MatrixReporter.pipelined_records: record-stream reports (bucketing, classification, the
    class kernels on the caller's and the side stream, stream-ordered scratch) captured as whole
    graphs, two in flight -- report for report the results of eager report_records, the
    individual history included.  R = 64 takes the fused reference and the pinned-buffer scores
    epilogue, R = 300 the column reduction and the result copy."""
    K, cap = 256, 128
    counts = synth.zipf_counts(K, top=512)
    slot, occ = synth.zipf_order(counts)
    t = lambda a: torch.from_numpy(a.view(np.int32)).cuda()  # noqa: E731
    N = slot.size
    streams = [synth.synth_records(R, t(slot), t(occ), K, int(counts.max()), seed=11 + i)
               for i in range(2)]
    rec_off = torch.arange(R + 1, dtype=torch.int64, device="cuda") * N
    a = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    b = batch.MatrixReporter(R, K, cap=cap, thr_rel=0.8, thr_ind=0.8)
    want = [a.report_records(streams[i % 2], rec_off) for i in range(5)]
    recs = torch.empty_like(streams[0])
    pipe = b.pipelined_records(recs, rec_off, timing=True, timing_reps=2)
    got = []
    for i in range(5):
        recs.copy_(streams[i % 2])
        pipe.submit(timed=i == 2)
        res, ms = pipe.collect()
        assert (ms is not None and ms > 0.0) if i == 2 else ms is None
        got.append(res)
    for w, g in zip(want, got):
        assert g.err == w.err == 0
        np.testing.assert_array_equal(w.gpu_relative, g.gpu_relative)
        np.testing.assert_array_equal(w.gpu_individual, g.gpu_individual)
        np.testing.assert_array_equal(w.stragglers_relative, g.stragglers_relative)
        np.testing.assert_array_equal(w.stragglers_individual, g.stragglers_individual)
    for f in ("num", "min", "max", "med", "avg", "std"):
        assert torch.equal(getattr(a.stats, f).view(torch.int32), getattr(b.stats, f).view(torch.int32)), f


def test_unpaired_statistics_replay_is_refused():
    """a captured statistics graph trusts the column reference that the previous
    report's scores epilogue re-initialised; replayed twice without its scores it would reuse a
    stale reference.  The replay order is checked, and paired replays still match report()."""
    R, K, S = 8, 64, 1000
    ns = synth.synth_matrix(R, K, S, device="cuda")
    rep = batch.MatrixReporter(R, K, cap=512, thr_rel=0.8, thr_ind=0.8)
    want = rep.report(ns, S)
    g = rep.graph(ns, S)
    pipe = rep.pipelined(ns, S)
    g.run_stats()
    with pytest.raises(RuntimeError):
        g.run_stats()
    with pytest.raises(RuntimeError):
        g.run()
    with pytest.raises(RuntimeError):
        pipe.submit()
    res = g.run_rest()  # pairs the first statistics phase: back in order
    np.testing.assert_array_equal(res.stragglers_relative, want.stragglers_relative)
    for res in (g.run(), (pipe.submit(), pipe.collect()[0])[1]):
        np.testing.assert_array_equal(res.stragglers_relative, want.stragglers_relative)


@pytest.mark.parametrize("mode", ["alt", "side", "whole", "alt3"])
@pytest.mark.parametrize("records", [False, True])
def test_two_in_flight_on_two_streams_keep_history_order(records, mode):
    """Two reports in flight on the two streams (each with its own statistics / reference /
    bucketing buffers): report i's scores wait for report i-1's, so the individual history --
    and every score -- equals eager reports in submission order; the inputs change only after
    the reports reading them were collected."""
    R, K = 32, 128
    depth = 3 if mode == "alt3" else 2  # alt3: three reports in flight, two statistics at once
    mode = mode.rstrip("3")
    if records:
        counts = synth.zipf_counts(K, top=600)
        slot, occ = synth.zipf_order(counts)
        t = lambda a: torch.from_numpy(a.view(np.int32)).cuda()  # noqa: E731
        src = [synth.synth_records(R, t(slot), t(occ), K, int(counts.max()), seed=5 + i) for i in range(2)]
        off = torch.arange(R + 1, dtype=torch.int64, device="cuda") * slot.size
        a = batch.MatrixReporter(R, K, cap=256, thr_rel=0.8, thr_ind=0.8)
        b = batch.MatrixReporter(R, K, cap=256, thr_rel=0.8, thr_ind=0.8)
        run = lambda x: a.report_records(x, off)  # noqa: E731
        buf = torch.empty_like(src[0])
        # (pipelined_records has no depth argument: PipelinedReports directly, as it builds it)
        pipe = batch.PipelinedReports(b, None, 0, timing=True, mode=mode, depth=depth,
                                      stats_bytes=8 * buf.shape[0],
                                      stats=lambda: b.compute_stats_records(buf, off))
    else:
        S = 700
        src = [synth.synth_matrix(R, K, S, seed=40 + i, device="cuda") for i in range(2)]
        a = batch.MatrixReporter(R, K, cap=512, thr_rel=0.8, thr_ind=0.8)
        b = batch.MatrixReporter(R, K, cap=512, thr_rel=0.8, thr_ind=0.8)
        run = lambda x: a.report(x, S)  # noqa: E731
        buf = torch.empty_like(src[0])
        pipe = b.pipelined(buf, S, timing=True, mode=mode, depth=depth)
    order = [0, 0, 1, 1, 0, 0, 1, 1]
    want = [run(src[i]) for i in order]
    got = []
    for j in range(0, len(order), 2):
        buf.copy_(src[order[j]])
        pipe.submit()
        pipe.submit(timed=j == 4)
        got += [pipe.collect()[0], pipe.collect()[0]]
    if depth > 2:  # three in flight over one input
        buf.copy_(src[0])
        want3 = [run(src[0]) for _ in range(3)]
        for _ in range(3):
            pipe.submit()
        got3 = [pipe.collect()[0] for _ in range(3)]
        want, got = want + want3, got + got3
    for w, g in zip(want, got):
        np.testing.assert_array_equal(w.gpu_relative, g.gpu_relative)
        np.testing.assert_array_equal(w.gpu_individual, g.gpu_individual)
        np.testing.assert_array_equal(w.stragglers_individual, g.stragglers_individual)


def test_launch_modes_agree_at_full_size():
    """configs[1] at full size (64 x 2048 x 10,000 pushed, 8,192 kept): the bench's launch mode
    (each report on its own stream, the stagger) and whole-report graphs on one stream give the same
    scores, bit for bit, report for report (the individual history included), and the injected
    straggler set."""
    R, K, S = 64, 2048, 10000
    ns = synth.synth_matrix(R, K, S, device="cuda")
    res = {}
    for mode in ("alt", "whole"):
        rep = batch.MatrixReporter(R, K, cap=8192, thr_rel=0.8, thr_ind=0.8)
        pipe = rep.pipelined(ns, S, mode=mode)
        got = []
        pipe.submit()
        for i in range(6):
            if i + 1 < 6:
                pipe.submit()
            got.append(pipe.collect()[0])
        res[mode] = got
    for a, b in zip(res["alt"], res["whole"]):
        assert np.array_equal(a.gpu_relative.view(np.uint64), b.gpu_relative.view(np.uint64))
        assert np.array_equal(a.gpu_individual.view(np.uint64), b.gpu_individual.view(np.uint64))
        assert np.array_equal(a.stragglers_relative, synth.straggler_ranks(R).astype(bool))


def _same(w, g):
    for f in ("gpu_relative", "gpu_individual"):
        assert np.array_equal(getattr(w, f).view(np.uint64), getattr(g, f).view(np.uint64)), f
    np.testing.assert_array_equal(w.stragglers_relative, g.stragglers_relative)
    np.testing.assert_array_equal(w.stragglers_individual, g.stragglers_individual)


@pytest.mark.parametrize("records", [False, True])
def test_eager_work_while_reports_in_flight_is_ordered(records):
    """in the two-stream modes slot 0 is the reporter's own buffer set and
    the history is shared, so report(), a history reset or a graph replay issued between
    submit() and collect() must queue behind the reports in flight.  The mixed sequence gives,
    bit for bit, what the same calls give one at a time on a fresh reporter."""
    R, K = 64, 512
    if records:
        counts = synth.zipf_counts(K, top=2000)
        slot, occ = synth.zipf_order(counts)
        t = lambda a: torch.from_numpy(a.view(np.int32)).cuda()  # noqa: E731
        src = [synth.synth_records(R, t(slot), t(occ), K, int(counts.max()), seed=60 + i) for i in range(2)]
        off = torch.arange(R + 1, dtype=torch.int64, device="cuda") * slot.size
        mk = lambda: batch.MatrixReporter(R, K, cap=1024, thr_rel=0.8, thr_ind=0.8)  # noqa: E731
        a, b = mk(), mk()
        run = lambda rep, x: rep.report_records(x, off)  # noqa: E731
        pipe = b.pipelined_records(src[0], off, mode="alt")
        g = b.graph_records(src[1], off)
    else:
        S = 3000
        src = [synth.synth_matrix(R, K, S, seed=60 + i, device="cuda") for i in range(2)]
        mk = lambda: batch.MatrixReporter(R, K, cap=2048, thr_rel=0.8, thr_ind=0.8)  # noqa: E731
        a, b = mk(), mk()
        run = lambda rep, x: rep.report(x, S)  # noqa: E731
        pipe = b.pipelined(src[0], S, mode="alt")
        g = b.graph(src[1], S)
    want = [run(a, src[0]), run(a, src[1]), run(a, src[0]), run(a, src[0])]
    a.reset_history()
    want += [run(a, src[1]), run(a, src[0]), run(a, src[1])]
    got = []
    pipe.submit()                     # report 1 (src0) in flight on a private stream
    e1 = run(b, src[1])               # report 2, eager, on the caller's stream
    got += [pipe.collect()[0], e1]
    pipe.submit()                     # reports 3, 4 in flight
    pipe.submit()
    b.reset_history()                 # after both
    e5 = g.run()                      # report 5 (src1) as a graph replay
    got += [pipe.collect()[0], pipe.collect()[0], e5]
    pipe.submit()                     # report 6 in flight, then report 7 eager
    e7 = run(b, src[1])
    got += [pipe.collect()[0], e7]
    assert len(got) == len(want)
    for w, x in zip(want, got):
        _same(w, x)


@pytest.mark.parametrize("mode", ["alt", "whole"])
def test_distinct_inputs_per_report_in_flight(mode):
    """pipelined([x0, x1]): report i reads x[i % 2] (bench.py's input-independence control for
    the headline) -- report for report the eager reports over the alternating inputs."""
    R, K, S = 32, 256, 1500
    src = [synth.synth_matrix(R, K, S, seed=80 + i, device="cuda") for i in range(2)]
    a = batch.MatrixReporter(R, K, cap=1024, thr_rel=0.8, thr_ind=0.8)
    b = batch.MatrixReporter(R, K, cap=1024, thr_rel=0.8, thr_ind=0.8)
    want = [a.report(src[i % 2], S) for i in range(6)]
    pipe = b.pipelined(src, S, mode=mode, timing=True)
    got = []
    pipe.submit()
    for i in range(6):
        if i + 1 < 6:
            pipe.submit()
        got.append(pipe.collect()[0])
    for w, x in zip(want, got):
        _same(w, x)
    with pytest.raises(ValueError):  # three input sets do not divide depth 2
        b.pipelined(src + [src[0]], S, mode=mode)


def test_input_modified_in_flight_is_refused():
    """An input changed by a torch in-place op between submit() and collect() is reported
    (the version counter of the tensor moved); changes between reports are fine."""
    R, K, S = 8, 64, 500
    ns = synth.synth_matrix(R, K, S, device="cuda")
    rep = batch.MatrixReporter(R, K, cap=256, thr_rel=0.8, thr_ind=0.8)
    pipe = rep.pipelined(ns, S)
    pipe.submit()
    pipe.collect()
    ns.add_(0)        # between reports: allowed
    pipe.submit()
    ns.add_(0)        # while the report reads it
    with pytest.raises(RuntimeError, match="modified in place"):
        pipe.collect()
    pipe.submit()
    pipe.collect()    # the pipeline goes on
