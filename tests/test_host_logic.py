"""CPU: host-side logic of the scoring path that involves no device -- the report interval
tracker (reference tests/straggler/unit/test_interval_tracker.py), name-id agreement across
ranks (name_mapper.py:56-81) and the dist_utils collectives, on gloo worlds."""

import pytest

from _mp import run_world


def test_interval_estimate_single_process(monkeypatch):
    # a fake monotonic clock in exact binary steps (1/64 s), so the estimate is exact and
    # the test does not depend on how long sleeps take on a loaded host
    from types import SimpleNamespace

    from nvidia_resiliency_ext.straggler import interval_tracker

    clock = SimpleNamespace(t=1000.0)
    monkeypatch.setattr(interval_tracker, "time", SimpleNamespace(monotonic=lambda: clock.t))
    tr = interval_tracker.ReportIntervalTracker()
    tr.time_interval = 0.5
    assert tr.iter_interval is None
    for i in range(120):
        tr.iter_increase()
        clock.t += 1 / 64
        if tr.current_iter <= tr.INTERVAL_ESTIMATION_ITERS:
            assert tr.iter_interval is None
        else:
            assert tr.is_interval_elapsed() == (tr.current_iter % tr.iter_interval == 0)
        if i < tr.INTERVAL_ESTIMATION_ITERS // 2:
            clock.t += 4 / 64  # slow warm-up steps do not move the (lower) median
    assert not tr.step_times
    assert tr.iter_interval == 32  # 0.5 s / (1/64 s)


def test_interval_never_below_profiling_interval():
    from nvidia_resiliency_ext.straggler.interval_tracker import ReportIntervalTracker

    tr = ReportIntervalTracker(time_interval=1e-6, profiling_interval=7)
    for _ in range(tr.INTERVAL_ESTIMATION_ITERS + 1):
        tr.iter_increase()
    assert tr.iter_interval == 7
    with pytest.raises(AssertionError):
        tr._gather_report_interval()


def test_interval_is_max_over_ranks():
    # rank 1 steps 4x faster -> more iterations per interval; every rank takes the MAX
    res = run_world(2, "_host_workers", "interval_world", step_s=[0.02, 0.005])
    assert res[0] == res[1]
    assert 40 <= res[0] <= 90


@pytest.mark.parametrize("ws", [2, 3])
def test_name_ids_agree_across_ranks(ws):
    res = run_world(ws, "_host_workers", "name_mapper_world")
    ref = res[0]
    for r in range(ws):
        assert res[r] == ref
    kid, sid = ref["r1"]
    # gathered order: rank by rank, list order
    want = {}
    for r in range(ws):
        for n in (f"k_rank{r}", "shared"):
            want.setdefault(n, len(want))
    assert kid == want and sid == {"sec": 0}
    assert ref["r2"] == kid
    kid3, sid3 = ref["r3"]
    assert kid3 == {**want, "late_b": len(want), "late_a": len(want) + 1}
    assert sid3 == {"sec": 0, "sec2": 1}


def test_dist_utils_on_gloo():
    res = run_world(3, "_host_workers", "dist_utils_world")
    for r in range(3):
        o = res[r]
        assert (o["ws"], o["rank"], o["dev"]) == (3, r, "cpu")
        assert o["all_true"] is True and o["one_false"] is False
        assert o["objs"] == [{"r": 0}, {"r": 1}, {"r": 2}]
        assert o["sum"] == 6.0
    assert res[0]["gather"] == [[0.0, 0.0], [1.0, 10.0], [2.0, 20.0]]
    assert res[1]["gather"] is None and res[2]["gather"] is None


def test_dist_utils_single_process_is_local():
    import torch

    from nvidia_resiliency_ext.straggler import dist_utils as du

    assert du.get_world_size() == 1 and du.get_rank() == 0
    t = torch.tensor([3.0])
    du.all_reduce(t)
    assert t.item() == 3.0
    assert du.gather_on_rank0(t)[0] is t
    assert du.is_all_true(False) is False and du.all_gather_object(5) == [5]


def test_detection_section_fails_if_not_initialized():
    # test_det_section_api.py:42-46 (no GPU needed: checked before anything is profiled)
    from nvidia_resiliency_ext import straggler

    assert not straggler.Detector.initialized
    with pytest.raises(RuntimeError):
        with straggler.Detector.detection_section("section00"):
            pass


class _FakeEvent:
    """query() turns True after `ready_after` polls (never when None); synchronize() is
    recorded with the time it was called."""

    def __init__(self, ready_after=None):
        import time
        self.t0 = time.perf_counter_ns()
        self.ready_after, self.polls, self.sync_at = ready_after, 0, None

    def query(self):
        self.polls += 1
        return self.ready_after is not None and self.polls > self.ready_after

    def synchronize(self):
        import time
        self.sync_at = time.perf_counter_ns() - self.t0


def test_wait_event_bounded_spin_then_block():
    """the default wait polls for at most SPIN_BOUND_US, then blocks in
    synchronize() (a blocking-sync event) instead of holding a host core for the whole report."""
    from nvidia_resiliency_ext.straggler import batch

    assert batch.sync_mode() == "bounded" or "NVRX_SYNC" in __import__("os").environ
    never = _FakeEvent(ready_after=None)  # a long report: the bound expires, then block
    batch.wait_event(never, mode="bounded", bound_us=50)
    assert never.sync_at is not None and never.polls >= 1
    # the poll loop stopped at the bound (50 us), not after the whole wait; generous slack for
    # a loaded CI host
    assert never.sync_at < 50_000_000, never.sync_at
    quick = _FakeEvent(ready_after=3)  # lands within the bound: no blocking call at all
    batch.wait_event(quick, mode="bounded", bound_us=1e6)
    assert quick.sync_at is None and quick.polls == 4
    spin = _FakeEvent(ready_after=200)  # "spin" (bench.py) never blocks
    batch.wait_event(spin, mode="spin")
    assert spin.sync_at is None and spin.polls == 201
    block = _FakeEvent(ready_after=None)  # "block" blocks at once, no polling
    batch.wait_event(block, mode="block")
    assert block.sync_at is not None and block.polls == 0


def test_sync_mode_switch():
    from nvidia_resiliency_ext.straggler import batch

    prev = batch.set_sync_mode("spin")
    try:
        assert batch.sync_mode() == "spin"
        with pytest.raises(ValueError):
            batch.set_sync_mode("busy")
    finally:
        batch.set_sync_mode(prev)
    assert batch.sync_mode() == prev


def test_summary_columns_and_nccl_filter():
    """Host side of a report on the reference's {name: {Statistic: value}} summaries: the columns
    read for scoring, and the ncclDev filter (reporting.py:330-336) returning a new mapping in
    the caller's order, with or without names to drop."""
    import pickle

    import numpy as np

    from nvidia_resiliency_ext.straggler import Statistic as S
    from nvidia_resiliency_ext.straggler.reporting import ReportGenerator
    from nvidia_resiliency_ext.straggler.summaries import columns_of

    kk = {f"k{i}": {S.MIN: 0.5, S.MAX: 9.0, S.MED: 1.0 + i, S.AVG: 2.0 + i, S.STD: 0.0, S.NUM: 3 + i}
          for i in range(5)}
    med, avg, num = columns_of(kk)
    assert med.dtype == np.float64 and avg.dtype == np.float64 and num.dtype == np.int64
    assert med.tolist() == [1.0, 2.0, 3.0, 4.0, 5.0] and num.tolist() == [3, 4, 5, 6, 7]
    assert [len(c) for c in columns_of({})] == [0, 0, 0]
    out = ReportGenerator._filter_out_nccl_kernels(kk)
    assert out == kk and out is not kk and list(out) == list(kk)
    kk2 = dict(kk)
    kk2["ncclDevKernel_AllReduce_blk_256_1_1_grid_1_1_1"] = kk["k0"]
    kk2["k9"] = kk["k1"]
    out2 = ReportGenerator._filter_out_nccl_kernels(kk2)
    assert list(out2) == ["k0", "k1", "k2", "k3", "k4", "k9"]
    # Statistic keys: identity hash, same dict semantics, survive pickling (all_gather_object)
    d = pickle.loads(pickle.dumps({S.MED: 1.5, S.NUM: 2}))
    assert d[S.MED] == 1.5 and d[S.NUM] == 2 and hash(S.AVG) == object.__hash__(S.AVG)


def test_name_mapper_known_kernels_still_assigns_new_sections():
    """gather_and_assign_ids(kernels_known=True) -- the ReportGenerator's shortcut while the kernel
    names repeat -- skips only the kernel lookups: a new section still gets its id."""
    from nvidia_resiliency_ext.straggler.name_mapper import NameMapper

    nm = NameMapper()
    nm.gather_and_assign_ids(["ka", "kb"], ["s0"])
    assert nm.kernel_name_to_id == {"ka": 0, "kb": 1} and nm.section_name_to_id == {"s0": 0}
    nm.gather_and_assign_ids(["ka", "kb"], ["s0", "s1"], kernels_known=True)
    assert nm.section_name_to_id == {"s0": 0, "s1": 1} and nm.kernel_counter == 2
    nm.gather_and_assign_ids(["ka", "kb", "kc"], ["s1"])
    assert nm.kernel_name_to_id["kc"] == 2
