"""Rank workers for tests/test_gpu_detector_api.py: the reference's Detector-level unit tests
(tests/straggler/unit/test_sections.py, test_reporting.py, test_reporting_elapsed.py) restated
for gloo worlds whose ranks share the one test GPU.  Every worker registers the dispatch capture
before its first HIP call (spawned processes start without one)."""
import random
import time
from unittest import mock


def _capture_first():
    from nvidia_resiliency_ext.straggler import cupti

    cupti.enable_capture()


def _model(dev, hidden=128, layers=4):
    import torch.nn as nn

    return nn.Sequential(*[nn.Linear(hidden, hidden, bias=False) for _ in range(layers)]).to(dev)


# ---------------------------------------------------------------- test_sections.py:27-153
SECTIONS = ("section00", "section01", "section02")


def _section_work(section, rank, sc, slow_iter):
    rel = (section, rank) in sc.get("stragglers", ())
    ind = (section, rank) in sc.get("indiv_stragglers", ())
    mu, sigma = sc["avg"], sc["std"]
    if rel or (ind and slow_iter):
        mu, sigma = sc["avg_straggler"], sc["std"]
    time.sleep(max(0.0, random.gauss(mu, sigma)))


def sections_scenarios(rank, ws, scenarios):
    """For each scenario: 3 sections per iteration timed with sleeps (slower on the straggler
    (section, rank) pairs; individual stragglers slow down only in the second half), one report
    at half time and one at the end; rank 0 returns the final report's straggler sets."""
    _capture_first()
    from nvidia_resiliency_ext import straggler

    out = []
    for sc in scenarios:
        random.seed(rank)
        straggler.Detector.initialize(node_name="dummy_node_name")
        try:
            half = sc["iters"] // 2
            for i in range(sc["iters"]):
                for s in SECTIONS:
                    with straggler.Detector.detection_section(s):
                        _section_work(s, rank, sc, slow_iter=i > half)
                if i == half:
                    straggler.Detector.generate_report()
            rep = straggler.Detector.generate_report()
            if rank == 0:
                f = rep.identify_stragglers()
                out.append({k: (sorted((s.rank, s.node) for s in v) if isinstance(v, set) else
                                {sec: sorted((s.rank, s.node) for s in ids) for sec, ids in v.items()})
                            for k, v in f.items()})
        finally:
            straggler.Detector.shutdown()
    return out


# ---------------------------------------------------------------- test_reporting.py:63-190
def reporting_options(rank, ws, scenarios, iters=12, report_interval=4, forbid_gather=False):
    """wrap_callables(model.forward); a report every `report_interval` iterations; per report
    the checks of test_reporting.py:134-185.  forbid_gather: torch.distributed.all_gather_object
    raises (test_no_gather_called)."""
    _capture_first()
    import torch

    from nvidia_resiliency_ext import straggler

    dev = torch.device("cuda", 0)
    checked = 0
    patcher = None
    if forbid_gather:
        patcher = mock.patch("torch.distributed.all_gather_object",
                             side_effect=RuntimeError("distributed communication must not be used"))
        gather_mock = patcher.start()
    try:
        for sc in scenarios:
            model = _model(dev)
            stc, gather = sc["scores_to_compute"], sc["gather_on_rank0"]
            straggler.Detector.initialize(scores_to_compute=stc, gather_on_rank0=gather)
            straggler.Detector.wrap_callables(callable_ids=[straggler.CallableId(model, "forward")])
            try:
                for i in range(iters):
                    model(torch.rand(16, 128, device=dev))
                    if i % report_interval:
                        continue
                    rep = straggler.Detector.generate_report()
                    if gather and rank != 0:
                        assert rep is None
                        continue
                    n = ws if gather else 1
                    want = ["relative_perf_scores", "individual_perf_scores"] if stc == "all" else stc
                    if "relative_perf_scores" in want:
                        assert len(rep.gpu_relative_perf_scores) == n
                        assert all(len(v) == n for v in rep.section_relative_perf_scores.values())
                    if "individual_perf_scores" in want:
                        assert len(rep.gpu_individual_perf_scores) == n
                        assert all(len(v) == n for v in rep.section_individual_perf_scores.values())
                    f = rep.identify_stragglers()
                    for kind in ("straggler_gpus_relative", "straggler_gpus_individual",
                                 "straggler_sections_relative", "straggler_sections_individual"):
                        assert kind in f
                    assert bool(rep.gpu_relative_perf_scores) == ("relative_perf_scores" in want)
                    assert bool(rep.section_relative_perf_scores) == ("relative_perf_scores" in want)
                    assert bool(rep.gpu_individual_perf_scores) == ("individual_perf_scores" in want)
                    assert bool(rep.section_individual_perf_scores) == ("individual_perf_scores" in want)
                    assert len(rep.local_kernel_summaries) > 0  # captured GEMM kernels
                    checked += 1
            finally:
                straggler.Detector.shutdown()
        if forbid_gather:
            assert gather_mock.call_count == 0
    finally:
        if patcher is not None:
            patcher.stop()
    return checked


# ---------------------------------------------------------------- test_reporting_elapsed.py
def report_elapsed(rank, ws, scenarios, iters=60):
    """generate_report_if_interval_elapsed with wrap_callables (:61-130) or a detection section
    (:140-200): the tracker's iteration count, the estimated interval after 16 timed steps, a
    report exactly when the interval elapsed (rank 0 when gathering)."""
    _capture_first()
    import torch

    from nvidia_resiliency_ext import straggler

    D = straggler.Detector
    dev = torch.device("cuda", 0)
    nreports = []
    for sc in scenarios:
        model = _model(dev)
        D.initialize(report_time_interval=sc["report_time_interval"],
                     gather_on_rank0=sc["gather_on_rank0"])
        if sc["mode"] == "wrap":
            D.wrap_callables(callable_ids=[straggler.CallableId(model, "forward")])
        try:
            got = 0
            for i in range(iters):
                x = torch.rand(16, 128, device=dev)
                if sc["mode"] == "wrap":
                    model(x)
                else:
                    with D.detection_section("fwd", profile_cuda=True):
                        model(x)
                assert i == D.report_interval_tracker.current_iter
                if i > D.report_interval_tracker.INTERVAL_ESTIMATION_ITERS:
                    assert D.report_interval_tracker.iter_interval is not None
                rep = D.generate_report_if_interval_elapsed()
                if not sc["gather_on_rank0"] or rank == 0:
                    assert D.report_interval_tracker.is_interval_elapsed() == (rep is not None)
                assert D.report_interval_tracker.is_interval_elapsed() == D.is_interval_elapsed()
                got += rep is not None
            nreports.append(got)
        finally:
            D.shutdown()
    return nreports


def min_interval_is_profiling_interval(rank, ws, profiling_interval=1000, iters=1100):
    """test_reporting_elapsed.py:211-245: the estimated report interval is never below the
    profiling interval (1000, as there: 0.01 s of ~0.1 ms steps asks for ~100)."""
    _capture_first()
    import torch

    from nvidia_resiliency_ext import straggler

    D = straggler.Detector
    dev = torch.device("cuda", 0)
    model = _model(dev)
    D.initialize(profiling_interval=profiling_interval, report_time_interval=0.01,
                 gather_on_rank0=True)
    try:
        for _ in range(iters):
            with D.detection_section("fwd", profile_cuda=True):
                model(torch.rand(16, 128, device=dev))
            rep = D.generate_report_if_interval_elapsed()
            if D.is_interval_elapsed():  # the same iteration on every rank (report on rank 0)
                assert (rep is not None) == (rank == 0)
                break
        return D.report_interval_tracker.iter_interval
    finally:
        D.shutdown()
