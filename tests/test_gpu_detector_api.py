"""GPU: the reference's Detector-level unit tests restated (tests/straggler/unit/
test_det_section_api.py, test_sections.py, test_reporting.py, test_reporting_elapsed.py), in this
process or in gloo worlds whose ranks share the one test GPU (tests/_api_workers.py)."""
import inspect

import pytest

from _mp import run_world

pytestmark = pytest.mark.gpu


@pytest.fixture
def detector():
    from nvidia_resiliency_ext import straggler

    straggler.Detector.initialize()
    try:
        yield straggler.Detector
    finally:
        straggler.Detector.shutdown()


def test_reused_name_extends_one_section(detector):
    # test_det_section_api.py:48-55 expects a ValueError but is skipped there: the reference's
    # check is commented out (straggler.py:319), so a name reused at another code location
    # keeps adding entries to the one section -- the behaviour restated here
    with detector.detection_section("section00"):
        pass
    with detector.detection_section("section00"):
        pass
    assert list(detector.custom_sections) == ["section00"]
    assert detector.custom_sections["section00"].total_entry_cnt == 2


def test_default_names_are_unique_and_located(detector):
    # test_det_section_api.py:58-80: an unnamed section is named by its with-block location
    with detector.detection_section():
        pass
    with detector.detection_section():
        pass
    secs = list(detector.custom_sections.values())
    assert len(secs) == 2 and secs[0].name != secs[1].name
    here = inspect.getframeinfo(inspect.currentframe())
    assert secs[1].location.endswith(f"{here.filename}:{here.lineno - 4}")


def test_can_handle_empty_elapseds(detector):
    # test_det_section_api.py:125-137
    with detector.detection_section(name="one", profile_cuda=True):
        pass
    detector.generate_report()
    detector.generate_report()  # every elapsed of "one" was cleared by the first report


SC = dict(avg=0.006, std=0.0015, avg_straggler=0.010, iters=40)


def test_straggler_sections_detected():
    # test_sections.py:75-206 (four of its eight scenarios, one 4-rank world)
    scenarios = [dict(SC, stragglers=[("section00", 0)]),
                 dict(SC, stragglers=[("section00", 0), ("section01", 1)]),
                 dict(SC, stragglers=[]),
                 dict(SC, indiv_stragglers=[("section00", 0), ("section01", 1)])]
    res = run_world(4, "_api_workers", "sections_scenarios", timeout=400, scenarios=scenarios)[0]
    for sc, f in zip(scenarios, res):
        assert not f["straggler_gpus_relative"] and not f["straggler_gpus_individual"]
        for key, kind in (("stragglers", "straggler_sections_relative"),
                          ("indiv_stragglers", "straggler_sections_individual")):
            if key not in sc:
                continue
            if not sc[key]:
                assert not f[kind], f[kind]
            for sec, rank in sc[key]:
                assert sec in f[kind] and [rank, "dummy_node_name"] in [list(x) for x in f[kind][sec]], f


REPORTING = [{"scores_to_compute": "all", "gather_on_rank0": True},
             {"scores_to_compute": "all", "gather_on_rank0": False},
             {"scores_to_compute": ["relative_perf_scores"], "gather_on_rank0": True},
             {"scores_to_compute": ["relative_perf_scores"], "gather_on_rank0": False},
             {"scores_to_compute": ["individual_perf_scores"], "gather_on_rank0": True},
             {"scores_to_compute": ["individual_perf_scores"], "gather_on_rank0": False}]


def test_reporting_options():
    # test_reporting.py:63-190: every scores_to_compute x gather_on_rank0 combination, 2 ranks
    res = run_world(2, "_api_workers", "reporting_options", timeout=400, scenarios=REPORTING)
    assert res[0] == 6 * 3 and res[1] == 3 * 3  # reports checked (rank 1: non-gathering only)


def test_no_gather_called():
    # test_reporting.py:192-204: individual scores without gathering use no all_gather_object
    res = run_world(2, "_api_workers", "reporting_options", timeout=400,
                    scenarios=[{"scores_to_compute": ["individual_perf_scores"],
                                "gather_on_rank0": False}], forbid_gather=True)
    assert res[0] == 3 and res[1] == 3


def test_report_elapsed():
    # test_reporting_elapsed.py:61-200 (wrap_callables and detection_section, gather on/off)
    scenarios = [dict(mode=m, report_time_interval=t, gather_on_rank0=g)
                 for m in ("wrap", "section") for t in (5, 0) for g in (True, False)]
    res = run_world(2, "_api_workers", "report_elapsed", timeout=400, scenarios=scenarios)
    for sc, n0, n1 in zip(scenarios, res[0], res[1]):
        if sc["report_time_interval"] == 0:
            assert n0 > 0  # a report every iteration once the interval is estimated
        if sc["gather_on_rank0"]:
            assert n1 == 0


def test_report_min_interval_is_profiling_interval():
    # test_reporting_elapsed.py:211-245
    res = run_world(2, "_api_workers", "min_interval_is_profiling_interval", timeout=400)
    assert res[0] == res[1] == 1000
