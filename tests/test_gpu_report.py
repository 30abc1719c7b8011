"""GPU: the HIP-backed ReportGenerator against (a) the reference's own KATs, restated, and
(b) the golden multi-rank scenarios recorded from the reference (tests/golden).

Bar: scores within 1e-6 relative (north_star); NaN where the reference has NaN; same
keys, key order, rank_to_node, all_gather_object counts and NameMapper ids."""
import json
import math
import os

import numpy as np
import pytest

from _mp import run_world
import scenarios as SC

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
W = "_report_workers"


def dec(x):
    return SC.decode_value(x)


def approx(a, b, rtol=1e-12):
    return abs(a - b) <= rtol * abs(b)


# ------------------------------------------------------------ single process KATs
def test_relative_one_rank():
    # test_relative_gpu_scores.py:46-62
    from nvidia_resiliency_ext import straggler
    from _report_workers import get_summary

    rg = straggler.reporting.ReportGenerator(['relative_perf_scores'], gather_on_rank0=False,
                                             node_name='testnode')
    r = rg.generate_report({}, kernel_summaries={'kernel0': get_summary(np.array([1.0, 1.0, 2.0]))})
    assert r.gpu_relative_perf_scores[0] == pytest.approx(1.0)
    r = rg.generate_report({}, kernel_summaries={'kernel0': get_summary(1.25 * np.array([1.0, 1.0, 2.0]))})
    assert r.gpu_relative_perf_scores[0] == pytest.approx(1.0)


def test_individual_one_rank_history():
    # test_individual_gpu_scores.py:46-121: 1.0, 0.8, 0.5, 0.333, 0.25, 0.2, NaN, 1.0, 1.0, 0.5
    from nvidia_resiliency_ext import straggler
    from _report_workers import get_summary

    rg = straggler.reporting.ReportGenerator(['individual_perf_scores'], gather_on_rank0=False,
                                             node_name='testnode')
    a, b = np.array([1.0, 1.0, 2.0]), np.array([2.0, 2.0, 3.0])

    def rep(ks):
        return rg.generate_report({}, kernel_summaries=ks).gpu_individual_perf_scores[0]

    assert rep({'kernel0': get_summary(a), 'kernel1': get_summary(b)}) == pytest.approx(1.0)
    assert rep({'kernel0': get_summary(1.25 * a), 'kernel1': get_summary(1.25 * b)}) == pytest.approx(1 / 1.25)
    assert rep({'kernel0': get_summary(2.0 * a), 'kernel1': get_summary(2.0 * b)}) == pytest.approx(0.5)
    assert rep({'kernel0': get_summary(3.0 * a), 'kernel1': get_summary(3.0 * b)}) == pytest.approx(0.333, abs=0.001)
    assert rep({'kernel0': get_summary(4.0 * a)}) == pytest.approx(0.25)
    assert rep({'kernel1': get_summary(5.0 * b)}) == pytest.approx(0.2)
    assert np.isnan(rep({}))
    assert rep({'new_kernel': get_summary(a), 'another_new_kernel': get_summary(b)}) == pytest.approx(1.0)
    assert rep({'kernel0': get_summary(0.5 * a), 'kernel1': get_summary(0.5 * b)}) == pytest.approx(1.0)
    assert rep({'kernel0': get_summary(a), 'kernel1': get_summary(b)}) == pytest.approx(0.5)


@pytest.mark.parametrize("gather", [False, True])
def test_first_report_sections_only(gather):
    # no kernel captured yet (e.g. sections timed with profile_cuda=False): the GPU scores
    # are NaN (reporting.py:237-253, empty kernel summaries), the section scores are 1.0
    from nvidia_resiliency_ext import straggler
    from _report_workers import get_summary

    rg = straggler.reporting.ReportGenerator(['relative_perf_scores', 'individual_perf_scores'],
                                             gather_on_rank0=gather, node_name='testnode')
    for _ in range(2):
        r = rg.generate_report({'step': get_summary(np.array([3.0, 4.0, 5.0]))}, {})
        assert math.isnan(r.gpu_relative_perf_scores[0])
        assert math.isnan(r.gpu_individual_perf_scores[0])
        assert r.section_relative_perf_scores['step'][0] == pytest.approx(1.0)
        assert r.section_individual_perf_scores['step'][0] == pytest.approx(1.0)


def test_name_mapper_single_rank():
    # test_name_mapper.py:48-123
    from nvidia_resiliency_ext import straggler
    from _report_workers import get_summary

    rg = straggler.reporting.ReportGenerator(scores_to_compute=['relative_perf_scores'],
                                             gather_on_rank0=True)
    rg.generate_report(kernel_summaries={'kernel0': get_summary([1.0, 1.0, 2.0]),
                                         'kernel1': get_summary([2.0, 3.0, 3.0])},
                       section_summaries={'section0': get_summary([1.0, 1.0, 2.0])})
    m = rg.name_mapper
    assert m.kernel_counter == 2 and m.get_kernel_name(0) == 'kernel0' and m.get_kernel_id('kernel1') == 1
    assert m.section_counter == 1 and m.get_section_id('section0') == 0
    rg.generate_report(kernel_summaries={'kernel2': get_summary([1.0, 2.0, 4.0])},
                       section_summaries={'section0': get_summary([1.0, 1.0, 2.0]),
                                          'section1': get_summary([1.0, 2.0, 4.0]),
                                          'section2': get_summary([3.0, 4.0, 4.0])})
    assert m.kernel_counter == 3 and m.get_kernel_id('kernel2') == 2
    assert [m.get_section_id(f'section{i}') for i in range(3)] == [0, 1, 2]
    rg2 = straggler.reporting.ReportGenerator(scores_to_compute=['individual_perf_scores'],
                                              gather_on_rank0=False)
    rg2.generate_report(kernel_summaries={'kernel0': get_summary([1.0, 1.0, 2.0])},
                        section_summaries={'section0': get_summary([1.0, 1.0, 2.0])})
    with pytest.raises(KeyError):
        rg2.name_mapper.get_kernel_id('kernel0')
    with pytest.raises(KeyError):
        rg2.name_mapper.get_section_id('section0')


def test_zero_median_raises_zero_division():
    from nvidia_resiliency_ext import straggler

    S = straggler.Statistic
    rg = straggler.reporting.ReportGenerator(['individual_perf_scores'], gather_on_rank0=False)
    ks = {'k': {S.MIN: 0.0, S.MAX: 0.0, S.MED: 0.0, S.AVG: 0.0, S.STD: 0.0, S.NUM: 3}}
    with pytest.raises(ZeroDivisionError):
        rg.generate_report({}, kernel_summaries=ks)


def test_identify_stragglers_semantics():
    from nvidia_resiliency_ext.straggler import Report, StragglerId

    rep = Report(gpu_relative_perf_scores={0: 1.0, 1: 0.5, 2: float('nan'), 3: 0.75},
                 section_relative_perf_scores={'s': {0: 0.1, 1: 0.9}, 't': {0: 1.0, 1: 1.0}},
                 gpu_individual_perf_scores={0: 0.7, 1: 0.8, 2: 0.2, 3: 1.0},
                 section_individual_perf_scores={},
                 rank_to_node={0: 'a', 1: 'b', 2: 'c', 3: 'd'}, local_section_summaries={},
                 local_kernel_summaries={}, generate_report_elapsed_time=0.0,
                 gather_on_rank0=True, rank=0)
    s = rep.identify_stragglers()
    assert s['straggler_gpus_relative'] == {StragglerId(1, 'b')}      # 0.75 is not < 0.75
    assert s['straggler_gpus_individual'] == {StragglerId(0, 'a'), StragglerId(2, 'c')}
    assert s['straggler_sections_relative'] == {'s': {StragglerId(0, 'a')}}
    assert s['straggler_sections_individual'] == {}


# ------------------------------------------------------------ multi-rank KATs (gloo, one GPU)
@pytest.mark.parametrize("gather", [True, False])
def test_relative_multi_rank(gather):
    res = run_world(4, W, "rel_scores", gather_on_rank0=gather)
    if gather:
        r0 = res[0]
        sc = {int(k): dec(v) for k, v in r0["gpu_relative_perf_scores"].items()}
        assert sorted(sc) == [0, 1, 2, 3]
        for r in range(4):
            assert approx(sc[r], 1.0 / (r + 1), 1e-6)
        assert all(res[r] is None for r in (1, 2, 3))
        assert r0["rank_to_node"] == {str(r): f"testnode{r}" for r in range(4)}
        assert r0["gpu_individual_perf_scores"] == {}
    else:
        for r in range(4):
            sc = res[r]["gpu_relative_perf_scores"]
            assert list(sc) == [str(r)] and approx(dec(sc[str(r)]), 1.0 / (r + 1), 1e-12)
            assert res[r]["rank_to_node"] == {str(r): f"testnode{r}"}


def test_relative_some_common_kernels():
    res = run_world(4, W, "rel_some_common")
    sc = {int(k): dec(v) for k, v in res[0]["gpu_relative_perf_scores"].items()}
    for r in range(4):
        assert approx(sc[r], 1.0 / (r + 1), 1e-6)


@pytest.mark.parametrize("kw", [dict(ranks_with_unique_kernels=(1, 2)),
                                dict(ranks_without_kernels=(1, 3))])
def test_relative_no_common_kernels_all_nan(kw):
    res = run_world(4, W, "rel_no_common", **kw)
    sc = res[0]["gpu_relative_perf_scores"]
    assert len(sc) == 4 and all(math.isnan(dec(v)) for v in sc.values())


@pytest.mark.parametrize("gather", [True, False])
def test_individual_multi_rank(gather):
    res = run_world(4, W, "indiv_scores", gather_on_rank0=gather)
    for r in range(4):
        rep = res[0] if gather else res[r]
        assert approx(dec(rep["gpu_individual_perf_scores"][str(r)]), 1.0 / (r + 1), 1e-6)
        assert rep["gpu_relative_perf_scores"] == {}


@pytest.mark.parametrize("gather", [False, True])
def test_name_mapping_consistency(gather):
    # test_name_mapper.py:126-356 (exact == 0.5 / 1.0, NaN for rank-only sections)
    res = run_world(2, W, "mapping_consistency", gather_on_rank0=gather)
    m0, m1 = res[0], res[1]
    assert m0["kernel_counter"] == 6 and m0["section_counter"] == 6
    assert m0["kernel_ids"] == m1["kernel_ids"] and m0["section_ids"] == m1["section_ids"]
    if not gather:
        r0, r1 = m0["report"], m1["report"]
        assert dec(r0["gpu_relative_perf_scores"]["0"]) == 0.5
        assert dec(r1["gpu_relative_perf_scores"]["1"]) == 1.0
        assert set(r0["section_relative_perf_scores"]) == {"s1", "s2", "rank0_only"}
        assert dec(r0["section_relative_perf_scores"]["s1"]["0"]) == 0.5
        assert dec(r0["section_relative_perf_scores"]["s2"]["0"]) == 0.5
        assert math.isnan(dec(r0["section_relative_perf_scores"]["rank0_only"]["0"]))
        assert dec(r1["section_relative_perf_scores"]["s1"]["1"]) == 1.0
        assert math.isnan(dec(r1["section_relative_perf_scores"]["rank1_only"]["1"]))
    else:
        r0 = m0["report"]
        assert m1["report"] is None
        assert dec(r0["gpu_relative_perf_scores"]["0"]) == 0.5
        assert dec(r0["gpu_relative_perf_scores"]["1"]) == 1.0
        srp = r0["section_relative_perf_scores"]
        assert set(srp) == {"s1", "s2", "initial_section_rank0", "initial_section_rank1",
                            "rank0_only", "rank1_only"}
        assert [dec(v) for v in srp["s1"].values()] == [0.5, 1.0]
        assert [dec(v) for v in srp["s2"].values()] == [0.5, 1.0]
        for name in ("initial_section_rank0", "initial_section_rank1", "rank0_only", "rank1_only"):
            assert list(srp[name]) == ["0", "1"] and all(math.isnan(dec(v)) for v in srp[name].values())


def test_all_gather_object_call_counts():
    res = run_world(4, W, "all_gather_counts", timeout=600)
    for r in range(4):
        assert res[r] == [2, 0, 1, 0, 1], res[r]


# ------------------------------------------------------------ golden scenarios (reference outputs)
def _cmp(got, want, where):
    assert set(got) == set(want), (where, set(got) ^ set(want))
    assert list(got) == list(want), (where, "order")
    for k, v in want.items():
        if isinstance(v, dict):
            _cmp(got[k], v, f"{where}/{k}")
        else:
            g, w = dec(got[k]), dec(v)
            if math.isnan(w):
                assert math.isnan(g), (where, k)
            else:
                assert abs(g - w) <= 1e-6 * abs(w), (where, k, g, w)


@pytest.mark.parametrize("scname", sorted(SC.SCENARIOS))
@pytest.mark.parametrize("stats_source", ["oracle", "gpu_exact"])
def test_golden_scenarios(scname, stats_source):
    with open(os.path.join(HERE, "golden", f"report_{scname}.json")) as f:
        fx = json.load(f)
    sc = SC.SCENARIOS[scname]
    res = run_world(sc["ws"], W, "golden_scenario", scname=scname, stats_source=stats_source)
    for r in range(sc["ws"]):
        got = res[r]
        for t in range(sc["reports"]):
            assert got["digests"][t] == fx["kernel_summary_sha256"][t][r], (t, r)
            want = fx["reports"][t][r]
            if want is None:
                assert got["outs"][t] is None
                continue
            for f in SC.REPORT_FIELDS:
                _cmp(got["outs"][t][f], want[f], f"{scname}/t{t}/r{r}/{f}")
            assert got["outs"][t]["rank_to_node"] == want["rank_to_node"]
        assert got["gathers"] == [fx["all_gather_object_calls"][t][r] for t in range(sc["reports"])]
    if sc["gather"] or "relative_perf_scores" in sc["scores"]:
        assert res[0]["mapper"]["kernel"] == fx["name_mapper"]["kernel"]
        assert res[0]["mapper"]["section"] == fx["name_mapper"]["section"]


def test_dropin_2048_kernels_with_name_churn_matches_restatement():
    """One rank's ReportGenerator at the bench's drop-in size (2,048 kernels, 3 sections) over
    reports whose kernel set repeats (the id / history-slot cache), shrinks, grows and gains
    ncclDev names -- every report's GPU and section scores against the CPU restatement of the
    reference (oracle/oracle_report.py), within the 1e-6 bar; individual history included."""
    import oracle_report as OR

    from nvidia_resiliency_ext.straggler import Statistic as S
    from nvidia_resiliency_ext.straggler import reporting, synth

    rng = np.random.default_rng(11)
    names = synth.kernel_names(2048 + 64)
    base = {n: (int(rng.integers(1, 8193)), float(np.float32(rng.uniform(2.0, 2000.0))))
            for n in names}
    sets = [names[:2048], names[:2048], names[100:2048], names[100:2048] + names[2048:2098],
            names[100:2048] + names[2048:2098],
            names[:2048] + ["ncclDevKernel_AllReduce_blk_256_1_1_grid_8_1_1"]]
    base["ncclDevKernel_AllReduce_blk_256_1_1_grid_8_1_1"] = (5, 3.0)
    scores = ["relative_perf_scores", "individual_perf_scores"]
    gen = reporting.ReportGenerator(scores_to_compute=scores, gather_on_rank0=False)
    sim = OR.SimWorld(1, scores, gather_on_rank0=False)
    for i, ks in enumerate(sets):
        j = 1.0 + 0.03 * ((i * 5) % 7)
        kk = {n: {S.MIN: 0.1, S.MAX: 1e4, S.MED: float(np.float32(base[n][1] * j)),
                  S.AVG: float(np.float32(base[n][1] * j * 1.01)), S.STD: 0.5, S.NUM: base[n][0]}
              for n in ks}
        ss = {f"section_{s}": {S.MIN: 1.0, S.MAX: 9.0, S.MED: 3.0 + s * j, S.AVG: 3.0, S.STD: 0.1,
                               S.NUM: 10} for s in range(3)}
        str_k = {n: {OR.MED: v[S.MED], OR.AVG: v[S.AVG], OR.NUM: v[S.NUM]} for n, v in kk.items()}
        str_s = {n: {OR.MED: v[S.MED], OR.AVG: v[S.AVG], OR.NUM: v[S.NUM]} for n, v in ss.items()}
        got = gen.generate_report(ss, kk)
        want = sim.generate_report([str_s], [str_k])[0]
        for f in ("gpu_relative_perf_scores", "gpu_individual_perf_scores"):
            assert math.isclose(getattr(got, f)[0], want[f][0], rel_tol=1e-6), (i, f)
        for f in ("section_relative_perf_scores", "section_individual_perf_scores"):
            for sec, per_rank in want[f].items():
                assert math.isclose(getattr(got, f)[sec][0], per_rank[0], rel_tol=1e-6), (i, f, sec)
        assert "ncclDevKernel_AllReduce_blk_256_1_1_grid_8_1_1" not in got.local_kernel_summaries
