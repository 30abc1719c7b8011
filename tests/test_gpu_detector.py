"""GPU: Detector end to end -- sections timed on the host, kernel executions in the device
record log, section + kernel statistics and every score on HIP kernels."""
import time

import numpy as np
import pytest

import oracle as O
from _mp import run_world

pytestmark = pytest.mark.gpu


def test_detector_single_rank_report():
    from nvidia_resiliency_ext import straggler

    D = straggler.Detector
    D.initialize(scores_to_compute="all", gather_on_rank0=False, profiling_interval=1,
                 node_name="n0")
    try:
        durations = [1500, 1700, 1600, 2200, 1800, 1650]
        for d in durations:
            with D.detection_section("step"):
                D.cupti_manager.push("k_blk_64_1_1_grid_4_1_1", [d])
                time.sleep(0.001)
        with D.detection_section("other", profile_cuda=False):
            pass
        rep = D.generate_report()
        ks = rep.local_kernel_summaries["k_blk_64_1_1_grid_4_1_1"]
        r = O.compute_stats(O.ns_to_us(np.array(durations, np.uint32)))
        S = straggler.Statistic
        assert ks[S.NUM] == 6 and np.float32(ks[S.MED]) == np.float32(r.median)
        assert np.float32(ks[S.AVG]) == np.float32(r.avg)  # EXACT mode profiler: bit-exact
        sec = rep.local_section_summaries["step"]
        assert sec[S.NUM] == 6 and sec[S.MIN] <= sec[S.MED] <= sec[S.MAX]
        assert rep.gpu_relative_perf_scores == {0: 1.0}
        assert rep.gpu_individual_perf_scores == {0: 1.0}
        assert rep.section_relative_perf_scores["step"][0] == pytest.approx(1.0, abs=1e-6)
        # sections and kernel records were reset by the report (straggler.py:242-243)
        rep2 = D.generate_report()
        assert len(rep2.local_kernel_summaries) == 0 and rep2.local_section_summaries == {}
    finally:
        D.shutdown()


@pytest.mark.parametrize("lengths", [(1, 2, 3, 10, 1000, 8192),
                                     # CustomSection.max_elapseds_len raised past the LDS path
                                     (5, 16385, 40000, 0, 70001)])
def test_section_stats_torch_semantics(lengths):
    import torch

    from nvidia_resiliency_ext.straggler import ops

    rng = np.random.default_rng(1)
    secs = [rng.random(n) * 10 for n in lengths]
    off = np.zeros(len(secs) + 1, np.int64)
    off[1:] = np.cumsum([len(s) for s in secs])
    num, out = ops.section_stats(torch.from_numpy(np.concatenate(secs)).cuda(),
                                 torch.from_numpy(off).cuda(), max(lengths))
    out = out.cpu().numpy()
    for i, s in enumerate(secs):
        t = torch.tensor(s, dtype=torch.float64)
        assert num[i].item() == len(s)
        if len(s) == 0:
            assert np.all(np.isnan(out[:, i]))
            continue
        assert out[0, i] == torch.min(t).item() and out[1, i] == torch.max(t).item()
        assert out[2, i] == torch.median(t).item()  # lower median, exact
        assert out[3, i] == pytest.approx(torch.mean(t).item(), rel=1e-14)
        if len(s) == 1:
            assert np.isnan(out[4, i])
        else:
            assert out[4, i] == pytest.approx(torch.std(t).item(), rel=1e-12)


def test_detector_two_ranks_flags_the_slow_rank():
    res = run_world(2, "_detector_workers", "detector_two_ranks", slow_rank=1)
    reps = res[0]
    assert len(reps) == 2 and res[1] == []
    for rep in reps:
        assert rep["rel"][0] == pytest.approx(1.0, abs=0.03)
        assert rep["rel"][1] == pytest.approx(1 / 1.3, abs=0.03)
        assert {s.rank for s in rep["strag"]["straggler_gpus_relative"]} == {1}
        assert rep["nkern"] == 6
    assert reps[0]["ind"] == {0: 1.0, 1: 1.0}
