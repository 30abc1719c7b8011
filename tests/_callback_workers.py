"""Rank bodies for tests/test_ptl_callback.py (CPU, gloo): the callback's stop decision is
made on rank 0 and broadcast (straggler_det_callback.py:213-242).  The Detector's report
calls are replaced by fakes so that only the callback's control flow runs."""


class _Trainer:
    should_stop = False
    checkpoint_callback = None

    def __init__(self, rank):
        self.global_rank = rank


def stop_flag_world(rank, ws, rel_score=0.5, stop_if_detected=True):
    from nvidia_resiliency_ext import straggler
    from nvidia_resiliency_ext.ptl_resiliency import StragglerDetectionCallback

    rep = straggler.Report(
        gpu_relative_perf_scores={r: (rel_score if r == 1 else 1.0) for r in range(ws)},
        section_relative_perf_scores={}, gpu_individual_perf_scores={},
        section_individual_perf_scores={}, rank_to_node={r: "n" for r in range(ws)},
        local_section_summaries={}, local_kernel_summaries={}, generate_report_elapsed_time=0.0,
        gather_on_rank0=True, rank=rank)
    calls = {"reports": 0}

    def fake_generate():
        calls["reports"] += 1
        return rep if rank == 0 else None  # gather_on_rank0: only rank 0 holds the report

    D = straggler.Detector
    saved = (D.__dict__["generate_report_if_interval_elapsed"], D.__dict__["is_interval_elapsed"])
    D.generate_report_if_interval_elapsed = staticmethod(fake_generate)
    D.is_interval_elapsed = staticmethod(lambda: True)
    try:
        cb = StragglerDetectionCallback(
            report_time_interval=1.0, calc_relative_gpu_perf=True, calc_individual_gpu_perf=False,
            num_gpu_perf_scores_to_print=0, gpu_relative_perf_threshold=0.8,
            gpu_individual_perf_threshold=0.8, stop_if_detected=stop_if_detected,
            enable_ptl_logging=False)
        tr = _Trainer(rank)
        cb.on_train_batch_end(tr, None, None, None, 0)
    finally:
        D.generate_report_if_interval_elapsed, D.is_interval_elapsed = saved
    return {"should_stop": tr.should_stop, "reports": calls["reports"]}
