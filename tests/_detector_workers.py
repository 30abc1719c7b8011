"""Rank workers for the Detector end-to-end tests."""
import time

import numpy as np


def detector_two_ranks(rank, ws, slow_rank):
    from nvidia_resiliency_ext import straggler

    D = straggler.Detector
    D.initialize(scores_to_compute="all", gather_on_rank0=True, node_name=f"node{rank}")
    try:
        rng = np.random.default_rng(100 + rank)
        scale = 1.3 if rank == slow_rank else 1.0
        reports = []
        for it in range(2):
            for step in range(20):
                with D.detection_section("fwd"):
                    time.sleep(0.002 * scale)
                    for k in range(6):  # kernel executions of this step, as a tracer would feed them
                        base = 10_000 * (k + 1)
                        D.cupti_manager.push(f"kernel{k}_blk_256_1_1_grid_{k + 1}_1_1",
                                             [int(base * scale * (1 + 0.05 * rng.random()))])
            rep = D.generate_report()
            if rep is not None:
                reports.append(dict(
                    rel=dict(rep.gpu_relative_perf_scores), ind=dict(rep.gpu_individual_perf_scores),
                    sec_rel={k: dict(v) for k, v in rep.section_relative_perf_scores.items()},
                    strag=rep.identify_stragglers(gpu_rel_threshold=0.85,
                                                  section_rel_threshold=0.85),
                    nkern=len(rep.local_kernel_summaries),
                    kern=dict(rep.local_kernel_summaries["kernel0_blk_256_1_1_grid_1_1_1"])))
        return reports
    finally:
        D.shutdown()
