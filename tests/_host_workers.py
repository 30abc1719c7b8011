"""Rank bodies for tests/test_host_logic.py (CPU, gloo): name-id agreement, the interval
MAX-reduce and the dist_utils collectives, with no device involved."""


def name_mapper_world(rank, ws):
    from nvidia_resiliency_ext.straggler.name_mapper import NameMapper

    nm = NameMapper()
    # round 1: each rank has one private kernel + one shared kernel and a shared section
    nm.gather_and_assign_ids([f"k_rank{rank}", "shared"], ["sec"])
    r1 = (dict(nm.kernel_name_to_id), dict(nm.section_name_to_id))
    # round 2: nothing new anywhere -> ids unchanged
    nm.gather_and_assign_ids(["shared"], ["sec"])
    r2 = dict(nm.kernel_name_to_id)
    # round 3: only the last rank sees new names -> everyone assigns them, same ids
    new = ["late_b", "late_a"] if rank == ws - 1 else []
    nm.gather_and_assign_ids(new, ["sec2"] if rank == 0 else [])
    r3 = (dict(nm.kernel_name_to_id), dict(nm.section_name_to_id))
    return {"r1": r1, "r2": r2, "r3": r3}


def interval_world(rank, ws, step_s):
    import time

    from nvidia_resiliency_ext.straggler.interval_tracker import ReportIntervalTracker

    tr = ReportIntervalTracker(time_interval=0.4, profiling_interval=1)
    for _ in range(tr.INTERVAL_ESTIMATION_ITERS + 1):
        tr.iter_increase()
        time.sleep(step_s[rank])
    return tr.iter_interval


def dist_utils_world(rank, ws):
    import torch

    from nvidia_resiliency_ext.straggler import dist_utils as du

    out = {"ws": du.get_world_size(), "rank": du.get_rank(),
           "dev": str(du.get_device_for_backend()),
           "all_true": du.is_all_true(True), "one_false": du.is_all_true(rank != 1)}
    g = du.gather_on_rank0(torch.tensor([float(rank), 10.0 * rank]))
    out["gather"] = None if g is None else [t.tolist() for t in g]
    out["objs"] = du.all_gather_object({"r": rank})
    t = torch.tensor([float(rank + 1)])
    du.all_reduce(t)
    out["sum"] = t.item()
    return out
