"""Probe (not part of the library): where Detector.generate_report's time goes on a live capture
-- GPT-2-sized kernel mix replaced by a synthetic loop of NK distinct kernels x REPS launches per
window (torch ops of distinct shapes), then the report's phases timed one by one."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))
from nvidia_resiliency_ext.straggler import cupti  # noqa: E402

cupti.enable_capture()
import torch  # noqa: E402

from nvidia_resiliency_ext import straggler  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29777")
torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
D = straggler.Detector
D.initialize(scores_to_compute="all", gather_on_rank0=True, report_time_interval=1e9)
xs = [torch.randn(64 + 8 * i, 256, device="cuda") for i in range(40)]
w = torch.randn(256, 256, device="cuda")


def window(reps):
    for _ in range(reps):
        with D.detection_section("step"):
            for x in xs:
                y = torch.relu(x @ w)
                y.sum()


res = {}
for reps in (8, 32, 128):
    window(reps)
    D.generate_report()  # first-sight allocations
    t = {}
    for it in range(5):
        window(reps)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sec = D._get_section_summaries()
        t1 = time.perf_counter()
        ks = D._get_kernel_summaries()
        t2 = time.perf_counter()
        rep = D.reporter.generate_report(sec, ks)
        t3 = time.perf_counter()
        D._reset_sections_elapseds()
        D.cupti_manager.reset_results()
        t4 = time.perf_counter()
        for k, v in (("sections", t1 - t0), ("kernel_stats", t2 - t1), ("report_generator", t3 - t2),
                     ("reset", t4 - t3)):
            t.setdefault(k, []).append(v * 1e3)
    nrec = sum(int(v[straggler.Statistic.NUM]) for v in ks.values())
    res[reps] = {"records": nrec, "keys": len(ks), **{k: sorted(v)[2] for k, v in t.items()}}
    print(reps, res[reps], flush=True)
print("RESULT " + json.dumps(res))
D.shutdown()
torch.distributed.destroy_process_group()
