"""Functional straggler run in the shape of the reference's tests/straggler/func/ddp_test.py
(:172-245): a DDP model whose forward is wrapped by Detector.wrap_callables, periodic reports,
and the report / straggler-set lines printed in the reference's format (:126-158) so that a log
checker (check_log.py:29-51; tests/test_gpu_functional_ddp.py) can assert the detected set.

Slowness is injected, as the test environment has one GPU for all ranks: every forward ends
with a spin kernel (torch.cuda._sleep: same launch shape on every rank, so the same composite
kernel key) that runs --slow-factor times longer on the ranks in --slow-ranks.  Launched with
torch.distributed.run; gloo process group, all ranks on GPU LOCAL_RANK % device_count."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))

from nvidia_resiliency_ext.straggler import cupti  # noqa: E402

cupti.enable_capture()  # rocprofiler-sdk: before this process's first HIP call

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from nvidia_resiliency_ext import straggler  # noqa: E402


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--layers", type=int, default=4)
    p.add_argument("--batch", type=int, default=16)
    p.add_argument("--hidden", type=int, default=256)
    p.add_argument("--iters", type=int, default=60)
    p.add_argument("--report-iter-interval", type=int, default=20)
    p.add_argument("--spin-cycles", type=int, default=2_000_000)
    p.add_argument("--slow-factor", type=float, default=1.5)
    p.add_argument("--slow-ranks", type=str, default="1")
    p.add_argument("--threshold", type=float, default=0.75)
    return p.parse_args()


class Model(nn.Module):
    def __init__(self, hidden, layers, spin):
        super().__init__()
        self.body = nn.Sequential(*[nn.Linear(hidden, hidden, bias=False) for _ in range(layers)])
        self.spin = spin

    def forward(self, x):
        y = self.body(x)
        torch.cuda._sleep(self.spin)  # the injected GPU work (longer on slow ranks)
        return y


def r2(d):
    return {k: round(v, 2) for k, v in d.items()}


def print_report(report, rank, idx):
    # ddp_test.py:126-158
    print(f"STRAGGLER REPORT #{idx}")
    print(f"=== GPUs perf scores. Report from rank {rank} ===")
    print("GPU relative perf scores:", r2(report.gpu_relative_perf_scores))
    print("GPU individual perf scores:", r2(report.gpu_individual_perf_scores))
    print(f"=== Sections perf scores. Report from rank {rank} ===")
    print("Sections relative perf scores:",
          {s: r2(v) for s, v in report.section_relative_perf_scores.items()})
    print("Sections individual perf scores:",
          {s: r2(v) for s, v in report.section_individual_perf_scores.items()})


def print_stragglers(st):
    for s in st["straggler_gpus_relative"]:
        print(f"DETECTED RELATIVE STRAGGLER GPU RANK={s.rank} NODE={s.node}")
    for s in st["straggler_gpus_individual"]:
        print(f"DETECTED INDIVIDUAL STRAGGLER GPU RANK={s.rank} NODE={s.node}")
    for sec, ids in st["straggler_sections_relative"].items():
        for s in ids:
            print(f"DETECTED RELATIVE STRAGGLER SECTION={sec} RANK={s.rank} NODE={s.node}")
    for sec, ids in st["straggler_sections_individual"].items():
        for s in ids:
            print(f"DETECTED INDIVIDUAL STRAGGLER SECTION={sec} RANK={s.rank} NODE={s.node}")


def main():
    args = parse_args()
    torch.distributed.init_process_group("gloo")
    rank = torch.distributed.get_rank()
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    os.environ["LOCAL_RANK"] = str(local)  # ranks share the box's GPU(s): get_current_device()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    slow = {int(r) for r in args.slow_ranks.split(",") if r}
    spin = int(args.spin_cycles * (args.slow_factor if rank in slow else 1.0))
    torch.manual_seed(0)
    model = nn.parallel.DistributedDataParallel(Model(args.hidden, args.layers, spin).to(dev))
    opt = torch.optim.SGD(model.parameters(), lr=1e-4)
    loss_fn = nn.MSELoss()

    straggler.Detector.initialize(scores_to_compute=["relative_perf_scores", "individual_perf_scores"],
                                  gather_on_rank0=True)
    straggler.Detector.wrap_callables(callable_ids=[straggler.CallableId(model, "forward")])
    idx = 1
    for i in range(args.iters):
        data = torch.rand(args.batch, args.hidden, device=dev)
        target = torch.rand(args.batch, args.hidden, device=dev)
        out = model(data)
        opt.zero_grad()
        loss_fn(out, target).backward()
        opt.step()
        if i > 0 and i % args.report_iter_interval == 0:
            report = straggler.Detector.generate_report()
            if report:  # rank 0 (gather_on_rank0)
                print_report(report, rank, idx)
                print_stragglers(report.identify_stragglers(gpu_rel_threshold=args.threshold,
                                                            gpu_indiv_threshold=args.threshold))
                idx += 1
    torch.cuda.synchronize()
    straggler.Detector.shutdown()
    torch.distributed.barrier()
    if rank == 0:
        print("DONE")
    torch.distributed.destroy_process_group()
    sys.stdout.flush()


if __name__ == "__main__":
    t0 = time.time()
    main()
