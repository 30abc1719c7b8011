"""Functional straggler run in the shape of the reference's tests/straggler/func/ddp_test.py
(:172-245): a DDP model whose forward is wrapped by Detector.wrap_callables, periodic reports,
and the report / straggler-set lines printed in the reference's format (:126-158) so that a log
checker (check_log.py:29-51; tests/test_gpu_functional_ddp.py) can assert the detected set.

Models: a small MLP (--model mlp, the reference's ddp_test shape) or GPT-2 small (--model gpt2:
12 layers, d=768, ctx 1024, bf16 autocast, AdamW; tools/gpt2_model.py) -- the configs[4] model,
hundreds of distinct kernel keys (GEMMs, attention, layer norms, the fused optimizer).

Slowness is injected, as the test environment has one GPU for all ranks: every forward ends
with a spin kernel (torch.cuda._sleep: same launch shape on every rank, so the same composite
kernel key) that runs --slow-factor times longer on the ranks in --slow-ranks.  --spin-ratio r
sizes the fast ranks' spin to r x the forward's kernel time per step as the detector weighs it
(sum of NUM x AVG over the captured forward kernels, the largest over ranks), so
that the spin carries a known share of the NUM*AVG weights whatever the model: with forward
time F and spin rF, a rank slowed s-fold scores (F + rF) / (F + s rF) (reporting.py:219-253),
0.69 at r = 10, s = 1.5.  Launched with torch.distributed.run; gloo process group, all ranks on
GPU LOCAL_RANK % device_count.  Prints the step time without and with the detector."""
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
    p.add_argument("--model", choices=("mlp", "gpt2"), default="mlp")
    p.add_argument("--seq", type=int, default=1024, help="gpt2: tokens per sample")
    p.add_argument("--spin-ratio", type=float, default=0.0,
                   help="> 0: spin = this x the forward's GPU time (overrides --spin-cycles)")
    p.add_argument("--base-iters", type=int, default=0,
                   help="timed steps before the detector is initialised (step overhead)")
    return p.parse_args()


class Model(nn.Module):
    def __init__(self, body, spin):
        super().__init__()
        self.body = body
        self.spin = spin

    def forward(self, x):
        y = self.body(x)
        if self.spin > 0:
            torch.cuda._sleep(self.spin)  # the injected GPU work (longer on slow ranks)
        return y


def gpu_ms(fn, n=5):
    """Mean GPU time of fn() between two events (fn's kernels run back to back on one stream)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


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
    if os.environ.get("NVRX_FUNC_WATCHDOG_S"):  # diagnostics: every thread's stack, then exit
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["NVRX_FUNC_WATCHDOG_S"]), exit=True)
    torch.distributed.init_process_group("gloo")
    rank = torch.distributed.get_rank()
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    os.environ["LOCAL_RANK"] = str(local)  # ranks share the box's GPU(s): get_current_device()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    slow = {int(r) for r in args.slow_ranks.split(",") if r}
    factor = args.slow_factor if rank in slow else 1.0
    torch.manual_seed(0)
    if args.model == "gpt2":
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from gpt2_model import GPT2

        body = GPT2().to(dev)
        data = torch.randint(0, 50257, (args.batch, args.seq + 1), device=dev,
                             generator=torch.Generator(device=dev).manual_seed(rank))

        def batch_fn():
            return data[:, :-1], data[:, 1:]

        def loss_fn(out, tgt):
            return nn.functional.cross_entropy(out.float().view(-1, out.shape[-1]), tgt.reshape(-1))
    else:
        body = nn.Sequential(*[nn.Linear(args.hidden, args.hidden, bias=False) for _ in range(args.layers)]).to(dev)
        mse = nn.MSELoss()

        def batch_fn():
            return (torch.rand(args.batch, args.hidden, device=dev),
                    torch.rand(args.batch, args.hidden, device=dev))

        def loss_fn(out, tgt):
            return mse(out, tgt)
    model_ = Model(body, 0)
    model = nn.parallel.DistributedDataParallel(model_)
    opt = (torch.optim.AdamW(model.parameters(), lr=1e-4, fused=True) if args.model == "gpt2"
           else torch.optim.SGD(model.parameters(), lr=1e-4))

    def fwd(x):
        if args.model == "gpt2":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return model(x)
        return model(x)

    def step(prof=None):
        x, tgt = batch_fn()
        if prof is not None:
            prof.start()
        out = fwd(x)
        if prof is not None:
            prof.stop()
        opt.zero_grad()
        if args.model == "gpt2":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = loss_fn(out, tgt)
        else:
            loss = loss_fn(out, tgt)
        loss.backward()
        opt.step()

    base = args.spin_cycles
    for _ in range(2):
        step()
    if args.spin_ratio > 0:
        # the forward's kernel time per step as the detector weighs it -- sum of NUM x MED of the
        # forward's captured kernels (reporting.py:248 weighs NUM x AVG) over 5 training steps, on a profiler
        # handle of its own (closed before the Detector creates its singleton); the ranks share
        # one GPU, so their kernels' durations include the other rank's concurrent work.  The
        # largest over ranks sizes one base spin for every rank; the spin's clock rate measured.
        prof = cupti.KernelProfiler(statsMaxLenPerKernel=8192)
        prof.initialize()
        for _ in range(3):  # first windows of a fresh capture: not weighed
            step(prof)
        torch.cuda.synchronize()
        prof.reset()
        for _ in range(5):
            step(prof)
        torch.cuda.synchronize()
        st = prof.get_stats()
        # NUM x MED: a kernel whose duration spikes once does not size the spin
        f_ms = sum(v.num_calls * v.median for v in st.values()) / 5 / 1e3
        if rank == 0:
            top = sorted(st.items(), key=lambda kv: -kv[1].num_calls * kv[1].avg)[:3]
            print("CALIB kernels=%d sum_num_avg_ms=%.3f sum_num_med_ms=%.3f top=%s" % (
                len(st), sum(v.num_calls * v.avg for v in st.values()) / 5 / 1e3, f_ms,
                [(k[:40], v.num_calls, round(v.avg, 1), round(v.median, 1)) for k, v in top]))
        prof.shutdown()
        prof.close()
        per_ms = 1e6 / gpu_ms(lambda: torch.cuda._sleep(1_000_000), n=3)
        t = torch.tensor([f_ms], dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        base = int(args.spin_ratio * min(float(t.item()), 50.0) * per_ms)  # at most 300 ms
        if rank == 0:
            print(f"SPIN forward_kernel_ms={float(t.item()):.3f} spin_cycles={base} "
                  f"cycles_per_ms={per_ms:.0f}")
    model_.spin = int(base * factor)
    step()
    step_ms_base = None
    if args.base_iters > 0:
        torch.cuda.synchronize()
        torch.distributed.barrier()
        t0 = time.perf_counter()
        for _ in range(args.base_iters):
            step()
        torch.cuda.synchronize()
        step_ms_base = (time.perf_counter() - t0) / args.base_iters * 1e3

    straggler.Detector.initialize(scores_to_compute=["relative_perf_scores", "individual_perf_scores"],
                                  gather_on_rank0=True)
    straggler.Detector.wrap_callables(callable_ids=[straggler.CallableId(model, "forward")])
    idx, t_steps, n_steps = 1, 0.0, 0
    torch.cuda.synchronize()
    torch.distributed.barrier()
    t0 = time.perf_counter()
    for i in range(args.iters):
        step()
        if i > 0 and i % args.report_iter_interval == 0:
            torch.cuda.synchronize()
            if idx > 1:  # step time between reports (the first window holds first-sight setup)
                t_steps += time.perf_counter() - t0
                n_steps += args.report_iter_interval
            report = straggler.Detector.generate_report()
            if report:  # rank 0 (gather_on_rank0)
                print_report(report, rank, idx)
                print_stragglers(report.identify_stragglers(gpu_rel_threshold=args.threshold,
                                                            gpu_indiv_threshold=args.threshold))
            idx += 1
            t0 = time.perf_counter()
    if rank == 0 and step_ms_base is not None and n_steps:
        with_det = t_steps / n_steps * 1e3
        print(f"STEP MS without_detector={step_ms_base:.3f} with_detector={with_det:.3f} "
              f"overhead_pct={(with_det / step_ms_base - 1) * 100:.2f}")
    torch.cuda.synchronize()
    straggler.Detector.shutdown()
    torch.distributed.barrier()
    if rank == 0:
        print("DONE")
    torch.distributed.destroy_process_group()
    sys.stdout.flush()


if __name__ == "__main__":
    main()
