"""configs[4] -- live capture: kernel-dispatch records (queue delivery by default,
NVRX_CAPTURE_DELIVERY selects rocprofiler-sdk tracing) from a GPT-2 small DDP training loop
feeding the on-GPU Reporter (Detector) of this package.

One process per GPU (torchrun; WORLD_SIZE=1 runs plain DDP on one GPU).  GPT-2 small
(12 layers, d=768, 12 heads, vocab 50257, ctx 1024; random init, synthetic tokens -- there is
no dataset offline), bf16 autocast, AdamW.  Every step runs inside
``Detector.detection_section("train_step")`` so each kernel dispatch of forward, backward,
all-reduce and optimizer lands in the profiler's device record log under the reference's
composite key; every ``--report-every`` steps ``Detector.generate_report()`` reduces them on
the GPU (bucketing + EXACT per-kernel statistics + scores) and gathers to rank 0.

Measured (rank 0 prints one JSON line):
  * step time without the detector, with the detector (capture on), overhead %;
  * report latency (generate_report wall time, and the report's own elapsed field);
  * records per report, distinct kernel keys, straggler sets.
``--dump PATH`` writes the last report window's raw records and statistics (npz) so that
tests/test_gpu_live.py can check them against the oracle (this tool never imports it).

Capture must be configured before the process's first HIP call, as CUPTI activity tracing
needs the first CUDA context: ``cupti.enable_capture()`` runs before torch touches the GPU.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nvidia-resiliency-ext-x_amd"))

from nvidia_resiliency_ext.straggler import cupti  # noqa: E402  (before any HIP call)

CAPTURE = cupti.enable_capture()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from nvidia_resiliency_ext import straggler  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gpt2_model import GPT2  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--base-steps", type=int, default=20, help="timed steps without the detector")
    ap.add_argument("--steps", type=int, default=60, help="timed steps with the detector")
    ap.add_argument("--report-every", type=int, default=20)
    ap.add_argument("--dump", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--profiling-interval", type=int, default=1,
                    help="Detector.initialize(profiling_interval=...): profile every k-th step")
    ap.add_argument("--profile-cuda", type=int, default=1,
                    help="0: sections time the CPU only (isolates the capture's cost)")
    ap.add_argument("--count-check", action="store_true",
                    help="no explicit flush before the reports; record each report's per-key "
                         "num_calls and those of a one-step window (capture completeness)")
    a = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    ws = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    torch.distributed.init_process_group("nccl", rank=rank, world_size=ws, device_id=dev)

    torch.manual_seed(1234 + rank)
    model = GPT2(layers=a.layers).to(dev)
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local])
    opt = torch.optim.AdamW(ddp.parameters(), lr=1e-4, fused=True)
    g = torch.Generator(device=dev)
    g.manual_seed(rank)
    tokens = torch.randint(0, 50257, (a.batch, a.seq + 1), device=dev, generator=g)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = ddp(tokens[:, :-1])
            loss = F.cross_entropy(logits.float().view(-1, logits.shape[-1]),
                                   tokens[:, 1:].reshape(-1))
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    def timed(n, fn):
        torch.cuda.synchronize()
        torch.distributed.barrier()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n

    for _ in range(a.warmup):
        step()
    t_base = timed(a.base_steps, step)

    D = straggler.Detector
    D.initialize(scores_to_compute="all", gather_on_rank0=True,
                 profiling_interval=a.profiling_interval, report_time_interval=1e9)
    prof = D.cupti_manager.cupti_ext

    def det_step():
        # no synchronize: kernels still running at the section's end are captured when they
        # complete, as CUPTI activity records are
        with D.detection_section("train_step", profile_cuda=bool(a.profile_cuda)):
            step()

    # cost of one start/stop pair of the dispatch context (no kernels in between)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        prof.start()
        prof.stop()
    t_pair = (time.perf_counter() - t0) / 200

    # one untimed window: first-sight allocations of the record log / work buffers
    for _ in range(a.report_every):
        det_step()
    D.generate_report()

    def counts(rep):
        return {k: int(v[straggler.Statistic.NUM]) for k, v in rep.local_kernel_summaries.items()}

    step_counts = None
    window_counts = []
    if a.count_check:  # a one-step window: the launches of one training step, per kernel key
        det_step()
        step_counts = counts(D.generate_report())

    reports = []
    t_flush = []
    t_flush2 = []
    det_time = 0.0
    last_report = None
    dump = None
    for w in range(max(1, a.steps // a.report_every)):
        det_time += timed(a.report_every, det_step) * a.report_every
        if w == max(1, a.steps // a.report_every) - 1 and a.dump:
            slots, ns = prof.get_records()
            names = {int(s): prof.name_of(s) for s in np.unique(slots)}
            dump = (slots, ns, names)
        if not a.count_check:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            D.cupti_manager.cupti_ext.flush_capture()
            t_flush.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            D.cupti_manager.cupti_ext.flush_capture()  # nothing left: the fixed cost of a flush
            t_flush2.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        rep = D.generate_report()  # its own synchronize + counted flush
        t_rep = time.perf_counter() - t0
        reports.append((t_rep, rep))
        window_counts.append(counts(rep))
        last_report = rep
    n_det = max(1, a.steps // a.report_every) * a.report_every
    t_det = det_time / n_det

    local_ks = last_report.local_kernel_summaries if last_report is not None else None
    if rank == 0 and dump is not None:
        slots, ns, names = dump
        S = straggler.Statistic
        ks = local_ks
        knames = list(ks.keys())
        np.savez(a.dump, slots=slots, ns=ns, slot_names=np.array([names[s] for s in sorted(names)]),
                 slot_ids=np.array(sorted(names), np.uint32), cap=np.int64(8192),
                 names=np.array(knames),
                 num=np.array([ks[n][S.NUM] for n in knames], np.int32),
                 min=np.array([ks[n][S.MIN] for n in knames], np.float32),
                 max=np.array([ks[n][S.MAX] for n in knames], np.float32),
                 med=np.array([ks[n][S.MED] for n in knames], np.float32),
                 avg=np.array([ks[n][S.AVG] for n in knames], np.float32),
                 std=np.array([ks[n][S.STD] for n in knames], np.float32))
    from nvidia_resiliency_ext.straggler import _native
    import ctypes
    cc = _native.CaptureCounters()
    _native.lib().nvrx_capture_stats(ctypes.byref(cc))
    counters = {f: getattr(cc, f) for f, _ in _native.CaptureCounters._fields_}
    D.shutdown()

    t_rep = [r[0] for r in reports]
    if rank == 0:
        rep = reports[-1][1]
        strag = rep.identify_stragglers(gpu_rel_threshold=0.8, gpu_indiv_threshold=0.8)
        nrec = sum(int(v[straggler.Statistic.NUM]) for v in (local_ks or {}).values())
        line = {
            "workload": "configs[4]: live kernel-dispatch capture, GPT-2 small DDP "
                        f"(layers={a.layers}, batch={a.batch}x{a.seq}, bf16 autocast, AdamW)",
            "capture_counters": counters,
            "n_gpus": ws, "capture": CAPTURE and cupti.capture_available(),
            "step_ms_without_detector": t_base * 1e3, "step_ms_with_detector": t_det * 1e3,
            "detector_overhead_pct": (t_det / t_base - 1) * 100,
            "report_every_steps": a.report_every, "profiling_interval": a.profiling_interval,
            "records_per_report": nrec, "kernel_keys": len(local_ks or {}),
            "report_ms": [x * 1e3 for x in t_rep],
            "report_ms_median": float(np.median(t_rep)) * 1e3,
            "capture_flush_ms_median": float(np.median(t_flush)) * 1e3 if t_flush else None,
            "empty_flush_ms_median": float(np.median(t_flush2)) * 1e3 if t_flush2 else None,
            "step_counts": step_counts, "window_counts": window_counts if a.count_check else None,
            "start_stop_pair_us": t_pair * 1e6,
            "report_elapsed_field_ms": rep.generate_report_elapsed_time,
            "gpu_relative_perf_scores": dict(rep.gpu_relative_perf_scores),
            "gpu_individual_perf_scores": dict(rep.gpu_individual_perf_scores),
            "stragglers_relative": sorted(s.rank for s in strag["straggler_gpus_relative"]),
            "stragglers_individual": sorted(s.rank for s in strag["straggler_gpus_individual"]),
            "tokens_per_s_with_detector": ws * a.batch * a.seq / t_det,
        }
        print(json.dumps(line))
        if a.out:
            with open(a.out, "w") as f:
                json.dump(line, f, indent=1)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
