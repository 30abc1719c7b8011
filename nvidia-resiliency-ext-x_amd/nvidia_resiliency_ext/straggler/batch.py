"""Batched scoring of many (simulated) ranks resident in HBM -- the hot path at scale.

``MatrixReporter`` runs the whole report for R ranks x K kernels in one pass over a
u32 duration-key matrix ``[R][K][S_push]`` (``_native.duration_keys``: the integer ns below
3.76 s; raw u32 ns reaching 3.76 s must go through ``ops.encode_ns_u32_`` first) (the last ``cap`` samples of every (rank, kernel)
retained, as the reference's per-kernel rings keep them), or over R push-ordered record
streams ``{slot, ns}`` (``compute_stats_records``: bucket by slot keeping the last ``cap``
of each, then length-classed segment statistics -- configs[3]):

  segment_stats (HIP) -> per-kernel reference = min over ranks (HIP)
  -> per-rank weighted relative / individual partial sums (HIP)
  -> [multi-GPU: one RCCL all_gather of the partials]
  -> scores + straggler masks (HIP) -> host.

It is the same arithmetic the reference ReportGenerator performs once per rank
(reporting.py:421-554) on the stats computeStats produced (CuptiProfiler.cpp:44-74),
batched over ranks.  Multi-GPU: the kernel columns are sharded by hash(kernel name) %
world size; every GPU holds all R ranks for its kernels, so the per-kernel reference
and the history are shard-local and the only exchange is the [R][6] f64 partials.
"""
from __future__ import annotations

import os
import time
import weakref
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import ops


# The per-kernel reference (min over ranks of MED) is fused into the stats epilogue as one
# global atomicMin per segment.  Those atomics serialise per column: with R rows every
# column address takes R of them, which costs more than a separate column reduction
# (kernel_ref: 64 rows per thread, R/64 atomics per column) once R is in the hundreds
# (measured on MI355X: 885k segments on 54 columns, 0.6 ms -> 4.3 ms fused).
FUSED_REF_MAX_ROWS = 256


# How the host waits for a report's results (they land in pinned host memory):
#   "bounded" (default) -- poll the completion event for at most SPIN_BOUND_US, then block in
#       hipEventSynchronize on a blocking-sync event: a report that lands within the bound
#       skips the driver's wake-up latency, a longer one does not hold a host core (in a
#       training process that calls this API every core belongs to the job; the reference's
#       report path blocks too, straggler.py:234-235, CuptiProfiler.cpp:136-146);
#   "spin" -- poll until done (bench.py: the wake-up latency is part of every timed report);
#   "block" -- block at once.
# NVRX_SYNC selects the mode per process; set_sync_mode() changes it at run time.
SYNC_MODES = ("bounded", "spin", "block")
SPIN_BOUND_US = float(os.environ.get("NVRX_SPIN_US", "50"))
_sync_mode = os.environ.get("NVRX_SYNC", "") or "bounded"
if _sync_mode not in SYNC_MODES:
    raise ValueError(f"NVRX_SYNC={_sync_mode!r}: one of {SYNC_MODES}")


def set_sync_mode(mode: str) -> str:
    """Select how report results are waited for (SYNC_MODES); returns the previous mode."""
    global _sync_mode
    if mode not in SYNC_MODES:
        raise ValueError(f"sync mode {mode!r}: one of {SYNC_MODES}")
    prev, _sync_mode = _sync_mode, mode
    return prev


def sync_mode() -> str:
    return _sync_mode


def wait_event(ev, mode: Optional[str] = None, bound_us: Optional[float] = None) -> None:
    """Wait until a recorded event has completed, in the current (or the given) sync mode.
    `ev` needs query() and synchronize(); the blocking fallback blocks only if the event was
    created with blocking=True (every event this module waits on is)."""
    mode = mode or _sync_mode
    if mode == "block":
        ev.synchronize()
        return
    if mode == "spin":
        while not ev.query():
            pass
        return
    bound = SPIN_BOUND_US if bound_us is None else bound_us
    deadline = time.perf_counter_ns() + int(bound * 1e3)
    while not ev.query():
        if time.perf_counter_ns() >= deadline:
            ev.synchronize()
            return


def _wait(device) -> None:
    """Wait for the device's current stream (wait_event on an event recorded on it)."""
    ev = torch.cuda.Event(blocking=True)
    ev.record(torch.cuda.current_stream(device))
    wait_event(ev)


@dataclass
class BatchResult:
    gpu_relative: Optional[np.ndarray]     # [R] f64 (NaN: no common kernel)
    gpu_individual: Optional[np.ndarray]   # [R] f64
    stragglers_relative: Optional[np.ndarray]   # [R] bool, score < thr_rel
    stragglers_individual: Optional[np.ndarray]  # [R] bool, score < thr_ind
    err: int = 0


class MatrixReporter:
    def __init__(self, R: int, K: int, *, cap: int = 8192, relative: bool = True,
                 individual: bool = True, thr_rel: float = 0.75, thr_ind: float = 0.75,
                 col_valid: Optional[torch.Tensor] = None, mode: int = ops.STATS_FAST,
                 round_f32: bool = False, group=None, device=None, exchange: Optional[bool] = None):
        self.R, self.K, self.cap = R, K, cap
        self.relative, self.individual = relative, individual
        self.thr_rel, self.thr_ind = thr_rel, thr_ind
        self.mode, self.round_f32 = mode, round_f32
        self.group = group
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        d = self.device
        self.world = 1
        self.gloo = False
        if group is not None or (torch.distributed.is_available() and torch.distributed.is_initialized()):
            self.world = torch.distributed.get_world_size(group)
            self.gloo = torch.distributed.get_backend(group) == torch.distributed.Backend.GLOO
        # exchange: the multi-GPU scoring (partials -> all_gather -> finalize) even in a world
        # of one -- how a one-GPU box runs the RCCL branch (tests); default: world > 1
        self.exchange = self.world > 1 if exchange is None else bool(exchange)
        if self.exchange and not (torch.distributed.is_available() and torch.distributed.is_initialized()):
            raise RuntimeError("MatrixReporter(exchange=True) needs an initialized process group")
        self.stats = ops.SegmentStats.empty(R * K, d)
        self.col_valid = col_valid
        # per-kernel reference, produced by the stats kernel's epilogue: [min bits | missing]
        self.col_ref = torch.empty(2 * max(K, 1), dtype=torch.int32, device=d)
        self._ref_f32 = torch.empty(max(K, 1), dtype=torch.float32, device=d)
        self.hist = torch.full((R, K), float("inf"), dtype=torch.float32, device=d) if individual else None
        self.partials = torch.empty((R, 6), dtype=torch.float64, device=d)
        self.gathered = (torch.empty((self.world, R, 6), dtype=torch.float64, device=d)
                         if self.exchange else None)
        # one packed result buffer -> one device-to-host copy per report:
        # [gpu_rel f64 R][gpu_ind f64 R][strag_rel u8 R][strag_ind u8 R][pad][err i32]
        self._e = (18 * R + 7) // 8 * 8
        nbytes = self._e + 8
        self.out = torch.zeros(nbytes, dtype=torch.uint8, device=d)
        self.h_out = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.views = dict(gpu_rel=self.out[0:8 * R].view(torch.float64),
                          gpu_ind=self.out[8 * R:16 * R].view(torch.float64),
                          strag_rel=self.out[16 * R:17 * R], strag_ind=self.out[17 * R:18 * R])
        self.err = self.out[self._e:self._e + 4].view(torch.int32)
        # self-resetting scores epilogue (nvrx_score_args.done): the scores kernel's last
        # workgroup stores the error bits and re-initialises col_ref for the next report, so a
        # report is two launches (statistics, scores) with no initialising fill in between
        self.done = torch.zeros(2, dtype=torch.int32, device=d)
        self._colref_clean = False  # col_ref holds the initial reference (set by the epilogue)
        self._pipes = weakref.WeakSet()  # PipelinedReports over this reporter

    def _order_after_inflight(self, exclude=None) -> None:
        """The caller's stream waits for every pipelined report still in flight on this reporter.
        Those reports run on private streams and use slot 0's buffers (the reporter's own
        statistics, reference and results) and the shared history, so an eager report, a graph
        replay or a history reset issued between submit() and collect() queues behind them
        instead of racing them.  A no-op while a graph is being captured (the captures pair
        their phases themselves) and with nothing in flight."""
        if not self._pipes or torch.cuda.is_current_stream_capturing():
            return
        cur = torch.cuda.current_stream(self.device)
        for p in list(self._pipes):
            if p is not exclude:
                for k, _ in p.pending:
                    cur.wait_event(p.done[k])

    def reset_history(self):
        if self.hist is not None:
            self._order_after_inflight()
            self.hist.fill_(float("inf"))

    # -- device phases, separately callable (bench times the stats kernel) --
    def _fuse_ref(self) -> bool:
        return self.relative and self.R <= FUSED_REF_MAX_ROWS

    def _column_ref(self):
        """Per-kernel reference by a separate column reduction into the col_ref layout."""
        if self.relative and not self._fuse_ref():
            st = self.stats.view(self.R, self.K)
            ops.kernel_ref(st.num, st.med, ref=self._ref_f32, scratch=self.col_ref)

    def compute_stats(self, ns: torch.Tensor, s_push: int) -> ops.SegmentStats:
        # (inside a graph capture the flag describes the device state when the graph replays:
        # the captured sequences always pair a statistics call with the scores that follow)
        self._order_after_inflight()
        st = ops.segment_stats_strided(ns.view(-1), self.R * self.K, s_push, 0, s_push,
                                       cap=self.cap, mode=self.mode, out=self.stats,
                                       col_ref=self.col_ref if self._fuse_ref() else None,
                                       ncols=self.K, colref_ready=self._colref_clean)
        self._colref_clean = False
        self._column_ref()
        return st

    def compute_stats_records(self, recs: torch.Tensor, rec_off: torch.Tensor) -> ops.SegmentStats:
        """recs [n, 2] int32 {slot, ns} of R streams (rec_off [R+1] int64, device): the
        reference's ring pushes (CuptiProfiler.cpp:168-203) + getStats, for every rank."""
        self._order_after_inflight()
        n = recs.shape[0]
        need = ops.records_bucket_capacity(n, self.R, self.K)
        b = getattr(self, "_bucket", None)
        if b is None or b[2].numel() < need:
            d = self.device
            # (no per-bucket push counts: a report needs the kept records only)
            b = (torch.empty(self.R * self.K, dtype=torch.int64, device=d),
                 torch.empty(self.R * self.K, dtype=torch.int32, device=d),
                 torch.empty(max(need, 1), dtype=torch.int32, device=d), None)
            self._bucket = b
        max_len = min(self.cap, n) if self.cap > 0 else n
        self._colref_clean = False
        return ops.records_stats(recs, rec_off, self.K, self.cap, max(max_len, 1), mode=self.mode,
                                 out=self.stats, bucket=b,
                                 col_ref=self.col_ref if self.relative else None)

    def report_records(self, recs: torch.Tensor, rec_off: torch.Tensor) -> BatchResult:
        """One full report from record streams resident in HBM."""
        self.compute_stats_records(recs, rec_off)
        self.compute_scores()
        return self.land()

    def _outputs(self, buf: Optional[torch.Tensor] = None):
        R = self.R
        b = self.out if buf is None else buf
        return dict(gpu_rel=b[0:8 * R].view(torch.float64) if self.relative else None,
                    gpu_ind=b[8 * R:16 * R].view(torch.float64) if self.individual else None,
                    strag_rel=b[16 * R:17 * R] if self.relative else None,
                    strag_ind=b[17 * R:18 * R] if self.individual else None,
                    thr_rel=self.thr_rel, thr_ind=self.thr_ind, round_f32=self.round_f32)

    def compute_scores(self, out_buf: Optional[torch.Tensor] = None) -> None:
        """Scores + straggler masks into the packed buffer (one kernel on 1 GPU; partials ->
        RCCL all_gather -> finalize on N GPUs).  out_buf: another packed buffer of the same
        layout (1 GPU), e.g. pinned host memory the kernel writes directly (no copy)."""
        R, K = self.R, self.K
        self._order_after_inflight()
        st = self.stats.view(R, K)
        ref = self.col_ref.view(torch.float32)[:K] if self.relative else None
        missing = self.col_ref[K:2 * K] if self.relative else None
        # the self-resetting epilogue where the per-kernel reference is fused into the
        # statistics (R <= FUSED_REF_MAX_ROWS): one completion counter per report, whose
        # same-address atomics would cost ~0.15 / 1 ms at 4,096 / 16,384 rows
        fused = self._fuse_ref()
        reset = self.col_ref[:2 * K] if fused else None
        done = self.done if fused else None
        if not self.exchange:
            b = self.out if out_buf is None else out_buf
            err = b[self._e:self._e + 4].view(torch.int32)
            if not fused:
                err.zero_()
            ops.scores(st.num, st.med, st.avg, col_valid=self.col_valid, ref=ref,
                       ref_missing=missing, hist=self.hist, err=err,
                       finalize=self._outputs(b), done=done, reset_col_ref=reset)
            self._colref_clean = fused
            return
        self._scores_partials()
        self._exchange()
        self._finalize()

    # -- the N-GPU scoring in three phases: per-rank partials of this shard's kernels (HIP), the
    # all_gather of the partials (RCCL / gloo), the combine in shard order (HIP) --
    def _scores_partials(self) -> None:
        R, K = self.R, self.K
        st = self.stats.view(R, K)
        ref = self.col_ref.view(torch.float32)[:K] if self.relative else None
        missing = self.col_ref[K:2 * K] if self.relative else None
        fused = self._fuse_ref()
        if not fused:
            self.err.zero_()
        ops.scores(st.num, st.med, st.avg, col_valid=self.col_valid, ref=ref,
                   ref_missing=missing, hist=self.hist, partials=self.partials, err=self.err,
                   done=self.done if fused else None,
                   reset_col_ref=self.col_ref[:2 * K] if fused else None)
        self._colref_clean = fused

    def _exchange(self) -> None:
        R = self.R
        flat = self.gathered.view(self.world * R, 6)
        if self.gloo:  # gloo collectives take host tensors
            hg = torch.empty((self.world * R, 6), dtype=torch.float64)
            torch.distributed.all_gather_into_tensor(hg, self.partials.cpu(), group=self.group)
            flat.copy_(hg)
        else:          # RCCL over xGMI, device to device
            torch.distributed.all_gather_into_tensor(flat, self.partials, group=self.group)

    def _finalize(self) -> None:
        R = self.R
        o = self._outputs()
        ops.finalize_scores(self.gathered, R, self.world, self.round_f32, self.thr_rel,
                            self.thr_ind, rel=self.relative, ind=self.individual, err=self.err,
                            out={k: o[k] for k in ("gpu_rel", "gpu_ind", "strag_rel", "strag_ind")})

    def land(self) -> BatchResult:
        """The one device-to-host copy of the packed results, then host views."""
        self.h_out.copy_(self.out, non_blocking=True)
        _wait(self.device)
        return self._unpack()

    def report(self, ns: torch.Tensor, s_push: int) -> BatchResult:
        """One full report: samples resident in HBM -> scores + straggler sets on host."""
        self.compute_stats(ns, s_push)
        self.compute_scores()
        return self.land()

    def graph(self, ns: torch.Tensor, s_push: int) -> "ReportGraph":
        """The report's device work captured once as HIP graphs, replayed per report (the
        launch sequence -- reference init, stats, scores, result copy -- costs one graph
        launch instead of one host launch per operation).  1 GPU, or the stats phase only
        on N GPUs (the partials exchange stays an eager collective)."""
        return ReportGraph(self, ns, s_push)

    def graph_records(self, recs: torch.Tensor, rec_off: torch.Tensor) -> "ReportGraph":
        """graph() over record streams resident in HBM (compute_stats_records captured)."""
        return ReportGraph(self, None, 0, stats=lambda: self.compute_stats_records(recs, rec_off))

    def pipelined(self, ns, s_push: int, timing: bool = False,
                  mode: Optional[str] = None, depth: int = 2,
                  timing_reps: int = 1) -> "PipelinedReports":
        """Reports replayed two deep: report i+1's device work is queued before report i's
        results are read on the host, each report landing in its own pinned buffer (N GPUs: the
        partials exchange of each report stays an eager collective, issued in report order).
        ns: one input matrix, or a list of them (report i reads ns[i % len(ns)]; len(ns) divides
        depth) -- e.g. a fresh matrix per report in flight.  An input must not be modified while
        a report that reads it is in flight: collect() raises if a torch in-place operation
        changed it (its version counter moved) between that report's submit() and collect()."""
        ins = list(ns) if isinstance(ns, (list, tuple)) else [ns]
        return PipelinedReports(self, None, s_push, timing, mode=mode, depth=depth,
                                timing_reps=timing_reps,
                                stats=[lambda x=x: self.compute_stats(x, s_push) for x in ins],
                                stats_bytes=self._matrix_bytes(s_push), inputs=[(x,) for x in ins])

    def _matrix_bytes(self, s_push: int) -> int:
        keep = min(s_push, self.cap) if self.cap > 0 else s_push
        return 4 * self.R * self.K * keep  # 4 B per retained sample

    def pipelined_records(self, recs, rec_off: torch.Tensor, timing: bool = False,
                          mode: Optional[str] = None, timing_reps: int = 1) -> "PipelinedReports":
        """pipelined() over record streams resident in HBM (compute_stats_records: bucketing,
        classification and the class kernels -- side-stream fork / join and stream-ordered
        scratch included -- captured into the report graphs).  recs: one record tensor or a list
        of them (same layout, rec_off shared), as ns for pipelined()."""
        ins = list(recs) if isinstance(recs, (list, tuple)) else [recs]
        return PipelinedReports(self, None, 0, timing, mode=mode, stats_bytes=8 * ins[0].shape[0],
                                timing_reps=timing_reps,
                                stats=[lambda r=r: self.compute_stats_records(r, rec_off) for r in ins],
                                inputs=[(r, rec_off) for r in ins])

    def _unpack(self, buf: Optional[torch.Tensor] = None) -> BatchResult:
        R = self.R
        h = (self.h_out if buf is None else buf).numpy()
        gr = h[0:8 * R].view(np.float64).copy() if self.relative else None
        gi = h[8 * R:16 * R].view(np.float64).copy() if self.individual else None
        sr = h[16 * R:17 * R].astype(bool) if self.relative else None
        si = h[17 * R:18 * R].astype(bool) if self.individual else None
        return BatchResult(gr, gi, sr, si, int(h[self._e:self._e + 4].view(np.int32)[0]))


class ReportGraph:
    """HIP graphs over a MatrixReporter's fixed buffers.  1 GPU: ``full`` is the whole
    report (column-reference init, segment statistics, scores + straggler masks, the
    device-to-host copy of the packed results) and is what ``run()`` replays; the same work
    is also captured as two halves, ``stats`` and ``rest``, for callers that record timing
    events between them (``run_stats()`` + ``run_rest()``).  One graph instead of two saves
    ~12 us per configs[1] report on MI355X (0.685 -> 0.673 ms, tools/ab_report_overhead.py).
    N GPUs: ``stats`` only; the partials exchange stays an eager collective."""

    def __init__(self, rep: MatrixReporter, ns: Optional[torch.Tensor], s_push: int, stats=None):
        self.rep = rep
        if stats is None:  # the statistics phase (record streams: MatrixReporter.graph_records)
            stats = lambda: rep.compute_stats(ns, s_push)  # noqa: E731
        _warm_up(rep, stats)
        # the captured statistics phase trusts col_ref as the previous report's scores epilogue
        # left it (colref_ready at capture): replays must pair it with the scores (run_rest),
        # which run_stats checks against the reporter's flag -- kept current by every replay
        self._needs_clean = rep._colref_clean
        self.stats = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.stats):
            stats()
        self.rest = self.full = None
        if rep.exchange:
            # N GPUs: the shard's partials and the combine (+ the result copy) as graphs too;
            # only the all_gather of the partials between them runs eagerly
            self.partials = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.partials):
                rep._scores_partials()
            self.finalize = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.finalize):
                rep._finalize()
                rep.h_out.copy_(rep.out, non_blocking=True)
        else:
            self.rest = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.rest):
                rep.compute_scores()
                rep.h_out.copy_(rep.out, non_blocking=True)
            self.full = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.full):
                stats()
                rep.compute_scores()
                rep.h_out.copy_(rep.out, non_blocking=True)

    def _check_clean(self) -> None:
        if self._needs_clean and not self.rep._colref_clean:
            raise RuntimeError("ReportGraph: the statistics graph was captured to follow a scores "
                               "phase (its epilogue re-initialises the column reference); the last "
                               "statistics phase was not followed by run_rest()")

    def run_stats(self) -> None:
        self._check_clean()
        self.rep._order_after_inflight()
        self.stats.replay()
        self.rep._colref_clean = False

    def run_rest(self) -> BatchResult:
        rep = self.rep
        rep._order_after_inflight()
        if self.rest is None:  # N GPUs: partials graph, eager all_gather, combine graph
            self.partials.replay()
            rep._colref_clean = rep._fuse_ref()
            rep._exchange()
            self.finalize.replay()
            _wait(rep.device)
            return rep._unpack()
        self.rest.replay()
        rep._colref_clean = rep._fuse_ref()
        _wait(rep.device)
        return rep._unpack()

    def run(self) -> BatchResult:
        if self.full is None:
            self.run_stats()
            return self.run_rest()
        self._check_clean()
        self.rep._order_after_inflight()
        self.full.replay()
        self.rep._colref_clean = self.rep._fuse_ref()
        _wait(self.rep.device)
        return self.rep._unpack()


def _warm_up(rep: MatrixReporter, stats) -> None:
    """One eager report on a side stream (first-launch setup outside any graph capture);
    stats() runs the statistics phase.  The individual history is restored afterwards: the
    warm-up must not fold whatever the inputs hold now into it (the graphs' reports advance it
    exactly as report() does)."""
    d = rep.device
    rep._order_after_inflight()
    saved = rep.hist.clone() if rep.hist is not None else None
    side = torch.cuda.Stream(d)
    side.wait_stream(torch.cuda.current_stream(d))
    with torch.cuda.stream(side):
        stats()
        if not rep.exchange:
            rep.compute_scores()
        elif rep._fuse_ref():  # N GPUs: leave col_ref initialised without the exchange
            rep.col_ref[:rep.K].fill_(0x7F800000)
            rep.col_ref[rep.K:2 * rep.K].zero_()
            rep._colref_clean = True
        if saved is not None:
            rep.hist.copy_(saved)
    torch.cuda.current_stream(d).wait_stream(side)
    torch.cuda.synchronize(d)


# NVRX_PIPE_D2H=copy: pipelined reports write a device buffer and copy it to the pinned one
# (one more graph node) instead of the scores kernel writing pinned host memory directly
_PIPE_COPY = os.environ.get("NVRX_PIPE_D2H", "") == "copy"
# NVRX_PIPE_MODE (timing A/B; PipelinedReports(mode=...) overrides the default, "auto"): "alt" each
# report on its own stream of two; "side" the statistics phases on one stream, the rest of every
# report on another; "whole" one whole-report graph per report on the caller's stream (round 4)
_PIPE_MODE = os.environ.get("NVRX_PIPE_MODE", "")
# "auto": alt while a report's statistics phase reads at most this many bytes.  Two reports'
# statistics kernels then overlap at their launch boundaries (one launch's ramp and tail, ~15-35
# us) -- configs[1] (4.3 GB) 0.673-0.687 -> 0.638-0.651 ms per report (with the stagger below,
# profiles/r05/pipe_modes.json); a longer phase gains
# nothing there and loses to the two kernels sharing the GPU for their whole duration: configs[2]
# (34 GB) 5.57 ms whole, 5.65 side, 5.79 alt (profiles/r05/pipe_modes.json).  Above it: whole on 1
# GPU, side on N GPUs (the exchange sits between a report's phases, so it needs two streams).
PIPE_ALT_MAX_BYTES = 8 << 30

TIMED_SPIN_CYCLES = 50_000  # ~20-25 us of device spin ahead of a timed report
STAGGER_FRAC = 0.25  # PipelinedReports: a burst's second report starts this much of a phase later


def _spin(cycles: int) -> None:
    """A one-wave device spin on the current stream (torch's private _sleep kernel)."""
    spin = getattr(torch.cuda, "_sleep", None)
    if spin is not None:
        spin(int(cycles))


class _Slot:
    """The buffers of one report in flight: segment statistics, column reference (+ its f32
    form), the scores epilogue's completion counter, the record-stream bucketing output, the
    packed results (+ error word) and, on N GPUs, the shard's partials and their gathered copy.
    Slot 0 is the reporter's own set; `clean` mirrors MatrixReporter._colref_clean for this
    slot's column reference."""

    _FIELDS = ("stats", "col_ref", "_ref_f32", "done", "_bucket", "out", "err", "partials", "gathered")

    def __init__(self, rep: MatrixReporter, primary: bool):
        self.primary = primary
        if primary:
            self.vals = [getattr(rep, f, None) for f in _Slot._FIELDS]
            self.clean = rep._colref_clean
        else:
            out = torch.zeros_like(rep.out)
            self.vals = [ops.SegmentStats.empty(rep.R * rep.K, rep.device), torch.empty_like(rep.col_ref),
                         torch.empty_like(rep._ref_f32), torch.zeros_like(rep.done), None, out,
                         out[rep._e:rep._e + 4].view(torch.int32), torch.empty_like(rep.partials),
                         torch.empty_like(rep.gathered) if rep.gathered is not None else None]
            self.clean = False  # uninitialised: its first statistics phase initialises it

    def bind(self, rep: MatrixReporter):
        """Context: rep's buffers are this slot's (graph capture bakes them into the kernels; the
        eager exchange reads and writes them)."""
        slot = self

        class _Bound:
            def __enter__(self):
                self.saved = [getattr(rep, f, None) for f in _Slot._FIELDS] + [rep._colref_clean]
                for f, v in zip(_Slot._FIELDS, slot.vals):
                    setattr(rep, f, v)
                rep._colref_clean = slot.clean

            def __exit__(self, *exc):
                slot.clean = rep._colref_clean
                slot.vals = [getattr(rep, f, None) for f in _Slot._FIELDS]  # a bucket allocated inside
                restore = slot.vals if slot.primary else self.saved[:-1]
                for f, v in zip(_Slot._FIELDS, restore):
                    setattr(rep, f, v)
                rep._colref_clean = slot.clean if slot.primary else self.saved[-1]
                return False

        return _Bound()


class PipelinedReports:
    """Full reports as HIP graphs, two in flight.  Each report -- column-reference init,
    statistics, scores + straggler masks -- ends with its packed results landing in one of two
    pinned host buffers, so the host can read report i while report i+1 runs: the GPU sees
    back-to-back reports instead of one report per host round trip.
    mode "alt": report i runs on stream i % 2 with its own set of statistics / reference
    buffers (_Slot), so report i+1's statistics kernel starts while report i's drains instead of
    after it (the launch-to-launch transition of one stream); report i's scores wait for report
    i-1's, so the individual history advances in submission order.  "side": every statistics
    phase on one stream, every rest on another (buffer sets per report in flight as in alt).
    "whole": one whole-report graph per report on the caller's stream (1 GPU).  "auto" (default):
    alt for statistics phases up to PIPE_ALT_MAX_BYTES, else whole (side on N GPUs); on N GPUs
    the choice takes the largest shard's bytes -- one all_reduce in the constructor, so every
    rank constructs its PipelinedReports at the same point, as it calls report().  With two
    streams the inputs a report reads must not change until it is collected (collect() orders
    the caller's stream after it).  N GPUs (exchange): per report the statistics, the shard's
    partials and the combine (+ result copy) are graphs and the all_gather of the partials is
    issued eagerly between them, in report order on every rank (the gathered buffers are per
    report in flight too).
    timing: submit(timed=True) first lets the reports in flight finish, then replays the
    statistics phase as its own graph between two timing events (ROCm's torch refuses events
    inside a capture) and the rest of the report as another -- a clean measurement of the
    statistics kernel on an otherwise idle device, for a sample of the reports.  timing_reps=n: that
    graph holds the statistics phase n times back to back (same inputs and outputs each time) and
    collect() returns the mean per phase, so the events' own overhead and a graph launch are spread
    over n phases.
    stats: the statistics phase as a callable, or a list of them, one per input set (report i
    runs stats[i % len(stats)]; default: compute_stats(ns, s_push); record streams:
    MatrixReporter.pipelined_records).  inputs: per input set, the tensors its statistics phase
    reads; collect() raises if one of them was modified in place by torch while the report was
    in flight.
    Other work on the same reporter (report(), a ReportGraph, compute_stats, reset_history)
    issued before collect() is ordered after the reports in flight
    (MatrixReporter._order_after_inflight)."""

    def __init__(self, rep: MatrixReporter, ns: Optional[torch.Tensor], s_push: int,
                 timing: bool = False, stats=None, mode: Optional[str] = None,
                 timing_reps: int = 1,
                 stats_bytes: Optional[int] = None, depth: int = 2, inputs=None):
        self.mode = mode or _PIPE_MODE or "auto"
        if stats_bytes is None:  # the matrix path: 4 B per retained sample
            stats_bytes = rep._matrix_bytes(s_push)
        if stats is None:
            stats = [lambda: rep.compute_stats(ns, s_push)]  # noqa: E731
            inputs = [(ns,)] if inputs is None else inputs
        elif callable(stats):
            stats = [stats]
        self.inputs = list(inputs) if inputs is not None else [() for _ in stats]
        if len(self.inputs) != len(stats) or depth % len(stats) != 0:
            raise ValueError(f"pipelined reports: {len(stats)} input sets for depth {depth} "
                             "(one inputs entry per set; the set count divides depth)")
        if self.mode == "auto":
            if rep.exchange and rep.world > 1:  # one mode on every rank (shards differ in size)
                x = torch.tensor([float(stats_bytes)], dtype=torch.float64,
                                 device="cpu" if rep.gloo else rep.device)
                torch.distributed.all_reduce(x, torch.distributed.ReduceOp.MAX, group=rep.group)
                stats_bytes = int(x.item())
            self.mode = ("alt" if stats_bytes <= PIPE_ALT_MAX_BYTES else
                         "side" if rep.exchange else "whole")
        if self.mode not in ("alt", "side", "whole"):
            raise ValueError(f"pipelined reports: mode {self.mode!r} (auto | alt | side | whole)")
        if rep.exchange and self.mode == "whole":
            raise RuntimeError("pipelined reports on N GPUs: two streams only (mode 'whole' is 1 GPU)")
        self.alt = self.mode != "whole"  # two streams, a buffer set per report in flight
        if depth < 2 or (depth > 2 and not self.alt):
            raise ValueError("pipelined reports: depth >= 2 (> 2 with two streams only)")
        self.depth = depth
        self.rep, self.timing = rep, timing
        if timing_reps < 1:
            raise ValueError("timing_reps >= 1")
        self.timing_reps = timing_reps
        self.bufs = [torch.zeros_like(rep.h_out).pin_memory() for _ in range(depth)]

        def scores(k: int):
            # the scores kernel writes the pinned buffer itself when its epilogue stores the
            # error word (fused reference, R <= FUSED_REF_MAX_ROWS); otherwise the error word is
            # zeroed on the device first and the results copied
            if _PIPE_COPY or not rep._fuse_ref():
                rep.compute_scores()
                self.bufs[k].copy_(rep.out, non_blocking=True)
            else:
                rep.compute_scores(out_buf=self.bufs[k])

        def capture(with_stats: bool, rest: bool, k: int, reps: int = 1):
            g = torch.cuda.CUDAGraph()
            ready = rep._colref_clean
            with torch.cuda.graph(g):
                for i in range(reps if with_stats else 0):
                    # a repeated phase reads the same inputs: the fused reference the previous one
                    # left is the same minimum, so it needs no re-initialisation either
                    rep._colref_clean = ready
                    stats[k % len(stats)]()
                if rest:
                    scores(k)
            return g

        def capture_fn(fn):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            return g

        if self.alt:
            self.slots = [_Slot(rep, True)] + [_Slot(rep, False) for _ in range(depth - 1)]
            self.stats_g, self.rest_g, self.part_g, self.fin_g, self.stats_t = [], [], [], [], []
            for k, slot in enumerate(self.slots):
                with slot.bind(rep):
                    _warm_up(rep, stats[k % len(stats)])  # initialises this slot's column reference too
                    ready = rep._colref_clean
                    self.stats_g.append(capture(True, False, k))
                    if timing:  # the timed statistics phase, timing_reps times in one graph,
                        rep._colref_clean = ready  # replacing stats_g in a timed report
                        self.stats_t.append(capture(True, False, k, self.timing_reps))
                    if rep.exchange:  # N GPUs: partials | eager all_gather | combine + result copy
                        self.part_g.append(capture_fn(rep._scores_partials))
                        self.fin_g.append(capture_fn(lambda k=k: (
                            rep._finalize(), self.bufs[k].copy_(rep.out, non_blocking=True))))
                    else:
                        self.rest_g.append(capture(False, True, k))
            self._needs_clean = rep._colref_clean
            self.streams = [torch.cuda.Stream(rep.device) for _ in range(depth)]
            self.hist_done = [torch.cuda.Event() for _ in range(depth)]
            self.stats_done = [torch.cuda.Event() for _ in range(depth)]
        else:
            _warm_up(rep, stats[0])
            self._needs_clean = rep._colref_clean  # as ReportGraph: every graph here pairs both phases
            self.full = [capture(True, True, k) for k in range(2)]
            if timing:
                self.stats = capture(True, False, 0, self.timing_reps)
                self.rest = [capture(False, True, k) for k in range(2)]
        if timing:
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        # blocking-sync events: wait_event's fallback sleeps instead of polling
        self.done = [torch.cuda.Event(blocking=True) for _ in range(depth)]
        self._versions = [None] * depth  # the inputs' version counters at each slot's submit
        # the one-time stagger of a burst's second report: a quarter of the statistics phase at
        # ~6.5 TB/s (STAGGER_FRAC; NVRX_PIPE_STAGGER=0 disables), in spin cycles of ~2.2 GHz
        frac = float(os.environ.get("NVRX_PIPE_STAGGER", STAGGER_FRAC))
        self.stagger_cycles = int(frac * stats_bytes / 6.5e12 * 2.2e9) if stats_bytes else 0
        self._burst = -2
        self.pending = []  # (slot, statistics phases timed or 0) in flight, oldest first
        self.ready = []    # results collected early (a timed submit drains), oldest first
        self.n = 0
        self.last_input = None
        rep._pipes.add(self)

    def submit(self, timed: bool = False) -> None:
        """Queue the next report (at most `depth` in flight: collect() the oldest first)."""
        if len(self.pending) == self.depth:
            raise RuntimeError(f"{self.depth} reports in flight: collect() one first")
        if self._needs_clean and not self.rep._colref_clean:
            raise RuntimeError("PipelinedReports: an unpaired statistics phase (ReportGraph."
                               "run_stats without run_rest) left the column reference in use")
        if timed and not self.timing:
            raise RuntimeError("PipelinedReports(timing=True) is needed for timed reports")
        k = self.n % self.depth
        if timed:
            while self.pending:  # the device idles before the measured statistics phase
                self.ready.append(self._land())
        self.rep._order_after_inflight(exclude=self)  # another pipeline's reports on this reporter
        self._versions[k] = [t._version for t in self.inputs[k % len(self.inputs)]]
        if timed:
            # a short spin keeps the device busy while the host queues the graphs, so the
            # first event fires right before the statistics phase rather than a graph-launch
            # latency ahead of it
            _spin(TIMED_SPIN_CYCLES)
        if self.alt:
            # alt: report i on stream i % 2; side: every statistics phase on stream 0, every rest
            # on stream 1 (slot k's previous report has finished with its buffers: done[k])
            s = self.streams[k] if self.mode == "alt" else self.streams[0]
            # the caller's work so far (inputs; the wait for the collected reports) comes first
            s.wait_stream(torch.cuda.current_stream(self.rep.device))
            s.wait_event(self.done[k])
            if self.mode == "alt" and self.depth > 2:
                # at most two statistics phases at once: report i's starts on the device as soon
                # as report i-2's has finished, with no host round trip in between
                s.wait_event(self.stats_done[(k - 2) % self.depth])
            if (self.mode == "alt" and self.stagger_cycles > 0 and len(self.pending) == 1
                    and self.n == self._burst + 1):
                # the second report of a burst (the pipeline was empty when the first was
                # submitted) starts a quarter of a statistics phase after the first: staggered,
                # one report's statistics kernel covers the other's end, scores and the host's
                # next submission; started together, the two stay locked and the device idles at
                # every pair's end
                with torch.cuda.stream(s):
                    _spin(self.stagger_cycles)
            with torch.cuda.stream(s):
                if timed:
                    self.ev[0].record(s)
                (self.stats_t[k] if timed else self.stats_g[k]).replay()
                if timed:
                    self.ev[1].record(s)
            self.stats_done[k].record(s)
            if self.mode == "side":
                s = self.streams[1]
                s.wait_event(self.stats_done[k])
            with torch.cuda.stream(s):
                s.wait_event(self.hist_done[(k - 1) % self.depth])  # report i-1's history update first
                if self.rep.exchange:
                    self.part_g[k].replay()
                    self.hist_done[k].record(s)
                    # the eager all_gather of this slot's partials, ordered after them on s (every
                    # rank submits its reports, hence its collectives, in the same order)
                    with self.slots[k].bind(self.rep):
                        self.rep._exchange()
                    self.fin_g[k].replay()
                else:
                    self.rest_g[k].replay()
                    self.hist_done[k].record(s)
            self.done[k].record(s)
        else:
            if timed:
                self.ev[0].record()
                self.stats.replay()
                self.ev[1].record()
                self.rest[k].replay()
            else:
                self.full[k].replay()
            self.done[k].record()
        self.rep._colref_clean = self.rep._fuse_ref()
        if not self.pending:
            self._burst = self.n  # the first report of a burst (submitted to an empty pipeline)
        self.pending.append((k, self.timing_reps if timed else 0))
        self.n += 1

    def _land(self):
        k, timed = self.pending.pop(0)  # timed: the timed statistics phases (0: untimed)
        ev = self.done[k]
        wait_event(ev)
        if self.alt:  # the caller's later work (new inputs, the history) follows this report
            torch.cuda.current_stream(self.rep.device).wait_event(ev)
        self.last_input = k % len(self.inputs)  # the input set the collected report read
        now = [t._version for t in self.inputs[k % len(self.inputs)]]
        if now != self._versions[k]:
            raise RuntimeError("PipelinedReports: an input of this report was modified in place "
                               "while the report was in flight (submit() -> collect()); its "
                               "results are undefined -- modify inputs only after collect()")
        ms = self.ev[0].elapsed_time(self.ev[1]) / timed if timed else None
        return self.rep._unpack(self.bufs[k]), ms

    def collect(self):
        """(BatchResult, statistics ms for a timed report or None) of the oldest report, once it
        landed."""
        if self.ready:
            return self.ready.pop(0)
        return self._land()
