"""Batched scoring of many (simulated) ranks resident in HBM -- the hot path at scale.

``MatrixReporter`` runs the whole report for R ranks x K kernels in one pass over a
uint32 ns matrix ``[R][K][S_push]`` (the last ``cap`` samples of every (rank, kernel)
retained, as the reference's per-kernel rings keep them):

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

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import ops


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
                 round_f32: bool = False, group=None, device=None):
        self.R, self.K, self.cap = R, K, cap
        self.relative, self.individual = relative, individual
        self.thr_rel, self.thr_ind = thr_rel, thr_ind
        self.mode, self.round_f32 = mode, round_f32
        self.group = group
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        d = self.device
        self.world = 1
        if group is not None or (torch.distributed.is_available() and torch.distributed.is_initialized()):
            self.world = torch.distributed.get_world_size(group)
        self.stats = ops.SegmentStats.empty(R * K, d)
        self.col_valid = col_valid
        self.ref = torch.empty(K, dtype=torch.float32, device=d)
        self.ref_scratch = torch.empty(2 * max(K, 1), dtype=torch.int32, device=d)
        self.hist = torch.full((R, K), float("inf"), dtype=torch.float32, device=d) if individual else None
        self.partials = torch.empty((R, 6), dtype=torch.float64, device=d)
        self.gathered = (torch.empty((self.world, R, 6), dtype=torch.float64, device=d)
                         if self.world > 1 else None)
        self.err = torch.zeros(1, dtype=torch.int32, device=d)
        # pinned host landing buffers for the scores / straggler masks
        self.h_scores = torch.empty((2, R), dtype=torch.float64, pin_memory=True)
        self.h_masks = torch.empty((2, R), dtype=torch.uint8, pin_memory=True)
        self.h_err = torch.empty(1, dtype=torch.int32, pin_memory=True)

    def reset_history(self):
        if self.hist is not None:
            self.hist.fill_(float("inf"))

    # -- the three device phases, separately callable (bench times the stats kernel) --
    def compute_stats(self, ns: torch.Tensor, s_push: int) -> ops.SegmentStats:
        return ops.segment_stats_strided(ns.view(-1), self.R * self.K, s_push, 0, s_push,
                                         cap=self.cap, mode=self.mode, out=self.stats)

    def compute_partials(self) -> torch.Tensor:
        R, K = self.R, self.K
        st = self.stats.view(R, K)
        self.err.zero_()
        if self.relative:
            ops.kernel_ref(st.num, st.med, ref=self.ref, scratch=self.ref_scratch)
        ops.scores(st.num, st.med, st.avg, col_valid=self.col_valid,
                   ref=self.ref if self.relative else None, hist=self.hist,
                   partials=self.partials, err=self.err)
        if self.world > 1:
            torch.distributed.all_gather_into_tensor(self.gathered, self.partials, group=self.group)
            return self.gathered
        return self.partials

    def finalize(self, partials: torch.Tensor) -> BatchResult:
        nshards = partials.shape[0] if partials.dim() == 3 else 1
        gr, gi, sr, si = ops.finalize_scores(partials, self.R, nshards, self.round_f32,
                                             self.thr_rel, self.thr_ind, rel=self.relative,
                                             ind=self.individual, err=self.err)
        if gr is not None:
            self.h_scores[0].copy_(gr, non_blocking=True)
            self.h_masks[0].copy_(sr, non_blocking=True)
        if gi is not None:
            self.h_scores[1].copy_(gi, non_blocking=True)
            self.h_masks[1].copy_(si, non_blocking=True)
        self.h_err.copy_(self.err, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return BatchResult(
            self.h_scores[0].numpy().copy() if gr is not None else None,
            self.h_scores[1].numpy().copy() if gi is not None else None,
            self.h_masks[0].numpy().astype(bool) if gr is not None else None,
            self.h_masks[1].numpy().astype(bool) if gi is not None else None,
            int(self.h_err[0]),
        )

    def report(self, ns: torch.Tensor, s_push: int) -> BatchResult:
        """One full report: samples resident in HBM -> scores + straggler sets on host."""
        self.compute_stats(ns, s_push)
        return self.finalize(self.compute_partials())
