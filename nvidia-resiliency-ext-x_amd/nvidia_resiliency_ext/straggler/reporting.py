"""Report, StragglerId and the HIP-backed ReportGenerator (drop-in for straggler/reporting.py).

Same constructor, same ``generate_report(section_summaries, kernel_summaries)`` contract,
same Report fields and formats as the reference (reporting.py:31-554).  What changed is
where the arithmetic runs: the per-kernel reference pack, the individual-history update
and every score are HIP kernels (libnvrx_hip.so, csrc/scores.hip) on the rank's GPU, and
the MIN all-reduce runs on the device tensor when the backend is RCCL ("nccl").

Exact reference quirks kept: kernel/section MED packed as float32 for the MIN reduce
(relative references are float32 values); -1 sentinel => NaN; history updated before the
individual score; "ncclDev" kernels dropped; scores gathered to rank 0 as float32;
MED == 0 (or zero total weight) raises ZeroDivisionError as the Python division does.
"""
from __future__ import annotations

import collections
import dataclasses
import math
import time
from typing import Any, Dict, List, Mapping, Optional, Tuple

import numpy as np
import torch

from . import dist_utils, ops
from .name_mapper import NameMapper
from .statistics import Statistic
from .summaries import KernelSummaries, columns_of
from ..common.device_utils import get_current_device

_SummaryType = Mapping[Statistic, float]


@dataclasses.dataclass(frozen=True)
class StragglerId:
    """Straggler identity (reporting.py:31-38)."""

    rank: int
    node: str


@dataclasses.dataclass(frozen=True)
class Report:
    """Performance report (reporting.py:41-82).

    Relative scores (0..1) compare a rank with the best rank; individual scores compare it
    with its own best history.  With ``gather_on_rank0=True`` the ``*_perf_scores`` hold
    every rank (only on rank 0); otherwise only the current rank.
    """

    gpu_relative_perf_scores: Mapping[int, float]
    section_relative_perf_scores: Mapping[str, Mapping[int, float]]
    gpu_individual_perf_scores: Mapping[int, float]
    section_individual_perf_scores: Mapping[str, Mapping[int, float]]
    rank_to_node: Mapping[int, str]
    local_section_summaries: Mapping[str, Any]
    local_kernel_summaries: Mapping[str, Any]
    generate_report_elapsed_time: float
    gather_on_rank0: bool
    rank: Optional[int]

    def identify_stragglers(self, gpu_rel_threshold: float = 0.75,
                            section_rel_threshold: float = 0.75,
                            gpu_indiv_threshold: float = 0.75,
                            section_indiv_threshold: float = 0.75) -> Dict[str, Any]:
        """Ranks whose score is strictly below the threshold (NaN never is) -- reporting.py:84-151."""

        def below(scores: Mapping[int, float], thr: float):
            return {StragglerId(rank=r, node=self.rank_to_node[r])
                    for r, d in scores.items() if d < thr}

        out: Dict[str, Any] = {
            "straggler_gpus_relative": below(self.gpu_relative_perf_scores, gpu_rel_threshold),
            "straggler_gpus_individual": below(self.gpu_individual_perf_scores, gpu_indiv_threshold),
            "straggler_sections_relative": {},
            "straggler_sections_individual": {},
        }
        for key, table, thr in (
                ("straggler_sections_relative", self.section_relative_perf_scores, section_rel_threshold),
                ("straggler_sections_individual", self.section_individual_perf_scores,
                 section_indiv_threshold)):
            for section, scores in (table or {}).items():
                s = below(scores, thr)
                if s:
                    out[key][section] = s
        return out


StragglerReport = Report


class _History:
    """Per-name running minimum of MED on the device (min_local_*_times, reporting.py:186-191)."""

    def __init__(self):
        self.slot: Dict[str, int] = {}
        self.names: List[str] = []
        self.values: Optional[torch.Tensor] = None  # f64 [capacity], +inf where unseen

    def slots_for(self, names: List[str], device) -> np.ndarray:
        for n in names:
            if n not in self.slot:
                self.slot[n] = len(self.names)
                self.names.append(n)
        need = len(self.names)
        cap = 0 if self.values is None else self.values.numel()
        if need > cap or self.values is None:  # allocated on first use, even with no names
            new = torch.full((max(need, 2 * cap, 64),), float("inf"), dtype=torch.float64,
                             device=device)
            if self.values is not None:
                new[:cap].copy_(self.values)
            self.values = new
        return np.fromiter((self.slot[n] for n in names), dtype=np.int32, count=len(names))

    def as_dict(self) -> Dict[str, float]:
        d: Dict[str, float] = collections.defaultdict(lambda: float("inf"))
        if self.values is not None and self.names:
            vals = self.values[: len(self.names)].cpu().numpy()
            for n, v in zip(self.names, vals):
                d[n] = float(v)
        return d


class ReportGenerator:
    """Generates the performance report from section and kernel summaries; must be called
    on every rank (it synchronizes).  Drop-in for reporting.py:154-554."""

    def __init__(self, scores_to_compute, gather_on_rank0=True, pg=None,
                 node_name='<notset>') -> None:
        self.is_computing_rel_scores = 'relative_perf_scores' in scores_to_compute
        self.is_computing_indiv_scores = 'individual_perf_scores' in scores_to_compute
        self.gather_on_rank0 = gather_on_rank0
        self.group = pg
        self.world_size = dist_utils.get_world_size(self.group)
        self.rank = dist_utils.get_rank(self.group)
        self.node_name = node_name
        self._hist_k = _History()
        self._hist_s = _History()
        self.name_mapper = NameMapper(pg=pg)
        self._knames: Tuple[str, ...] = ()
        self._kcache = None  # (kernel names, their ids, their history slots) of the last report
        self.rank_to_node: Dict[int, str] = collections.defaultdict(lambda: '<unk>')
        self._device: Optional[torch.device] = None

    # reference attribute names, materialised from the device history on access
    @property
    def min_local_kernel_times(self) -> Dict[str, float]:
        return self._hist_k.as_dict()

    @property
    def min_local_section_times(self) -> Dict[str, float]:
        return self._hist_s.as_dict()

    def _dev(self) -> torch.device:
        if self._device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("the straggler scoring path runs on a HIP device (MI355X); "
                                   "no GPU is visible to this process")
            self._device = get_current_device()
        return self._device

    def _maybe_gather_rank_to_node(self) -> None:
        """reporting.py:316-328"""
        if not self.rank_to_node:
            if self.gather_on_rank0:
                gathered = dist_utils.all_gather_object((self.rank, self.node_name), self.group)
                self.rank_to_node = dict(gathered)
            else:
                self.rank_to_node[self.rank] = self.node_name

    @staticmethod
    def _filter_out_nccl_kernels(kernel_summaries):
        """reporting.py:330-336: drop names containing "ncclDev", keep order."""
        if isinstance(kernel_summaries, KernelSummaries):
            keep = np.fromiter(("ncclDev" not in n for n in kernel_summaries.names), dtype=bool,
                               count=len(kernel_summaries))
            return kernel_summaries if keep.all() else kernel_summaries.select(keep)
        if "ncclDev" not in "\0".join(kernel_summaries):  # (one search instead of one per name)
            return dict(kernel_summaries)  # (a new mapping, as the comprehension makes)
        return {k: v for k, v in kernel_summaries.items() if "ncclDev" not in k}

    # ------------------------------------------------------------------ device scoring
    def _score_local(self, section_summaries, kernel_summaries):
        """Individual / relative GPU and section scores of this rank, on the device."""
        dev = self._dev()
        knames = self._knames
        snames = list(section_summaries.keys())
        K, S = len(knames), len(snames)
        kmed, kavg, knum = columns_of(kernel_summaries)
        smed = np.fromiter((float(section_summaries[s][Statistic.MED]) for s in snames),
                           dtype=np.float64, count=S)
        rel, ind = self.is_computing_rel_scores, self.is_computing_indiv_scores
        nk = self.name_mapper.kernel_counter if rel else 0
        nsec = self.name_mapper.section_counter if rel else 0
        # the kernels' ids and history slots never change once assigned: a report over the same
        # kernel names as the previous one (the usual case) reuses them
        cache = self._kcache if self._kcache is not None and self._kcache[0] == knames else None
        kid = (cache[1] if cache is not None else
               np.fromiter((self.name_mapper.kernel_name_to_id[n] for n in knames), np.int32, K)
               if rel else np.zeros(0, np.int32))
        sid = (np.fromiter((nk + self.name_mapper.section_name_to_id[n] for n in snames),
                           np.int32, S) if rel else np.zeros(0, np.int32))
        kslot = (cache[2] if cache is not None and self._hist_k.values is not None else
                 self._hist_k.slots_for(knames, dev) if ind else np.zeros(0, np.int32))
        self._kcache = (knames, kid, kslot)
        sslot = self._hist_s.slots_for(snames, dev) if ind else np.zeros(0, np.int32)

        # one host->device transfer of every input column
        f64_in = np.concatenate([kmed, kavg, smed])
        i32_in = np.concatenate([np.minimum(knum, np.iinfo(np.int32).max).astype(np.int32),
                                 kid, sid, kslot, sslot]).astype(np.int32)
        # (pinned staging: asynchronous copies, ordered before the kernels on the stream)
        pin = dev.type == "cuda"
        f64_h, i32_h = torch.from_numpy(f64_in), torch.from_numpy(i32_in)
        if pin:
            f64_h, i32_h = f64_h.pin_memory(), i32_h.pin_memory()
        f64_d = f64_h.to(dev, non_blocking=pin)
        i32_d = i32_h.to(dev, non_blocking=pin)
        d_kmed, d_kavg, d_smed = f64_d[:K], f64_d[K:2 * K], f64_d[2 * K:]
        o = 0
        d_knum = i32_d[o:o + K]; o += K  # noqa: E702
        d_kid = i32_d[o:o + len(kid)]; o += len(kid)  # noqa: E702
        d_sid = i32_d[o:o + len(sid)]; o += len(sid)  # noqa: E702
        d_kslot = i32_d[o:o + len(kslot)]; o += len(kslot)  # noqa: E702
        d_sslot = i32_d[o:o + len(sslot)]  # noqa: E702
        err = torch.zeros(1, dtype=torch.int32, device=dev)

        times = None
        if rel:
            # reporting.py:269-281: float32 [K + Nsec] = -1, MED by id, MIN over ranks
            times = ops.pack_min_times(torch.cat([d_kmed, d_smed]), torch.cat([d_kid, d_sid]),
                                       nk + nsec)
            if self.world_size > 1:
                comm_dev = dist_utils.get_device_for_backend(self.group)
                if comm_dev.type == "cpu":
                    t = times.cpu()
                    dist_utils.all_reduce(t, op=torch.distributed.ReduceOp.MIN, group=self.group)
                    times = t.to(dev)
                else:
                    dist_utils.all_reduce(times, op=torch.distributed.ReduceOp.MIN, group=self.group)
        partials = ops.scores(d_knum.view(1, K), d_kmed.view(1, K), d_kavg.view(1, K),
                              ref=times if rel else None, ref_index=d_kid if rel else None,
                              hist=self._hist_k.values if ind else None,
                              hist_index=d_kslot if ind else None,
                              hist_stride=(self._hist_k.values.numel() if ind else 0), err=err)
        gr_d, gi_d, _, _ = ops.finalize_scores(partials, 1, rel=True, ind=True, err=err)
        parts = [gr_d, gi_d]
        if S > 0:
            h = self._hist_s.values[d_sslot.long()].view(1, S) if ind else None
            present = torch.ones((1, S), dtype=torch.uint8, device=dev)
            s_rel, s_ind = ops.section_scores(d_smed.view(1, S), present,
                                              ref_in=times if rel else None,
                                              ref_index=d_sid if rel else None,
                                              hist=h, rel=rel, ind=ind, err=err)
            if ind:
                self._hist_s.values[d_sslot.long()] = h.view(-1)
            parts += [s_rel.view(-1) if rel else torch.full((S,), math.nan, dtype=torch.float64, device=dev),
                      s_ind.view(-1) if ind else torch.full((S,), math.nan, dtype=torch.float64, device=dev)]
        parts.append(err.to(torch.float64))
        out = torch.cat(parts).cpu().numpy()  # the one device->host transfer (synchronizes)
        if int(out[-1]) != 0:
            raise ZeroDivisionError("float division by zero")
        gr, gi = float(out[0]), float(out[1])
        srel = dict(zip(snames, map(float, out[2:2 + S]))) if rel else {}
        sind = dict(zip(snames, map(float, out[2 + S:2 + 2 * S]))) if ind else {}
        return (gi if ind else float("nan")), sind, (gr if rel else float("nan")), srel

    # ------------------------------------------------------------------ gather (reporting.py:338-419)
    def _get_tensor_from_scores(self, gi, si, gr, sr):
        nsec = self.name_mapper.section_counter
        t = np.full(2 + 2 * nsec, np.nan, dtype=np.float32)
        t[0] = gi
        t[1] = gr
        for sid in range(nsec):
            name = self.name_mapper.get_section_name(sid)
            t[2 + sid] = si.get(name, float("nan"))
            t[2 + nsec + sid] = sr.get(name, float("nan"))
        return torch.from_numpy(t)

    def _get_scores_from_tensor(self, tensor) -> Tuple[float, Mapping, float, Mapping]:
        v = tensor.cpu().numpy().astype(np.float64)
        nsec = (len(v) - 2) // 2
        assert nsec == self.name_mapper.section_counter
        names = [self.name_mapper.get_section_name(i) for i in range(nsec)]
        si = {n: float(v[2 + i]) for i, n in enumerate(names)}
        sr = {n: float(v[2 + nsec + i]) for i, n in enumerate(names)}
        return float(v[0]), si, float(v[1]), sr

    def _gather_results_on_rank0(self, gi, si, gr, sr):
        tensor = self._get_tensor_from_scores(gi, si, gr, sr)
        gathered = dist_utils.gather_on_rank0(tensor, group=self.group)
        res_gi: Dict[int, float] = {}
        res_gr: Dict[int, float] = {}
        res_si: Dict[str, Dict[int, float]] = collections.defaultdict(dict)
        res_sr: Dict[str, Dict[int, float]] = collections.defaultdict(dict)
        if self.rank == 0:
            for r in range(self.world_size):
                g_i, s_i, g_r, s_r = self._get_scores_from_tensor(gathered[r])
                if self.is_computing_indiv_scores:
                    res_gi[r] = g_i
                    for s in s_i:
                        res_si[s][r] = s_i[s]
                if self.is_computing_rel_scores:
                    res_gr[r] = g_r
                    for s in s_r:
                        res_sr[s][r] = s_r[s]
        return res_gi, dict(res_si), res_gr, dict(res_sr)

    # ------------------------------------------------------------------ entry point
    def generate_report(self, section_summaries: Mapping[str, _SummaryType],
                        kernel_summaries: Mapping[str, _SummaryType]):
        """Report on rank 0 (all ranks) / None elsewhere when gathering; else this rank's
        report on every rank.  reporting.py:421-554."""
        report_start = time.perf_counter_ns()
        self.world_size = dist_utils.get_world_size(self.group)
        self.rank = dist_utils.get_rank(self.group)
        kernel_summaries = self._filter_out_nccl_kernels(kernel_summaries)
        self._knames = tuple(kernel_summaries.keys())
        self._maybe_gather_rank_to_node()
        if self.is_computing_rel_scores or self.gather_on_rank0:
            known = self._kcache is not None and self._kcache[0] == self._knames
            self.name_mapper.gather_and_assign_ids(kernel_names=list(self._knames),
                                                   section_names=list(section_summaries.keys()),
                                                   kernels_known=known)
        gi, si, gr, sr = self._score_local(section_summaries, kernel_summaries)

        res_gi: Mapping[int, float] = {}
        res_si: Mapping[str, Mapping[int, float]] = {}
        res_gr: Mapping[int, float] = {}
        res_sr: Mapping[str, Mapping[int, float]] = {}
        if self.gather_on_rank0:
            gathered = self._gather_results_on_rank0(gi, si, gr, sr)
            if self.rank == 0:
                res_gi, res_si, res_gr, res_sr = gathered
        else:
            if self.is_computing_indiv_scores:
                res_gi = {self.rank: gi}
                res_si = {k: {self.rank: v} for k, v in si.items()}
            if self.is_computing_rel_scores:
                res_gr = {self.rank: gr}
                res_sr = {k: {self.rank: v} for k, v in sr.items()}
        elapsed_ms = (time.perf_counter_ns() - report_start) * 1e-6
        report = Report(gpu_relative_perf_scores=res_gr, section_relative_perf_scores=res_sr,
                        gpu_individual_perf_scores=res_gi, section_individual_perf_scores=res_si,
                        rank_to_node=dict(self.rank_to_node),
                        local_section_summaries=section_summaries,
                        local_kernel_summaries=kernel_summaries,
                        generate_report_elapsed_time=elapsed_ms,
                        gather_on_rank0=self.gather_on_rank0, rank=self.rank)
        if self.gather_on_rank0:
            return report if self.rank == 0 else None
        return report
