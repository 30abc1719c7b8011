"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of the reference ReportGenerator
semantics (straggler/reporting.py, name_mapper.py) for a *simulated* world of ranks.

`SimWorld.generate_report` returns, for every rank, exactly what that rank's reference
`ReportGenerator.generate_report` would return when all ranks call it collectively
(gloo/NCCL collectives replaced by their results: MIN all-reduce, gather, gather of
names).  Pinned against tests/golden/report_*.json, which tests/golden/make_golden.py
recorded from the reference itself running on gloo.  Only tests/ use this module.

Anchors (reporting.py unless noted):
  filter ncclDev :330-336      rank_to_node :316-328     NameMapper :name_mapper.py:56-81
  individual     :469-478, 298-314, 219-253, 196-217
  relative       :482-493, 255-296 (float32 pack, -1 => NaN)
  gather         :382-419, 338-380 (float32 scores)      Report :535-554
"""
from __future__ import annotations

import itertools
import math
from typing import Dict, List, Mapping, Optional

import numpy as np

MIN, MAX, MED, AVG, STD, NUM = "MIN", "MAX", "MED", "AVG", "STD", "NUM"


def f32(x: float) -> float:
    """float -> float32 -> float (the torch float32 tensor round trip)."""
    return float(np.float32(x))


class NameMapperSim:
    """name_mapper.py:22-161 -- ids shared by all ranks."""

    def __init__(self):
        self.kernel_name_to_id: Dict[str, int] = {}
        self.id_to_kernel_name: Dict[int, str] = {}
        self.section_name_to_id: Dict[str, int] = {}
        self.id_to_section_name: Dict[int, str] = {}
        self.kernel_counter = 0
        self.section_counter = 0
        self.gathers = 0

    def gather_and_assign_ids(self, per_rank_kernels: List[List[str]],
                              per_rank_sections: List[List[str]]) -> None:
        has_all = all(
            all(n in self.kernel_name_to_id for n in ks) and
            all(n in self.section_name_to_id for n in ss)
            for ks, ss in zip(per_rank_kernels, per_rank_sections))
        if has_all:  # is_all_true (dist_utils.py:109-116)
            return
        self.gathers += 1
        for s in itertools.chain.from_iterable(per_rank_sections):  # sections first (:486)
            if s not in self.section_name_to_id:
                self.section_name_to_id[s] = self.section_counter
                self.id_to_section_name[self.section_counter] = s
                self.section_counter += 1
        for k in itertools.chain.from_iterable(per_rank_kernels):
            if k not in self.kernel_name_to_id:
                self.kernel_name_to_id[k] = self.kernel_counter
                self.id_to_kernel_name[self.kernel_counter] = k
                self.kernel_counter += 1


class SimWorld:
    def __init__(self, world_size: int, scores_to_compute, gather_on_rank0: bool = True,
                 node_names: Optional[List[str]] = None):
        self.ws = world_size
        self.rel = "relative_perf_scores" in scores_to_compute
        self.ind = "individual_perf_scores" in scores_to_compute
        self.gather = gather_on_rank0
        self.node_names = node_names or ["<notset>"] * world_size
        self.hist_k = [dict() for _ in range(world_size)]  # min_local_kernel_times
        self.hist_s = [dict() for _ in range(world_size)]  # min_local_section_times
        self.mapper = NameMapperSim()
        self.rank_to_node: Optional[Dict[int, str]] = None

    @staticmethod
    def _gpu_score(kernels: Mapping[str, Mapping], reference: Mapping[str, float]) -> float:
        """reporting.py:219-253, sequential in dict order."""
        rank_score = float("nan")
        if kernels:
            wss = 0.0
            ws = 0.0
            n = 0
            for k, s in kernels.items():
                ref = reference[k]
                if math.isnan(ref):
                    continue
                n += 1
                score = ref / s[MED]
                weight = s[NUM] * s[AVG]
                wss += score * weight
                ws += weight
            if n > 0:
                rank_score = wss / ws
        return rank_score

    def generate_report(self, sections: List[Mapping[str, Mapping]],
                        kernels: List[Mapping[str, Mapping]]) -> List[Optional[dict]]:
        ws = self.ws
        kernels = [{k: v for k, v in kd.items() if "ncclDev" not in k} for kd in kernels]
        if self.rank_to_node is None:
            if self.gather:
                self.rank_to_node = {r: self.node_names[r] for r in range(ws)}
        if self.rel or self.gather:
            self.mapper.gather_and_assign_ids([list(k.keys()) for k in kernels],
                                              [list(s.keys()) for s in sections])
        gi = [float("nan")] * ws
        si: List[Dict[str, float]] = [{} for _ in range(ws)]
        gr = [float("nan")] * ws
        sr: List[Dict[str, float]] = [{} for _ in range(ws)]
        if self.ind:
            for r in range(ws):
                for k, s in kernels[r].items():
                    self.hist_k[r][k] = min(self.hist_k[r].get(k, float("inf")), s[MED])
                for k, s in sections[r].items():
                    self.hist_s[r][k] = min(self.hist_s[r].get(k, float("inf")), s[MED])
                gi[r] = self._gpu_score(kernels[r], self.hist_k[r])
                si[r] = {k: self.hist_s[r][k] / s[MED] for k, s in sections[r].items()}
        if self.rel:
            nk, ns = self.mapper.kernel_counter, self.mapper.section_counter
            t = np.full(nk + ns, -1.0, dtype=np.float32)
            per_rank = []
            for r in range(ws):
                v = np.full(nk + ns, -1.0, dtype=np.float32)
                for k, s in kernels[r].items():
                    v[self.mapper.kernel_name_to_id[k]] = s[MED]
                for k, s in sections[r].items():
                    v[nk + self.mapper.section_name_to_id[k]] = s[MED]
                per_rank.append(v)
            t = np.minimum.reduce(per_rank) if per_rank else t
            mk = {self.mapper.id_to_kernel_name[i]: (float(t[i]) if t[i] >= 0 else float("nan"))
                  for i in range(nk)}
            ms = {self.mapper.id_to_section_name[i]: (float(t[nk + i]) if t[nk + i] >= 0 else float("nan"))
                  for i in range(ns)}
            for r in range(ws):
                gr[r] = self._gpu_score(kernels[r], mk)
                sr[r] = {k: ms[k] / s[MED] for k, s in sections[r].items()}
        out: List[Optional[dict]] = []
        if self.gather:
            nsec = self.mapper.section_counter
            res_gi, res_gr = {}, {}
            res_si: Dict[str, Dict[int, float]] = {}
            res_sr: Dict[str, Dict[int, float]] = {}
            for r in range(ws):
                # float32 pack (reporting.py:354-360); missing sections -> NaN
                if self.ind:
                    res_gi[r] = f32(gi[r])
                    for sid in range(nsec):
                        name = self.mapper.id_to_section_name[sid]
                        res_si.setdefault(name, {})[r] = f32(si[r].get(name, float("nan")))
                if self.rel:
                    res_gr[r] = f32(gr[r])
                    for sid in range(nsec):
                        name = self.mapper.id_to_section_name[sid]
                        res_sr.setdefault(name, {})[r] = f32(sr[r].get(name, float("nan")))
            for r in range(ws):
                if r == 0:
                    out.append(dict(gpu_relative_perf_scores=res_gr,
                                    section_relative_perf_scores=res_sr,
                                    gpu_individual_perf_scores=res_gi,
                                    section_individual_perf_scores=res_si,
                                    rank_to_node=dict(self.rank_to_node),
                                    gather_on_rank0=True, rank=0))
                else:
                    out.append(None)
        else:
            for r in range(ws):
                out.append(dict(
                    gpu_relative_perf_scores={r: gr[r]} if self.rel else {},
                    section_relative_perf_scores={k: {r: v} for k, v in sr[r].items()} if self.rel else {},
                    gpu_individual_perf_scores={r: gi[r]} if self.ind else {},
                    section_individual_perf_scores={k: {r: v} for k, v in si[r].items()} if self.ind else {},
                    rank_to_node={r: self.node_names[r]},
                    gather_on_rank0=False, rank=r))
        return out


def section_summary_torch_semantics(ms: List[float]) -> dict:
    """Detector._get_section_summaries (straggler.py:171-197): f64, lower median,
    unbiased std (NaN for n == 1)."""
    a = np.asarray(ms, dtype=np.float64)
    s = np.sort(a)
    n = len(a)
    return {MIN: float(s[0]), MAX: float(s[-1]), MED: float(s[(n - 1) // 2]),
            AVG: float(np.mean(a)), STD: float(np.std(a, ddof=1)) if n > 1 else float("nan"),
            NUM: n}
