"""Column-store summaries: a read-only Mapping view over statistics arrays.

``KernelSummaries`` is what the Detector hands to the ReportGenerator: the device-computed
per-kernel statistics landed on the host as numpy columns, exposed as the reference's
``{name: {Statistic: value}}`` mapping (CuptiProfiler::getStats order: sorted by name).
The ReportGenerator reads the columns directly; a per-kernel dict is only built when a
caller indexes it.  Values are the float32 statistics widened exactly to Python floats
(straggler.py:211-219).
"""
from __future__ import annotations

import operator
from typing import Dict, Iterator, List, Mapping, Sequence

import numpy as np

from .statistics import Statistic

_ORDER = (Statistic.MIN, Statistic.MAX, Statistic.MED, Statistic.AVG, Statistic.STD)


class KernelSummaries(Mapping):
    def __init__(self, names: Sequence[str], num, mn, mx, med, avg, std):
        self.names: List[str] = list(names)
        self.num = np.asarray(num, dtype=np.int64)
        self.min = np.asarray(mn, dtype=np.float32)
        self.max = np.asarray(mx, dtype=np.float32)
        self.med = np.asarray(med, dtype=np.float32)
        self.avg = np.asarray(avg, dtype=np.float32)
        self.std = np.asarray(std, dtype=np.float32)
        self._index: Dict[str, int] = {n: i for i, n in enumerate(self.names)}

    def __getitem__(self, name: str) -> Dict[Statistic, float]:
        i = self._index[name]
        return {Statistic.MIN: float(self.min[i]), Statistic.MAX: float(self.max[i]),
                Statistic.MED: float(self.med[i]), Statistic.AVG: float(self.avg[i]),
                Statistic.STD: float(self.std[i]), Statistic.NUM: int(self.num[i])}

    def __iter__(self) -> Iterator[str]:
        return iter(self.names)

    def __len__(self) -> int:
        return len(self.names)

    def __contains__(self, name) -> bool:
        return name in self._index

    def select(self, keep: np.ndarray) -> "KernelSummaries":
        idx = np.nonzero(keep)[0]
        return KernelSummaries([self.names[i] for i in idx], self.num[idx], self.min[idx],
                               self.max[idx], self.med[idx], self.avg[idx], self.std[idx])

    def columns(self):
        """(MED f64, AVG f64, NUM i64) as the scoring kernels consume them."""
        return self.med.astype(np.float64), self.avg.astype(np.float64), self.num

    def __repr__(self):
        return f"KernelSummaries({len(self)} kernels)"


def columns_of(summaries: Mapping[str, Mapping]) -> tuple:
    """(MED f64, AVG f64, NUM i64) columns of any name -> {Statistic: value} mapping."""
    if isinstance(summaries, KernelSummaries):
        return summaries.columns()
    n = len(summaries)
    vals = summaries.values()
    # C-level item getters over the values (no Python frame per summary)
    return (np.fromiter(map(_GET_MED, vals), np.float64, n),
            np.fromiter(map(_GET_AVG, vals), np.float64, n),
            np.fromiter(map(_GET_NUM, vals), np.int64, n))


_GET_MED, _GET_AVG, _GET_NUM = (operator.itemgetter(k) for k in (Statistic.MED, Statistic.AVG,
                                                                  Statistic.NUM))
