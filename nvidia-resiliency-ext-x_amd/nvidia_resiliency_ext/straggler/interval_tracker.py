"""Report interval estimation (reference: straggler/interval_tracker.py:25-83).

After INTERVAL_ESTIMATION_ITERS timed iterations the report interval in iterations is
time_interval / median(step time), MAX-reduced over ranks and never below the profiling
interval; the interval has elapsed whenever current_iter % iter_interval == 0.
"""
import dataclasses
import time
from typing import List, Optional

import torch

from . import dist_utils


@dataclasses.dataclass
class ReportIntervalTracker:
    INTERVAL_ESTIMATION_ITERS: int = 16
    time_interval: float = 60.0
    current_iter: int = 0
    iter_interval: Optional[int] = None
    prev_iter_start_time: Optional[float] = None
    step_times: List[float] = dataclasses.field(default_factory=list)
    profiling_interval: int = 1

    def _gather_report_interval(self, group: Optional[torch.distributed.ProcessGroup] = None):
        assert self.iter_interval is None, "Report iteration interval has already been gathered."
        median_step_time = torch.median(torch.tensor(self.step_times, dtype=torch.float32))
        gathered = (self.time_interval / median_step_time).to(dist_utils.get_device_for_backend(group))
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            torch.distributed.all_reduce(gathered, op=torch.distributed.ReduceOp.MAX, group=group)
        self.iter_interval = int(max(gathered.item(), self.profiling_interval))

    def iter_increase(self):
        self.current_iter += 1
        if self.iter_interval is None:
            now = time.monotonic()
            if self.prev_iter_start_time is not None:
                self.step_times.append(now - self.prev_iter_start_time)
                if len(self.step_times) == self.INTERVAL_ESTIMATION_ITERS:
                    self._gather_report_interval()
                    self.step_times.clear()
            self.prev_iter_start_time = time.monotonic()

    def is_interval_elapsed(self) -> bool:
        return self.iter_interval is not None and self.current_iter % self.iter_interval == 0
