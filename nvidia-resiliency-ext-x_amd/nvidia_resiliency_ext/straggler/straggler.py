"""Detector facade (drop-in for straggler/straggler.py:34-408).

Same classmethod API: initialize / shutdown / detection_section / wrap_callables /
restore_original_callables / generate_report / generate_report_if_interval_elapsed /
is_interval_elapsed.  Kernel durations go to the device-resident record log of the
nvrx profiler (cupti.py); at report time the section and kernel statistics and all
scores are computed by HIP kernels (nvrx_section_stats, nvrx_profiler_get_stats,
ReportGenerator).
"""
from __future__ import annotations

import collections
import dataclasses
import functools
import inspect
import socket
import time
from collections.abc import Callable
from contextlib import contextmanager
from typing import Any, Deque, Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from . import ops
from .cupti import CuptiManager
from .interval_tracker import ReportIntervalTracker
from .reporting import ReportGenerator
from .statistics import Statistic


@dataclasses.dataclass(frozen=True)
class CallableId:
    """A callable to wrap in a detection section: ``getattr(obj, name)`` (straggler.py:34-62)."""

    obj: object
    name: str
    arg_filter_fn: Optional[Callable[[inspect.BoundArguments], bool]] = None
    extra_args_fn: Optional[Callable[[inspect.BoundArguments], dict]] = None
    ignored_args: Optional[tuple] = None

    def __str__(self):
        if inspect.ismodule(self.obj):
            obj_name = self.obj.__name__
        elif inspect.isclass(self.obj):
            obj_name = f"{self.obj.__module__}.{self.obj.__name__}"
        elif hasattr(self.obj, "__class__"):
            obj_name = getattr(self.obj.__class__, "__name__", self.obj)
        else:
            obj_name = getattr(self.obj, "__name__", self.obj)
        return f"{obj_name}.{self.name}"


@dataclasses.dataclass
class CustomSection:
    """A user-defined section: CPU elapsed times (ms) of its profiled entries."""

    name: str
    location: str
    total_entry_cnt: int = 0
    max_elapseds_len: int = 8 * 1024
    cpu_elapsed_times: Deque[float] = dataclasses.field(
        default_factory=lambda: collections.deque(maxlen=CustomSection.max_elapseds_len))


class Detector:
    """Straggler detection entry point; class methods only (not instantiable)."""

    initialized: bool = False
    scores_to_compute: Sequence[str]
    gather_on_rank0: bool
    profiling_interval: int
    report_time_interval: float
    custom_sections: Dict[str, CustomSection]
    cupti_manager: CuptiManager
    reporter: ReportGenerator
    report_interval_tracker: ReportIntervalTracker
    original_callables: Optional[Dict[CallableId, Any]]

    def __new__(cls):
        raise RuntimeError(f"class {cls.__name__} should not be instantiated")

    @classmethod
    def initialize(cls, scores_to_compute: Union[Sequence[str], str] = "all",
                   gather_on_rank0: bool = True, profiling_interval: int = 1,
                   report_time_interval: float = 60, node_name: Optional[str] = None):
        assert not cls.initialized
        cls.scores_to_compute = (["relative_perf_scores", "individual_perf_scores"]
                                 if str(scores_to_compute) == "all" else scores_to_compute)
        cls.gather_on_rank0 = gather_on_rank0
        cls.profiling_interval = profiling_interval
        cls.custom_sections = {}
        cls.cupti_manager = CuptiManager(statsMaxLenPerKernel=8 * 1024)
        cls.cupti_manager.initialize()
        cls.reporter = ReportGenerator(scores_to_compute=cls.scores_to_compute,
                                       gather_on_rank0=gather_on_rank0,
                                       node_name=(node_name if node_name else socket.gethostname()))
        cls.report_interval_tracker = ReportIntervalTracker(time_interval=report_time_interval,
                                                            profiling_interval=profiling_interval)
        cls.initialized = True
        cls.original_callables = {}

    @classmethod
    def shutdown(cls):
        cls.cupti_manager.shutdown()
        cls.restore_original_callables()
        cls.cupti_manager = None
        cls.initialized = False

    @classmethod
    def _get_section_summaries(cls):
        """Section timing statistics, on the device (nvrx_section_stats)."""
        names: List[str] = []
        chunks: List[np.ndarray] = []
        for key, section in cls.custom_sections.items():
            assert key == section.name
            if len(section.cpu_elapsed_times) == 0:
                continue
            names.append(key)
            chunks.append(np.fromiter(section.cpu_elapsed_times, dtype=np.float64))
        if not names:
            return {}
        off = np.zeros(len(chunks) + 1, np.int64)
        off[1:] = np.cumsum([len(c) for c in chunks])
        dev = cls.reporter._dev()
        # pinned staging both ways and one synchronisation (four blocking round trips before:
        # ~0.2-0.4 ms of a live report, tools/probe_report_breakdown.py)
        pin = dev.type == "cuda"
        vals_h = torch.from_numpy(np.concatenate(chunks))
        off_h = torch.from_numpy(off)
        if pin:
            vals_h, off_h = vals_h.pin_memory(), off_h.pin_memory()
        num_d, out_d = ops.section_stats(vals_h.to(dev, non_blocking=pin), off_h.to(dev, non_blocking=pin),
                                         max(len(c) for c in chunks))
        num_t = torch.empty(num_d.shape, dtype=num_d.dtype, pin_memory=pin)
        out_t = torch.empty(out_d.shape, dtype=out_d.dtype, pin_memory=pin)
        num_t.copy_(num_d, non_blocking=pin)
        out_t.copy_(out_d, non_blocking=pin)
        if pin:
            torch.cuda.current_stream(dev).synchronize()
        num, out = num_t.numpy(), out_t.numpy()
        return {n: {Statistic.MIN: float(out[0, i]), Statistic.MAX: float(out[1, i]),
                    Statistic.MED: float(out[2, i]), Statistic.AVG: float(out[3, i]),
                    Statistic.STD: float(out[4, i]), Statistic.NUM: int(num[i])}
                for i, n in enumerate(names)}

    @classmethod
    def _get_kernel_summaries(cls):
        """Per-kernel statistics from the device record log (name-sorted mapping)."""
        return cls.cupti_manager.get_results_columns()

    @classmethod
    def _reset_sections_elapseds(cls):
        for section in cls.custom_sections.values():
            section.cpu_elapsed_times.clear()

    @classmethod
    def generate_report(cls):
        """ReportGenerator.generate_report over the current summaries, then reset them
        (straggler.py:227-245)."""
        assert cls.initialized
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        section_summaries = cls._get_section_summaries()
        kernel_summaries = cls._get_kernel_summaries()
        report = cls.reporter.generate_report(section_summaries, kernel_summaries)
        cls._reset_sections_elapseds()
        cls.cupti_manager.reset_results()
        return report

    @classmethod
    def generate_report_if_interval_elapsed(cls):
        assert cls.initialized
        cls.report_interval_tracker.iter_increase()
        if cls.report_interval_tracker.is_interval_elapsed():
            return cls.generate_report()
        return None

    @classmethod
    def is_interval_elapsed(cls) -> bool:
        return cls.report_interval_tracker.is_interval_elapsed()

    @staticmethod
    def _get_this_context_block_location() -> str:
        frame = inspect.currentframe().f_back.f_back.f_back  # type: ignore
        return f"{frame.f_code.co_filename}:{frame.f_lineno}"  # type: ignore

    @classmethod
    def _ensure_section_name_is_valid(cls, name, location):
        if name in cls.custom_sections and location != cls.custom_sections[name].location:
            raise ValueError(f"Section name '{name}' is already used at: "
                             f"{cls.custom_sections[name].location}")

    @classmethod
    @contextmanager
    def detection_section(cls, name: Optional[str] = None, profile_cuda: bool = True):
        """Monitor a block of user code: CPU time always, GPU kernels when profile_cuda.
        Only every `profiling_interval`-th entry of a section is profiled."""
        if not cls.initialized:
            raise RuntimeError("Detector is not initialized.")
        location = Detector._get_this_context_block_location()
        if name is None:
            name = location
        section = cls.custom_sections.get(name)
        if section is None:
            section = CustomSection(name=name, location=location)
            cls.custom_sections[name] = section
        profile_this_entry = (section.total_entry_cnt % cls.profiling_interval) == 0
        section.total_entry_cnt += 1
        if profile_this_entry:
            if profile_cuda:
                cls.cupti_manager.start_profiling()
            t0 = time.perf_counter_ns()
            try:
                yield
            except BaseException:
                if profile_cuda:
                    cls.cupti_manager.stop_profiling()
                raise
            section.cpu_elapsed_times.append((time.perf_counter_ns() - t0) * 1e-6)
            if profile_cuda:
                cls.cupti_manager.stop_profiling()
        else:
            yield

    @classmethod
    def _build_wrapper(cls, fn, callable_id, profile_cuda: bool = True):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            with cls.detection_section(name=str(callable_id), profile_cuda=profile_cuda):
                return fn(*args, **kwargs)

        return wrapper

    @classmethod
    def wrap_callables(cls, callable_ids: List[CallableId], profile_cuda: bool = True):
        cls.original_callables = {}
        for cid in callable_ids:
            original = getattr(cid.obj, cid.name)
            cls.original_callables[cid] = original
            setattr(cid.obj, cid.name, cls._build_wrapper(original, cid, profile_cuda=profile_cuda))

    @classmethod
    def restore_original_callables(cls):
        if cls.original_callables:
            for cid, original in cls.original_callables.items():
                setattr(cid.obj, cid.name, original)
