"""Kernel-duration capture manager (drop-in for straggler/cupti.py:19-95).

``KernelProfiler`` replaces the pybind11 ``nvrx_cupti_module.CuptiProfiler``
(cupti_module_py.cpp:33-54) with the nvrx_profiler handle of libnvrx_hip.so: records are
kept as a device-resident log in HBM and reduced to per-kernel statistics by the HIP
kernels at get_stats time (only the last ``statsMaxLenPerKernel`` records of every kernel
count, as the reference's rings keep them).  Records enter through the live capture
(capture_queue.cpp / capture.cpp: every kernel enqueued while the profiler is started, once it
completed, keyed like CuptiProfiler.cpp:182-185) and through ``push`` / ``ingest`` (external
tracers, tests).  rocprofiler-sdk tools configure when the ROCm runtime initialises, so capture
needs ``enable_capture()`` (or the first ``KernelProfiler``) before the process's first
HIP call -- the same constraint CUPTI activity tracing has on its first CUDA context.

``CuptiManager`` keeps the reference's thread-safe, refcounted start/stop semantics.
"""
from __future__ import annotations

import ctypes
import os
import threading
import warnings
from typing import Dict, Iterable, Optional, Sequence

import numpy as np

from . import _native as N
from .summaries import KernelSummaries


class KernelStats:
    """Per-kernel statistics as the reference module exposes them (CuptiProfiler.h:39-45)."""

    __slots__ = ("num_calls", "min", "max", "median", "avg", "stddev")

    def __init__(self, num_calls=0, mn=float("nan"), mx=float("nan"), median=float("nan"),
                 avg=float("nan"), stddev=float("nan")):
        self.num_calls, self.min, self.max = num_calls, mn, mx
        self.median, self.avg, self.stddev = median, avg, stddev

    def __str__(self):
        return (f" num calls: {self.num_calls}, min: {self.min}, max: {self.max}, median: "
                f"{self.median}, avg: {self.avg}, stddev: {self.stddev}")


_capture_state: Optional[bool] = None
_tool_env: list = []  # environment variables rocprofiler-sdk's configuration added


def _c_environ() -> Dict[str, str]:
    """The process environment as the C library sees it (os.environ is a start-up snapshot)."""
    libc = ctypes.CDLL(None)
    env = ctypes.POINTER(ctypes.c_char_p).in_dll(libc, "environ")
    out, i = {}, 0
    while env[i]:
        k, _, v = env[i].decode(errors="replace").partition("=")
        out[k] = v
        i += 1
    return out


def _scrub_tool_env() -> None:
    """rocprofiler_force_configure exports ROCPROFILER_REGISTER_FORCE_LOAD=1 (and GLOG_*)
    into this process's environment; inherited by a child process (torchrun workers, test
    subprocesses) it keeps that child from configuring its own capture.  Once this process's
    runtime has initialised -- or configuration was refused -- they are removed again."""
    while _tool_env:
        k = _tool_env.pop()
        os.environ.pop(k, None)
        os.unsetenv(k)


def enable_capture() -> bool:
    """Register the rocprofiler-sdk kernel-dispatch tool (idempotent).  Returns False when
    the ROCm runtime of this process is already initialised (capture then unavailable;
    records can still be pushed).  NVRX_CAPTURE=0 disables it."""
    global _capture_state
    if _capture_state is None:
        if os.environ.get("NVRX_CAPTURE", "1") == "0":
            _capture_state = False
        else:
            before = _c_environ()
            _capture_state = N.lib().nvrx_capture_configure() == 0
            _tool_env.extend(k for k in _c_environ() if k not in before)
            if not _capture_state:
                _scrub_tool_env()
    return _capture_state


def capture_available() -> bool:
    """True once the runtime has initialised with the capture tool configured."""
    return bool(N.lib().nvrx_profiler_capture_available())


class KernelProfiler:
    """nvrx_cupti_module.CuptiProfiler(bufferSize, numBuffers, statsMaxLenPerKernel)."""

    def __init__(self, bufferSize: int = 1024 * 1024 * 8, numBuffers: int = 8,
                 statsMaxLenPerKernel: int = 1024, device: Optional[int] = None,
                 exact: bool = True, capture: bool = True):
        if capture and not enable_capture() and _capture_state is False and \
                os.environ.get("NVRX_CAPTURE", "1") != "0":
            warnings.warn("kernel-dispatch capture unavailable: the ROCm runtime was initialised "
                          "before the straggler profiler (call nvidia_resiliency_ext.straggler."
                          "cupti.enable_capture() first); only pushed records are profiled",
                          RuntimeWarning, stacklevel=2)
        if device is None:
            import torch

            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        cfg = N.ProfilerConfig(bufferSize, numBuffers, statsMaxLenPerKernel, int(device),
                               N.NVRX_STATS_EXACT if exact else N.NVRX_STATS_FAST)
        h = ctypes.c_void_p()
        N.check(N.lib().nvrx_profiler_create(ctypes.byref(cfg), ctypes.byref(h)),
                "CuptiProfiler")
        self._h = h
        _scrub_tool_env()  # the runtime (and the tool, if configured) is initialised now
        self._slot_of: Dict[str, int] = {}
        self._names: list = []

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                N.lib().nvrx_profiler_destroy(h)
            except Exception:
                pass
            self._h = None

    def close(self):
        self.__del__()

    def initialize(self):
        N.call("nvrx_profiler_initialize", self._h)

    def shutdown(self):
        N.call("nvrx_profiler_shutdown", self._h)

    def start(self):
        N.call("nvrx_profiler_start", self._h)

    def stop(self):
        N.call("nvrx_profiler_stop", self._h)

    def reset(self):
        """Flush, then clear every kernel's records AND forget the kernels (as the
        reference's reset clears its per-kernel map, CuptiProfiler.cpp:148-152): slots are
        renumbered from 0 in the next interval, so the name caches here are dropped too."""
        N.call("nvrx_profiler_reset", self._h)
        self._slot_of.clear()
        self._names.clear()

    def register_kernel(self, name: str) -> int:
        s = self._slot_of.get(name)
        if s is None:
            out = ctypes.c_uint32()
            N.call("nvrx_profiler_register_kernel", self._h, name.encode(), ctypes.byref(out))
            s = int(out.value)
            self._slot_of[name] = s
            while len(self._names) <= s:
                self._names.append(None)
            self._names[s] = name
        return s

    def push(self, name: str, durations_ns: Iterable[int]) -> None:
        """Append kernel executions of `name` (durations in ns, push order)."""
        d = np.asarray(list(durations_ns) if not isinstance(durations_ns, np.ndarray)
                       else durations_ns, dtype=np.uint64)
        self.push_slots(np.full(d.size, self.register_kernel(name), np.uint32), d)

    def push_slots(self, slots: np.ndarray, durations_ns: np.ndarray) -> None:
        """Records of registered slots (valid until the next reset), durations in ns (any
        u64): stored as duration keys (_native.duration_keys), which keep exactly the f32(ns)
        the reference's (end - start) / 1000.0f keeps (CuptiProfiler.cpp:187)."""
        recs = np.empty((len(slots), 2), dtype=np.uint32)
        recs[:, 0] = slots
        recs[:, 1] = N.duration_keys(durations_ns)
        N.call("nvrx_profiler_push", self._h, recs.ctypes.data, len(slots))

    @property
    def generation(self) -> int:
        """Slot-numbering generation (bumped by every reset): pass the value read after
        registering to ``ingest`` so records built from slots of an earlier interval raise."""
        g = ctypes.c_uint64()
        N.call("nvrx_profiler_generation", self._h, ctypes.byref(g))
        return int(g.value)

    def ingest(self, records, stream=None, *, generation: int) -> None:
        """Append DEVICE records: an int32/uint32 tensor [n, 2] of {slot, ns} (registered slots,
        push order) resident on the profiler's device, copied into the device record log on
        `stream` (default: the current stream) -- no host round trip.  ``generation`` (required):
        the ``self.generation`` read after registering the slots; a reset since then raises
        RuntimeError instead of filing the records under slots that now name other kernels.
        Records of unregistered slots are dropped."""
        import torch

        N.require_device(records, "records")
        if records.dim() != 2 or records.shape[1] != 2 or records.element_size() != 4:
            raise ValueError("records must be a [n, 2] tensor of 32-bit {slot, ns}")
        records = records.contiguous()
        N.call("nvrx_profiler_ingest", self._h, records.data_ptr(), records.shape[0], int(generation),
               N.stream_handle(stream if stream is not None else torch.cuda.current_stream(records.device)))

    def saturated(self) -> int:
        """Durations of 3.76 s or more (wide duration keys; nothing lost) since the last
        reset -- a count of hung or very long kernels."""
        c = ctypes.c_int64()
        N.call("nvrx_profiler_saturated", self._h, ctypes.byref(c))
        return int(c.value)

    def get_stats_columns(self) -> KernelSummaries:
        """Per-kernel statistics (HIP) as columns, sorted by composite kernel name.  One
        device computation: the size query's result is cached by the library and the copying
        call reuses it (recomputed only if records arrived in between, hence the loop)."""
        L = N.lib()
        count = ctypes.c_int64()
        N.call("nvrx_profiler_get_stats", self._h, 0, ctypes.byref(count), None, None, None,
               None, None, None, None)
        p = lambda a: a.ctypes.data  # noqa: E731
        while True:
            n = int(count.value)
            slots = np.empty(n, np.uint32)
            num = np.empty(n, np.int32)
            cols = [np.empty(n, np.float32) for _ in range(5)]
            N.check(L.nvrx_profiler_get_stats(self._h, n, ctypes.byref(count), p(slots), p(num),
                                              *(p(c) for c in cols)), "get_stats")
            if int(count.value) <= n:
                break
        # the count may also have shrunk (a reset from another thread): only count.value
        # entries were written
        m = int(count.value)
        slots, num, cols = slots[:m], num[:m], [c[:m] for c in cols]
        names = [self._name_of(int(s)) for s in slots]
        return KernelSummaries(names, num, *cols)

    def get_records(self):
        """(slots u32, ns u32) of the device record log since the last reset, push order
        (nvrx_profiler_get_records) -- what the statistics are computed from."""
        count = ctypes.c_int64()
        N.call("nvrx_profiler_get_records", self._h, 0, ctypes.byref(count), None)
        recs = np.empty((int(count.value), 2), np.uint32)
        N.call("nvrx_profiler_get_records", self._h, len(recs), ctypes.byref(count),
               recs.ctypes.data)
        return recs[:, 0].copy(), recs[:, 1].copy()

    def flush_capture(self):
        """Deliver completed dispatch records now (cuptiActivityFlushAll)."""
        N.call("nvrx_capture_flush")

    def name_of(self, slot: int) -> str:
        """Composite kernel name of a record slot."""
        return self._name_of(int(slot))

    def _name_of(self, s: int) -> str:
        """Slot -> composite name; slots created by the capture callback are fetched once."""
        if s < len(self._names) and self._names[s] is not None:
            return self._names[s]
        buf = ctypes.create_string_buffer(8192)
        N.call("nvrx_profiler_kernel_name", self._h, s, buf, len(buf))
        name = buf.value.decode()
        while len(self._names) <= s:
            self._names.append(None)
        self._names[s] = name
        self._slot_of[name] = s
        return name

    @property
    def capture(self) -> bool:
        return capture_available()

    def get_stats(self) -> Dict[str, KernelStats]:
        ks = self.get_stats_columns()
        return {n: KernelStats(int(ks.num[i]), float(ks.min[i]), float(ks.max[i]),
                               float(ks.med[i]), float(ks.avg[i]), float(ks.std[i]))
                for i, n in enumerate(ks.names)}


class CuptiManager:
    """Thread-safe access to the profiler with a usage counter of active profiling runs."""

    def __init__(self, bufferSize=1_000_000, numBuffers=8, statsMaxLenPerKernel=4096):
        self.cupti_ext = KernelProfiler(bufferSize=bufferSize, numBuffers=numBuffers,
                                        statsMaxLenPerKernel=statsMaxLenPerKernel)
        self.is_initialized = False
        self.started_cnt = 0
        self.lock = threading.Lock()

    def _ensure_initialized(self):
        if not self.is_initialized:
            raise RuntimeError("CuptiManager was not initialized")

    def initialize(self):
        with self.lock:
            self.cupti_ext.initialize()
            self.is_initialized = True

    def shutdown(self):
        with self.lock:
            self.cupti_ext.shutdown()
            self.is_initialized = False
            self.started_cnt = 0
            self.cupti_ext.close()

    def start_profiling(self):
        with self.lock:
            self._ensure_initialized()
            if self.started_cnt == 0:
                self.cupti_ext.start()
            self.started_cnt += 1

    def stop_profiling(self):
        with self.lock:
            self._ensure_initialized()
            if self.started_cnt > 0:
                self.started_cnt -= 1
                if self.started_cnt == 0:
                    self.cupti_ext.stop()
            else:
                raise RuntimeError("No active profiling run.")

    def get_results(self):
        with self.lock:
            self._ensure_initialized()
            return self.cupti_ext.get_stats().copy()

    def get_results_columns(self) -> KernelSummaries:
        with self.lock:
            self._ensure_initialized()
            return self.cupti_ext.get_stats_columns()

    def reset_results(self):
        with self.lock:
            self._ensure_initialized()
            self.cupti_ext.reset()

    def push(self, name: str, durations_ns: Sequence[int]):
        """Feed kernel executions (e.g. from an external tracer) into the active run."""
        with self.lock:
            self.cupti_ext.push(name, durations_ns)

    def register_kernel(self, name: str) -> int:
        """Slot of a composite kernel name for ingest() records (valid until the next reset)."""
        with self.lock:
            return self.cupti_ext.register_kernel(name)

    @property
    def generation(self) -> int:
        """Slot-numbering generation to pass to ingest() (read after register_kernel)."""
        with self.lock:
            return self.cupti_ext.generation

    def ingest(self, records, stream=None, *, generation: int):
        """Device-resident {slot, ns} records from an external tracer into the active run."""
        with self.lock:
            self.cupti_ext.ingest(records, stream, generation=generation)
