"""ctypes binding of libnvrx_hip.so, the C ABI declared in include/nvrx_straggler.h.

The shared library holds the hand-written gfx950 kernels of the scoring path.  There is
no CPU fallback: if the library is missing or fails to load, every entry point raises.
Device arrays are passed as raw pointers (torch tensors' ``data_ptr()``), streams as the
HIP stream handle (``torch.cuda.current_stream().cuda_stream``).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

LIB_NAME = "libnvrx_hip.so"
ABI_VERSION = 6  # include/nvrx_straggler.h NVRX_ABI_VERSION
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

NVRX_OK = 0
NVRX_ERR_INVALID = -1
NVRX_ERR_HIP = -2
NVRX_ERR_STATE = -3
NVRX_ERR_SINGLETON = -4
NVRX_ERR_NOMEM = -5

NVRX_STATS_FAST = 0
NVRX_STATS_EXACT = 1
NVRX_STATS_COLREF_READY = 0x10
NVRX_MAX_SEGMENT = 1 << 30  # rings above 32,768 samples sort in device scratch

P = ctypes.c_void_p
i32 = ctypes.c_int32
i64 = ctypes.c_int64
u32 = ctypes.c_uint32
f64 = ctypes.c_double


class StatsSoA(ctypes.Structure):
    _fields_ = [("num", P), ("min", P), ("max", P), ("med", P), ("avg", P), ("std", P)]


class ScoreArgs(ctypes.Structure):
    _fields_ = [
        ("R", i64), ("K", i64), ("value_f64", i32),
        ("num", P), ("med", P), ("avg", P), ("col_valid", P),
        ("ref", P), ("ref_index", P), ("ref_missing", P),
        ("hist", P), ("hist_index", P), ("hist_stride", i64),
        ("partials", P), ("err", P),
        ("round_f32", i32), ("thr_rel", f64), ("thr_ind", f64),
        ("gpu_rel", P), ("gpu_ind", P), ("strag_rel", P), ("strag_ind", P),
        ("done", P), ("reset_col_ref", P), ("reset_ncols", i64),
    ]


class Record(ctypes.Structure):
    _fields_ = [("slot", u32), ("ns", u32)]


class CaptureCounters(ctypes.Structure):
    _fields_ = [("callbacks", i64), ("headers", i64), ("dispatches", i64),
                ("callback_ns", i64), ("flushes", i64), ("flush_ns", i64), ("runtime_kernels", i64),
                ("own_kernels", i64), ("flush_first_cb_ns", i64), ("flush_callbacks", i64),
                ("flush_tail_ns", i64), ("enqueues_counted", i64), ("counted_flushes", i64),
                ("quiet_flushes", i64), ("flush_timeouts", i64), ("owed_abandoned", i64),
                ("delivery", i32), ("marking", i32), ("queues", i64), ("ring_records", i64),
                ("pool_signals", i64), ("chained_signals", i64), ("ring_anomalies", i64),
                ("dropped", i64)]


class ProfilerConfig(ctypes.Structure):
    _fields_ = [
        ("buffer_size", i64), ("num_buffers", i64), ("stats_max_len_per_kernel", i64),
        ("device", i32), ("mode", i32),
    ]


# name -> (restype, argtypes); every symbol the header declares
SIGNATURES = {
    "nvrx_last_error": (ctypes.c_char_p, []),
    "nvrx_capture_configure": (ctypes.c_int, []),
    "nvrx_abi_version": (ctypes.c_int, []),
    "nvrx_duration_key": (u32, [ctypes.c_uint64]),
    "nvrx_encode_ns_u32": (ctypes.c_int, [P, i64, P]),
    "nvrx_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "nvrx_sync": (ctypes.c_int, [P]),
    "nvrx_segment_stats_strided": (ctypes.c_int, [P, i64, i64, i64, i64, i64, i32,
                                                  ctypes.POINTER(StatsSoA), P, i64, P]),
    "nvrx_segment_stats_ragged": (ctypes.c_int, [P, P, P, i64, i64, i64, i32, i32,
                                                 ctypes.POINTER(StatsSoA), P, i64, P]),
    "nvrx_kernel_ref": (ctypes.c_int, [P, P, i64, i64, P, P, P]),
    "nvrx_pack_min_times": (ctypes.c_int, [P, P, i64, P, i64, P]),
    "nvrx_scores": (ctypes.c_int, [ctypes.POINTER(ScoreArgs), P]),
    "nvrx_finalize_scores": (ctypes.c_int, [P, i64, i64, i32, f64, f64, P, P, P, P, P, P]),
    "nvrx_section_scores": (ctypes.c_int, [P, P, i64, i64, P, P, P, P, i32, P, P, P, P]),
    "nvrx_stragglers": (ctypes.c_int, [P, i64, f64, P, P]),
    "nvrx_section_stats": (ctypes.c_int, [P, P, i64, i64, P, P, P, P, P, P, P]),
    "nvrx_records_bucket_capacity": (i64, [i64, i64, i64]),
    "nvrx_records_stats": (ctypes.c_int, [P, P, i64, i64, i64, i32, i64, P, P, P, P,
                                          ctypes.POINTER(StatsSoA), P, P]),
    "nvrx_records_bucket": (ctypes.c_int, [P, P, i64, i64, i64, P, P, P, P, P]),
    "nvrx_records_max_slots": (i64, []),
    "nvrx_profiler_create": (ctypes.c_int, [ctypes.POINTER(ProfilerConfig), ctypes.POINTER(P)]),
    "nvrx_profiler_destroy": (ctypes.c_int, [P]),
    "nvrx_profiler_initialize": (ctypes.c_int, [P]),
    "nvrx_profiler_shutdown": (ctypes.c_int, [P]),
    "nvrx_profiler_start": (ctypes.c_int, [P]),
    "nvrx_profiler_stop": (ctypes.c_int, [P]),
    "nvrx_profiler_reset": (ctypes.c_int, [P]),
    "nvrx_profiler_register_kernel": (ctypes.c_int, [P, ctypes.c_char_p, ctypes.POINTER(u32)]),
    "nvrx_profiler_push": (ctypes.c_int, [P, P, i64]),
    "nvrx_profiler_ingest": (ctypes.c_int, [P, P, i64, ctypes.c_uint64, P]),
    "nvrx_profiler_generation": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_uint64)]),
    "nvrx_profiler_saturated": (ctypes.c_int, [P, ctypes.POINTER(i64)]),
    "nvrx_profiler_get_stats": (ctypes.c_int, [P, i64, ctypes.POINTER(i64), P, P, P, P, P, P, P]),
    "nvrx_profiler_kernel_name": (ctypes.c_int, [P, u32, ctypes.c_char_p, i64]),
    "nvrx_profiler_get_records": (ctypes.c_int, [P, i64, ctypes.POINTER(i64), P]),
    "nvrx_profiler_capture_available": (ctypes.c_int, []),
    "nvrx_capture_flush": (ctypes.c_int, []),
    "nvrx_capture_stats": (ctypes.c_int, [ctypes.POINTER(CaptureCounters)]),
}

_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


class NativeLibraryError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load libnvrx_hip.so (once).  Raises NativeLibraryError if it is missing: the HIP
    path is the product; nothing falls back to the CPU."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f"{LIB_NAME} not found at {LIB_PATH}; build it with "
                f"`make -C nvidia-resiliency-ext-x_amd/csrc` (hipcc --offload-arch=gfx950)")
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.nvrx_abi_version() != ABI_VERSION:
            raise NativeLibraryError("libnvrx_hip.so ABI version mismatch")
        _lib = L
        return _lib


def check(rc: int, what: str = "") -> None:
    """Map a status code to the reference's error behaviour (RuntimeError)."""
    if rc != NVRX_OK:
        msg = lib().nvrx_last_error().decode(errors="replace")
        raise RuntimeError(f"{what}: {msg}" if what else msg)


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


def ptr(t) -> Optional[int]:
    """Device (or host) pointer of a tensor / numpy array; None passes NULL."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return t.data_ptr()
    return t.ctypes.data


def stream_handle(stream=None) -> Optional[int]:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


KEY_WIDE = 0xE0000000
KEY_WIDE_F32BITS = 0x4F600000
KEY_MAX = 0xF0200000  # key of f32(2^64 - 1); larger u32 values come from no u64 duration


def duration_keys(ns):
    """u64 ns (array-like) -> u32 duration keys (include/nvrx_straggler.h): the ns below
    0xE0000000 (3.76 s), else 0xE0000000 + bits(f32(ns)) - bits(f32(0xE0000000)) -- exactly
    the f32(end - start) CuptiProfiler.cpp:187 keeps.  Vectorised twin of nvrx_duration_key."""
    import numpy as np

    ns = np.asarray(ns, dtype=np.uint64)
    f = ns.astype(np.float32).view(np.uint32).astype(np.uint64)
    wide = np.uint64(KEY_WIDE) + f - np.uint64(KEY_WIDE_F32BITS)
    return np.where(ns < KEY_WIDE, ns, wide).astype(np.uint32)


def require_device(t, name: str = "tensor") -> None:
    """Kernels only ever see device memory: a CPU tensor is a caller bug, raised loudly."""
    if t is not None and (not hasattr(t, "is_cuda") or not t.is_cuda):
        raise ValueError(f"{name} must be a device (HIP) tensor")
