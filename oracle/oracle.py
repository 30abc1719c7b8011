"""TEST INFRASTRUCTURE ONLY -- ctypes front end of the C oracle (oracle/nvrx_oracle.c).

The oracle is the parity checker for the HIP product path and the timed host-CPU
Reporter of bench.py (cpu_baseline.kind = "port").  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product package never does.

Pinning: tests/test_oracle_golden.py checks every function here against
tests/golden/*.json, which tests/golden/make_golden.py produced from the reference
itself (computeStats compiled from /root/reference by oracle/Makefile; the
reference ReportGenerator run on gloo).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

SEED = 0x5EED
SEED2 = 0xBA5E


class KStats(ctypes.Structure):
    _fields_ = [
        ("num_calls", ctypes.c_int32),
        ("min", ctypes.c_float),
        ("max", ctypes.c_float),
        ("median", ctypes.c_float),
        ("avg", ctypes.c_float),
        ("stddev", ctypes.c_float),
    ]


def build() -> str:
    """Compile liboracle.so (gcc) if missing or stale."""
    srcs = [os.path.join(_HERE, f) for f in ("nvrx_oracle.c", "baseline.cpp")]
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < max(map(os.path.getmtime, srcs)):
        subprocess.check_call(["make", "-s", "-C", _HERE, "all"])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i64 = ctypes.c_int64
        u64 = ctypes.c_uint64
        L.oracle_splitmix64.restype = u64
        L.oracle_splitmix64.argtypes = [u64]
        L.oracle_base_ns.restype = u64
        L.oracle_base_ns.argtypes = [u64, u64]
        L.oracle_sample_ns.restype = ctypes.c_uint32
        L.oracle_sample_ns.argtypes = [u64, u64, u64, u64, u64, u64, u64, ctypes.c_int]
        L.oracle_gen_matrix.argtypes = [P, i64, i64, i64, u64, u64, P]
        L.oracle_ns_to_us.restype = ctypes.c_float
        L.oracle_ns_to_us.argtypes = [u64]
        L.oracle_compute_stats.argtypes = [P, i64, ctypes.POINTER(KStats)]
        L.oracle_ring_linearize.restype = i64
        L.oracle_ring_linearize.argtypes = [P, i64, i64, P]
        L.oracle_matrix_stats.argtypes = [P, i64, i64, i64, i64, i64, P, P, P, P, P, P, ctypes.c_int]
        L.oracle_matrix_stats_route.argtypes = [P, i64, i64, i64, i64, i64, P, P, P, P, P, P,
                                                ctypes.c_int, ctypes.c_int]
        L.oracle_baseline_matrix_stats.argtypes = [P, i64, i64, i64, i64, i64, P, P, P, P, P, P,
                                                   ctypes.c_int]
        L.oracle_baseline_records_stats.argtypes = [P, P, i64, i64, i64, P, P, P, P, P, P,
                                                    ctypes.c_int]
        L.oracle_records_stats.argtypes = [P, P, i64, i64, i64, P, P, P, P, P, P, ctypes.c_int]
        L.oracle_duration_key.argtypes = [u64]
        L.oracle_duration_key.restype = ctypes.c_uint32
        L.oracle_key_to_us.argtypes = [ctypes.c_uint32]
        L.oracle_key_to_us.restype = ctypes.c_float
        L.oracle_records_moments.argtypes = [P, P, i64, i64, i64, P, P, ctypes.c_int]
        L.oracle_kernel_ref.argtypes = [P, P, i64, i64, P]
        L.oracle_scores.argtypes = [P, P, P, i64, i64, P, P, P, P, P]
        L.oracle_score_partials.argtypes = [P, P, P, i64, i64, P, P, P, P]
        L.oracle_stragglers.restype = i64
        L.oracle_stragglers.argtypes = [P, i64, ctypes.c_double, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


# ---------------------------------------------------------------- generator
def splitmix64(x: int) -> int:
    return int(lib().oracle_splitmix64(x & 0xFFFFFFFFFFFFFFFF))


def straggler_ranks(R: int, seed: int = SEED, frac_div: int = 100) -> np.ndarray:
    """Seeded straggler-rank flags: max(1, R // frac_div) draws of splitmix64 % R."""
    flags = np.zeros(R, dtype=np.uint8)
    n = max(1, R // frac_div)
    for j in range(n):
        flags[splitmix64(seed ^ (0xC0FFEE + j)) % R] = 1
    return flags


def gen_matrix(R, K, s_push, seed=SEED, seed2=SEED2, straggler=None) -> np.ndarray:
    if straggler is None:
        straggler = straggler_ranks(R, seed)
    straggler = np.ascontiguousarray(straggler, dtype=np.uint8)
    out = np.empty((R, K, s_push), dtype=np.uint32)
    lib().oracle_gen_matrix(_p(out), R, K, s_push, seed, seed2, _p(straggler))
    return out


# ---------------------------------------------------------------- statistics
def ns_to_us(ns) -> np.ndarray:
    """CuptiProfiler.cpp:187 conversion, elementwise (u64 -> f32 RN, then / 1000.0f)."""
    ns = np.asarray(ns, dtype=np.uint64)
    f = ns.astype(np.float32)  # RN, exact below 2**24
    return (f / np.float32(1000.0)).astype(np.float32)


KEY_WIDE = 0xE0000000
KEY_WIDE_F32BITS = 0x4F600000


def duration_key(ns) -> np.ndarray:
    """u64 ns -> u32 duration keys (the record-log / matrix element format, nvrx_common.h):
    ns below 0xE0000000, else 0xE0000000 + bits(f32(ns)) - bits(f32(0xE0000000))."""
    ns = np.asarray(ns, dtype=np.uint64)
    f = ns.astype(np.float32).view(np.uint32).astype(np.uint64)
    wide = np.uint64(KEY_WIDE) + f - np.uint64(KEY_WIDE_F32BITS)
    return np.where(ns < KEY_WIDE, ns, wide).astype(np.uint32)


def key_to_f32(keys) -> np.ndarray:
    """f32(ns) of duration keys (what the reference divides by 1000)."""
    k = np.asarray(keys, dtype=np.uint32)
    wide = (k.astype(np.uint64) - KEY_WIDE + KEY_WIDE_F32BITS).astype(np.uint32).view(np.float32)
    return np.where(k < KEY_WIDE, k.astype(np.float32), wide).astype(np.float32)


def key_to_us(keys) -> np.ndarray:
    """CuptiProfiler.cpp:187 applied to the durations keys encode: f32(ns) / 1000.0f."""
    return (key_to_f32(keys) / np.float32(1000.0)).astype(np.float32)


def compute_stats(values_f32) -> KStats:
    v = np.ascontiguousarray(values_f32, dtype=np.float32)
    st = KStats()
    lib().oracle_compute_stats(_p(v), v.size, ctypes.byref(st))
    return st


def ring_linearize(pushed_f32, cap: int) -> np.ndarray:
    v = np.ascontiguousarray(pushed_f32, dtype=np.float32)
    out = np.empty(min(v.size, cap), dtype=np.float32)
    n = lib().oracle_ring_linearize(_p(v), v.size, cap, _p(out))
    return out[:n]


def matrix_stats(ns: np.ndarray, nseg: int, seg_stride: int, seg_begin: int, seg_len: int,
                 cap: int = 0, nthreads: int = 1, route: str = "radix") -> dict:
    """Stats of segments ns.flat[s*seg_stride+seg_begin : +seg_len], last `cap` kept.
    route "radix": integer keys radix-sorted, then converted (fast; the checker's default);
    "qsort": converted, then a comparison sort of the floats as computeStats does;
    "baseline": every sample pushed through a ring, then std::sort computeStats (baseline.cpp,
    what bench.py times as the host-CPU Reporter).  All give the same sorted float array,
    hence identical statistics (tests/test_oracle_semantics.py)."""
    ns = np.ascontiguousarray(ns, dtype=np.uint32)
    out = {
        "num": np.empty(nseg, np.int32),
        "min": np.empty(nseg, np.float32),
        "max": np.empty(nseg, np.float32),
        "med": np.empty(nseg, np.float32),
        "avg": np.empty(nseg, np.float32),
        "std": np.empty(nseg, np.float32),
    }
    assert route in ("radix", "qsort", "baseline"), route
    if route == "baseline":  # baseline.cpp: ring pushes + std::sort computeStats (timed)
        lib().oracle_baseline_matrix_stats(_p(ns), nseg, seg_stride, seg_begin, seg_len, cap,
                                           _p(out["num"]), _p(out["min"]), _p(out["max"]),
                                           _p(out["med"]), _p(out["avg"]), _p(out["std"]),
                                           int(nthreads))
        return out
    lib().oracle_matrix_stats_route(_p(ns), nseg, seg_stride, seg_begin, seg_len, cap,
                                    _p(out["num"]), _p(out["min"]), _p(out["max"]), _p(out["med"]),
                                    _p(out["avg"]), _p(out["std"]), int(nthreads),
                                    1 if route == "qsort" else 0)
    return out


def records_stats(recs: np.ndarray, rec_off: np.ndarray, nslots: int, cap: int = 0,
                  nthreads: int = 1, route: str = "radix") -> dict:
    """Stats of every (stream, slot) of push-ordered {slot, ns} record streams
    (CuptiProfiler.cpp:168-203 ring pushes + getStats), out[t*nslots + s].  route "baseline":
    per-record ring pushes + std::sort computeStats (baseline.cpp; what bench.py times)."""
    recs = np.ascontiguousarray(recs, dtype=np.uint32).reshape(-1, 2)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.int64)
    nseg = (rec_off.size - 1) * nslots
    out = {k: np.empty(nseg, np.int32 if k == "num" else np.float32)
           for k in ("num", "min", "max", "med", "avg", "std")}
    assert route in ("radix", "baseline"), route
    fn = lib().oracle_baseline_records_stats if route == "baseline" else lib().oracle_records_stats
    fn(_p(recs), _p(rec_off), rec_off.size - 1, nslots, cap,
                               _p(out["num"]), _p(out["min"]), _p(out["max"]), _p(out["med"]),
                               _p(out["avg"]), _p(out["std"]), int(nthreads))
    return out


# ---------------------------------------------------------------- scoring
def records_moments(recs: np.ndarray, rec_off: np.ndarray, nslots: int, cap: int = 0,
                    nthreads: int = 1):
    """Exact mean and population std (us, float64) of every retained (stream, slot) run: what
    the FAST-mode AVG / STD are checked against (2.5e-7 / 1e-6 relative)."""
    recs = np.ascontiguousarray(recs, dtype=np.uint32)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.int64)
    nstreams = rec_off.size - 1
    mean = np.empty(nstreams * nslots, np.float64)
    std = np.empty(nstreams * nslots, np.float64)
    lib().oracle_records_moments(_p(recs), _p(rec_off), nstreams, nslots, cap, _p(mean), _p(std),
                                 nthreads)
    return mean, std


def kernel_ref(num: np.ndarray, med: np.ndarray) -> np.ndarray:
    R, K = num.shape
    ref = np.empty(K, np.float32)
    lib().oracle_kernel_ref(_p(np.ascontiguousarray(num, np.int32)),
                            _p(np.ascontiguousarray(med, np.float32)), R, K, _p(ref))
    return ref


def scores(num, med, avg, col_valid=None, ref=None, hist=None, rel=True, indiv=True):
    """Returns (gpu_rel[R] or None, gpu_ind[R] or None); hist ([R][K] f64) is updated."""
    num = np.ascontiguousarray(num, np.int32)
    med = np.ascontiguousarray(med, np.float32)
    avg = np.ascontiguousarray(avg, np.float32)
    R, K = num.shape
    if ref is None:
        ref = kernel_ref(num, med)
    ref = np.ascontiguousarray(ref, np.float32)
    if col_valid is not None:
        col_valid = np.ascontiguousarray(col_valid, np.uint8)
    if hist is None:
        hist = np.full((R, K), np.inf, np.float64)
    gr = np.empty(R, np.float64) if rel else None
    gi = np.empty(R, np.float64) if indiv else None
    lib().oracle_scores(_p(num), _p(med), _p(avg), R, K, _p(col_valid), _p(ref), _p(hist),
                        _p(gr), _p(gi))
    return gr, gi


def score_partials(num, med, avg, ref, col_in_shard=None, hist=None) -> np.ndarray:
    """[R][6] partial sums over the columns of one shard (rel: s*w, w, n; indiv: same)."""
    num = np.ascontiguousarray(num, np.int32)
    med = np.ascontiguousarray(med, np.float32)
    avg = np.ascontiguousarray(avg, np.float32)
    R, K = num.shape
    if hist is None:
        hist = np.full((R, K), np.inf, np.float64)
    out = np.empty((R, 6), np.float64)
    mask = None if col_in_shard is None else np.ascontiguousarray(col_in_shard, np.uint8)
    lib().oracle_score_partials(_p(num), _p(med), _p(avg), R, K, _p(mask),
                                _p(np.ascontiguousarray(ref, np.float32)), _p(hist), _p(out))
    return out


def stragglers(score: np.ndarray, thr: float) -> np.ndarray:
    score = np.ascontiguousarray(score, np.float64)
    mask = np.empty(score.size, np.uint8)
    lib().oracle_stragglers(_p(score), score.size, float(thr), _p(mask))
    return mask
