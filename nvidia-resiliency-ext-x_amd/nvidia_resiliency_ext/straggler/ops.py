"""Torch-tensor front end of the HIP kernels (thin: allocation + argument marshalling).

Every function takes/returns device tensors and enqueues work on the current HIP stream;
all arithmetic happens in libnvrx_hip.so.  Shape checks run on the host before any
launch (the C layer re-checks).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import torch

from . import _native as N

STATS_FAST = N.NVRX_STATS_FAST
STATS_EXACT = N.NVRX_STATS_EXACT


@dataclass
class SegmentStats:
    """SoA statistics of a batch of segments (device tensors, float32 microseconds)."""

    num: torch.Tensor
    min: torch.Tensor
    max: torch.Tensor
    med: torch.Tensor
    avg: torch.Tensor
    std: torch.Tensor

    @classmethod
    def empty(cls, n: int, device) -> "SegmentStats":
        f = lambda dt: torch.empty(n, dtype=dt, device=device)  # noqa: E731
        return cls(f(torch.int32), f(torch.float32), f(torch.float32), f(torch.float32),
                   f(torch.float32), f(torch.float32))

    def view(self, *shape) -> "SegmentStats":
        return SegmentStats(*(getattr(self, k).view(*shape) for k in
                              ("num", "min", "max", "med", "avg", "std")))

    def soa(self) -> N.StatsSoA:
        return N.StatsSoA(self.num.data_ptr(), self.min.data_ptr(), self.max.data_ptr(),
                          self.med.data_ptr(), self.avg.data_ptr(), self.std.data_ptr())

    def cpu(self) -> "SegmentStats":
        return SegmentStats(*(getattr(self, k).cpu() for k in
                              ("num", "min", "max", "med", "avg", "std")))


def _stream(stream):
    return N.stream_handle(stream)


def segment_stats_strided(ns: torch.Tensor, nseg: int, seg_stride: int, seg_begin: int,
                          seg_len: int, cap: int = 0, mode: int = STATS_FAST,
                          out: Optional[SegmentStats] = None, col_ref: Optional[torch.Tensor] = None,
                          ncols: int = 0, stream=None, colref_ready: bool = False) -> SegmentStats:
    """Stats of segments ns.flat[s*seg_stride + seg_begin : +seg_len] (u32 duration keys,
    ``_native.duration_keys``: plain ns below 3.76 s -- raw u32 ns of 3.76 s and more need
    ``encode_ns_u32_`` first; a u32 above ``_native.KEY_MAX`` comes from no u64 duration), last
    `cap` samples retained (CircularBuffer.h:53-69).  reference: CuptiProfiler.cpp:44-74."""
    N.require_device(ns, "ns")
    if ns.dtype not in (torch.int32, torch.uint32):
        raise TypeError("ns must be a 32-bit integer tensor of duration keys")
    if nseg > 0 and (nseg - 1) * seg_stride + seg_begin + seg_len > ns.numel():
        raise ValueError("segments exceed the ns tensor")
    if out is None:
        out = SegmentStats.empty(nseg, ns.device)
    soa = out.soa()
    if col_ref is not None and (col_ref.numel() < 2 * ncols or col_ref.dtype != torch.int32):
        raise ValueError("col_ref must be an int32 tensor of >= 2*ncols elements")
    if colref_ready:  # col_ref holds the initial reference already (a previous scores epilogue)
        mode |= N.NVRX_STATS_COLREF_READY
    N.call("nvrx_segment_stats_strided", ns.data_ptr(), nseg, seg_stride, seg_begin, seg_len,
           cap, mode, ctypes.byref(soa), N.ptr(col_ref), ncols, _stream(stream))
    return out


def encode_ns_u32_(ns: torch.Tensor, stream=None) -> torch.Tensor:
    """In place: raw u32 integer-ns durations (any value below 2^32, never encoded) -> duration
    keys.  Values below 3.76 s are unchanged; from 3.76 s up they become the key of f32(ns), the
    value CuptiProfiler.cpp:187 keeps.  Not idempotent: encode raw ns once."""
    N.require_device(ns, "ns")
    if ns.dtype not in (torch.int32, torch.uint32) or not ns.is_contiguous():
        raise TypeError("ns must be a contiguous 32-bit integer tensor")
    N.call("nvrx_encode_ns_u32", ns.data_ptr(), ns.numel(), _stream(stream))
    return ns


def segment_stats_ragged(ns: torch.Tensor, seg_off: torch.Tensor, seg_len: Optional[torch.Tensor],
                         max_len: int, cap: int = 0, mode: int = STATS_FAST, aligned16: bool = False,
                         out: Optional[SegmentStats] = None, col_ref: Optional[torch.Tensor] = None,
                         ncols: int = 0, stream=None) -> SegmentStats:
    """Stats of ragged segments; segments of <= 128 retained samples are bit-exact in every
    field.  col_ref ([2*ncols] int32): fused per-column reference, as for the strided call."""
    N.require_device(ns, "ns")
    N.require_device(seg_off, "seg_off")
    nseg = seg_off.numel() - (0 if seg_len is not None else 1)
    if seg_off.dtype != torch.int64 or (seg_len is not None and seg_len.dtype != torch.int32):
        raise TypeError("seg_off must be int64 and seg_len int32")
    if out is None:
        out = SegmentStats.empty(max(nseg, 0), ns.device)
    soa = out.soa()
    N.call("nvrx_segment_stats_ragged", ns.data_ptr(), seg_off.data_ptr(),
           N.ptr(seg_len), nseg, max_len, cap, mode, int(aligned16), ctypes.byref(soa),
           N.ptr(col_ref), ncols if col_ref is not None else 0, _stream(stream))
    return out


def kernel_ref(num: torch.Tensor, med: torch.Tensor, ref: Optional[torch.Tensor] = None,
               scratch: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    """ref[k] = min_r med[r, k] if every row has k (num > 0), else NaN (reporting.py:255-296)."""
    R, K = med.shape
    if ref is None:
        ref = torch.empty(K, dtype=torch.float32, device=med.device)
    if scratch is None:
        scratch = torch.empty(2 * K, dtype=torch.int32, device=med.device)
    N.call("nvrx_kernel_ref", num.data_ptr(), med.data_ptr(), R, K, ref.data_ptr(),
           scratch.data_ptr(), _stream(stream))
    return ref


def pack_min_times(med: torch.Tensor, ids: torch.Tensor, total: int,
                   out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    """times = -1; times[ids[i]] = float32(med[i]): the _all_reduce_times pack (reporting.py:269-279)."""
    if out is None:
        out = torch.empty(max(total, 1), dtype=torch.float32, device=med.device)
    N.call("nvrx_pack_min_times", med.data_ptr(), ids.data_ptr(), med.numel(), out.data_ptr(),
           total, _stream(stream))
    return out


def scores(num, med, avg, *, col_valid=None, ref=None, ref_index=None, ref_missing=None,
           hist=None, hist_index=None, hist_stride=0, partials=None, err=None,
           finalize: Optional[dict] = None, done=None, reset_col_ref=None, stream=None):
    """Per-row partial sums {sum s*w, sum w, n} for rel and indiv (reporting.py:219-253).
    finalize = dict(gpu_rel=, gpu_ind=, strag_rel=, strag_ind=, thr_rel=, thr_ind=,
    round_f32=) finishes the scores in the same kernel (single shard).  done (2 int32, zero
    before the first call): self-resetting epilogue -- err is stored, not OR-ed (no zeroing
    needed), and reset_col_ref ([2*K'] int32) is re-initialised for the next statistics call
    (segment_stats_strided(colref_ready=True))."""
    R, K = med.shape
    if partials is None and finalize is None:
        partials = torch.empty((R, 6), dtype=torch.float64, device=med.device)
    f64 = med.dtype == torch.float64
    if avg.dtype != med.dtype or (hist is not None and hist.dtype != med.dtype):
        raise TypeError("med, avg and hist must share one float dtype")
    fz = finalize or {}
    a = N.ScoreArgs(R, K, int(f64), num.data_ptr(), med.data_ptr(), avg.data_ptr(),
                    N.ptr(col_valid), N.ptr(ref), N.ptr(ref_index), N.ptr(ref_missing),
                    N.ptr(hist), N.ptr(hist_index), hist_stride, N.ptr(partials), N.ptr(err),
                    int(fz.get("round_f32", False)), float(fz.get("thr_rel", 0.75)),
                    float(fz.get("thr_ind", 0.75)), N.ptr(fz.get("gpu_rel")),
                    N.ptr(fz.get("gpu_ind")), N.ptr(fz.get("strag_rel")), N.ptr(fz.get("strag_ind")),
                    N.ptr(done), N.ptr(reset_col_ref),
                    reset_col_ref.numel() // 2 if reset_col_ref is not None else 0)
    N.call("nvrx_scores", ctypes.byref(a), _stream(stream))
    return partials


def finalize_scores(partials: torch.Tensor, R: int, nshards: int = 1, round_f32: bool = False,
                    thr_rel: float = 0.75, thr_ind: float = 0.75, rel=True, ind=True, err=None,
                    out: Optional[dict] = None, stream=None):
    """Scores + straggler masks from [nshards][R][6] partials (shards summed in order)."""
    dev = partials.device
    o = out or {}
    gr = o.get("gpu_rel", torch.empty(R, dtype=torch.float64, device=dev) if rel else None)
    gi = o.get("gpu_ind", torch.empty(R, dtype=torch.float64, device=dev) if ind else None)
    sr = o.get("strag_rel", torch.empty(R, dtype=torch.uint8, device=dev) if rel else None)
    si = o.get("strag_ind", torch.empty(R, dtype=torch.uint8, device=dev) if ind else None)
    N.call("nvrx_finalize_scores", partials.data_ptr(), R, nshards, int(round_f32),
           float(thr_rel), float(thr_ind), N.ptr(gr), N.ptr(gi), N.ptr(sr), N.ptr(si),
           N.ptr(err), _stream(stream))
    return gr, gi, sr, si


def section_scores(med: torch.Tensor, present: torch.Tensor, *, ref_in=None, ref_index=None,
                   hist=None, round_f32=False, rel=True, ind=True, err=None, stream=None):
    R, S = med.shape
    dev = med.device
    out_rel = torch.empty((R, S), dtype=torch.float64, device=dev) if rel else None
    out_ind = torch.empty((R, S), dtype=torch.float64, device=dev) if ind else None
    ref_work = torch.empty(S, dtype=torch.float32, device=dev) if (rel and ref_in is None) else None
    N.call("nvrx_section_scores", med.data_ptr(), present.data_ptr(), R, S, N.ptr(ref_in),
           N.ptr(ref_index), N.ptr(ref_work), N.ptr(hist), int(round_f32), N.ptr(out_rel),
           N.ptr(out_ind), N.ptr(err), _stream(stream))
    return out_rel, out_ind


def section_stats(values: torch.Tensor, off: torch.Tensor, max_len: int, stream=None):
    """Per-section (num, min, max, med, avg, std) of float64 ms timings (straggler.py:171-197)."""
    nsec = off.numel() - 1
    dev = values.device
    num = torch.empty(nsec, dtype=torch.int32, device=dev)
    out = torch.empty((5, nsec), dtype=torch.float64, device=dev)
    N.call("nvrx_section_stats", values.data_ptr(), off.data_ptr(), nsec, max_len, num.data_ptr(),
           *(out[i].data_ptr() for i in range(5)), _stream(stream))
    return num, out


def stragglers(score: torch.Tensor, thr: float, out: Optional[torch.Tensor] = None, stream=None):
    if out is None:
        out = torch.empty(score.numel(), dtype=torch.uint8, device=score.device)
    N.call("nvrx_stragglers", score.data_ptr(), score.numel(), float(thr), out.data_ptr(),
           _stream(stream))
    return out


def records_bucket_capacity(n: int, nstreams: int, nslots: int) -> int:
    return int(N.lib().nvrx_records_bucket_capacity(n, nstreams, nslots))


def records_bucket(recs: torch.Tensor, rec_off: torch.Tensor, nslots: int, cap: int, stream=None,
                   out=None):
    """recs: [n, 2] uint32/int32 {slot, ns}; rec_off: [nstreams+1] int64 (device).
    Returns (seg_off int64 [nstreams*nslots], seg_len int32, out_ns, counts int32); `out`
    may pass that tuple preallocated (out_ns >= records_bucket_capacity(...) elements)."""
    nstreams = rec_off.numel() - 1
    dev = recs.device
    n = recs.shape[0]
    cap_ns = records_bucket_capacity(n, nstreams, nslots)
    if out is None:
        seg_off = torch.empty(nstreams * nslots, dtype=torch.int64, device=dev)
        seg_len = torch.empty(nstreams * nslots, dtype=torch.int32, device=dev)
        counts = torch.empty(nstreams * nslots, dtype=torch.int32, device=dev)
        out_ns = torch.empty(max(cap_ns, 1), dtype=torch.int32, device=dev)
    else:
        seg_off, seg_len, out_ns, counts = out
        if (seg_off.numel() < nstreams * nslots or seg_len.numel() < nstreams * nslots or
                counts.numel() < nstreams * nslots or out_ns.numel() < cap_ns):
            raise ValueError("records_bucket: preallocated outputs too small")
    N.call("nvrx_records_bucket", recs.data_ptr(), rec_off.data_ptr(), nstreams, nslots, cap,
           seg_off.data_ptr(), seg_len.data_ptr(), out_ns.data_ptr(), counts.data_ptr(),
           _stream(stream))
    return seg_off, seg_len, out_ns, counts


def records_stats(recs: torch.Tensor, rec_off: torch.Tensor, nslots: int, cap: int, max_len: int,
                  mode: int = STATS_FAST, out: Optional[SegmentStats] = None, bucket=None,
                  col_ref: Optional[torch.Tensor] = None, stream=None) -> SegmentStats:
    """Per-(stream, slot) statistics of push-ordered record streams (ring retention of the
    last `cap` + computeStats): bucketing, then the length-classed segment kernels.  `bucket` may pass the
    (seg_off, seg_len, out_ns, counts) work tensors preallocated (counts may be None: the pushes
    per bucket are then not written); col_ref ([2*nslots] int32) receives the per-slot reference
    (min over streams of MED | missing)."""
    nstreams = rec_off.numel() - 1
    dev = recs.device
    n = recs.shape[0]
    cap_ns = records_bucket_capacity(n, nstreams, nslots)
    if bucket is None:
        bucket = (torch.empty(nstreams * nslots, dtype=torch.int64, device=dev),
                  torch.empty(nstreams * nslots, dtype=torch.int32, device=dev),
                  torch.empty(max(cap_ns, 1), dtype=torch.int32, device=dev),
                  torch.empty(nstreams * nslots, dtype=torch.int32, device=dev))
    seg_off, seg_len, out_ns, counts = bucket
    if out_ns.numel() < cap_ns or seg_off.numel() < nstreams * nslots:
        raise ValueError("records_stats: preallocated work tensors too small")
    if out is None:
        out = SegmentStats.empty(nstreams * nslots, dev)
    soa = out.soa()
    N.call("nvrx_records_stats", recs.data_ptr(), rec_off.data_ptr(), nstreams, nslots, cap, mode,
           max_len, seg_off.data_ptr(), seg_len.data_ptr(), out_ns.data_ptr(), N.ptr(counts),
           ctypes.byref(soa), N.ptr(col_ref), _stream(stream))
    return out
