"""Synthetic integer-ns duration workloads for tests and bench.py (not a reporting API).

Device side: libnvrx_synth.so (csrc/synth.hip), bit-identical to the oracle generator
(oracle/nvrx_oracle.c).  Host side helpers here only build the seeded
straggler-rank set and kernel names (tiny, deterministic).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import numpy as np
import torch

SEED = 0x5EED
SEED2 = 0xBA5E
_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnvrx_synth.so")
_lib = None

M64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def straggler_ranks(R: int, seed: int = SEED, frac_div: int = 100) -> np.ndarray:
    """Seeded straggler-rank flags: max(1, R // frac_div) draws of splitmix64 % R."""
    flags = np.zeros(R, dtype=np.uint8)
    for j in range(max(1, R // frac_div)):
        flags[splitmix64(seed ^ (0xC0FFEE + j)) % R] = 1
    return flags


def kernel_names(K: int) -> List[str]:
    """Composite names in the reference's "%s_blk_%d_%d_%d_grid_%d_%d_%d" form
    (CuptiProfiler.cpp:182-185); zero-padded so name order == index order."""
    return [f"synth_kernel_{k:05d}_blk_256_1_1_grid_{(k % 97) + 1}_1_1" for k in range(K)]


def kernel_hash(name: str) -> int:
    """Shard key of the multi-GPU path: 64-bit FNV-1a of the composite kernel name, finalised
    with splitmix64 so that the low bits (used by % n_gpus) are well mixed."""
    h = 0xCBF29CE484222325
    for b in name.encode():
        h = ((h ^ b) * 0x100000001B3) & M64
    return splitmix64(h)


def shard_kernels(names: Sequence[str], nshards: int, shard: int) -> np.ndarray:
    """Global kernel indices owned by `shard` under hash(name) % nshards, in name order."""
    return np.array([k for k, n in enumerate(names) if kernel_hash(n) % nshards == shard],
                    dtype=np.int64)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            raise RuntimeError(f"{_LIB} missing; build with make -C nvidia-resiliency-ext-x_amd/csrc")
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        i64 = ctypes.c_int64
        u64 = ctypes.c_uint64
        L.nvrx_synth_matrix.restype = ctypes.c_int
        L.nvrx_synth_matrix.argtypes = [P, i64, i64, i64, P, i64, u64, u64, P, P]
        L.nvrx_synth_records.restype = ctypes.c_int
        L.nvrx_synth_records.argtypes = [P, i64, i64, P, P, P, i64, i64, u64, u64, P, P]
        _lib = L
    return _lib


def synth_matrix(R: int, K_local: int, s_push: int, *, K_global: Optional[int] = None,
                 kmap: Optional[torch.Tensor] = None, straggler: Optional[torch.Tensor] = None,
                 seed: int = SEED, seed2: int = SEED2, device="cuda",
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint32 ns[R][K_local][s_push] (stored as int32) on the device."""
    if out is None:
        out = torch.empty((R, K_local, s_push), dtype=torch.int32, device=device)
    if straggler is None:
        straggler = torch.from_numpy(straggler_ranks(R, seed)).to(out.device)
    kg = K_global if K_global is not None else K_local
    rc = _load().nvrx_synth_matrix(out.data_ptr(), R, K_local, kg,
                                   kmap.data_ptr() if kmap is not None else None, s_push,
                                   seed, seed2, straggler.data_ptr(),
                                   torch.cuda.current_stream(out.device).cuda_stream)
    if rc != 0:
        raise RuntimeError(f"nvrx_synth_matrix failed ({rc})")
    return out


# ---------------------------------------------------------------- record streams (C4)
def zipf_counts(K: int = 2048, top: int = 8192, alpha: float = 1.1) -> np.ndarray:
    """Pushes per report interval of kernel k (0-based): max(1, floor(top / (k+1)^alpha))
    (47,482 records per rank at K=2048)."""
    k = np.arange(1, K + 1, dtype=np.float64)
    return np.maximum(1, np.floor(top / k ** alpha)).astype(np.int64)


def zipf_order(counts: np.ndarray):
    """Push order of one rank's interval: occurrence i of kernel k fires at (2i+1)/(2 n_k)
    of the interval (each kernel evenly spread), ties broken by kernel index.  Distinct
    fractions with denominators <= 2^15 differ by far more than an f64 ulp, so the f64 key
    orders them exactly.  Returns (slot uint32 [N], occ uint32 [N])."""
    counts = np.asarray(counts, np.int64)
    slot = np.repeat(np.arange(counts.size, dtype=np.int64), counts)
    first = np.repeat(np.cumsum(counts) - counts, counts)
    occ = np.arange(slot.size, dtype=np.int64) - first
    key = (2 * occ + 1) / (2 * counts[slot]).astype(np.float64)
    order = np.lexsort((slot, key))
    return slot[order].astype(np.uint32), occ[order].astype(np.uint32)


def synth_records(R: int, slot: torch.Tensor, occ: torch.Tensor, K: int, s_push: int, *,
                  kglob: Optional[torch.Tensor] = None, straggler: Optional[torch.Tensor] = None,
                  seed: int = SEED, seed2: int = SEED2,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Device record streams, int32 view of {slot, ns} pairs: [R * N, 2], rank-major.
    kglob (optional, [N]): global kernel index of each record for the sample hash when
    `slot` holds shard-local slots (K is then the global kernel count)."""
    N = slot.numel()
    dev = slot.device
    if out is None:
        out = torch.empty((R * N, 2), dtype=torch.int32, device=dev)
    if straggler is None:
        straggler = torch.from_numpy(straggler_ranks(R, seed)).to(dev)
    rc = _load().nvrx_synth_records(out.data_ptr(), R, N, slot.data_ptr(),
                                    kglob.data_ptr() if kglob is not None else None,
                                    occ.data_ptr(), K, s_push, seed, seed2, straggler.data_ptr(),
                                    torch.cuda.current_stream(dev).cuda_stream)
    if rc != 0:
        raise RuntimeError(f"nvrx_synth_records failed ({rc})")
    return out


def shard_order(slot: np.ndarray, occ: np.ndarray, kidx: np.ndarray):
    """Restrict a push order to the kernels `kidx` (global indices, this shard), keeping
    push order; returns (local slot, global kernel, occ), all uint32."""
    local = np.full(int(slot.max()) + 1 if slot.size else 1, -1, np.int64)
    local[kidx] = np.arange(kidx.size)
    keep = local[slot.astype(np.int64)] >= 0
    g = slot[keep]
    return local[g.astype(np.int64)].astype(np.uint32), g.astype(np.uint32), occ[keep]
