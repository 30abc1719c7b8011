"""Deterministic ReportGenerator scenarios shared by make_golden.py (which runs the
REFERENCE on them, in the dev container) and the tests (which run the oracle and the
HIP product path on them).  Inputs are integer-ns durations from the SURVEY 8(d)
generator; summaries are computeStats of the converted durations (the stats function is
passed in: the reference's own computeStats for the goldens, the oracle's or the GPU's
in the tests).  Nothing here imports the reference.
"""
from __future__ import annotations

import hashlib
import struct
from typing import Callable, Dict, List, Sequence

import numpy as np

STAT_KEYS = ("MIN", "MAX", "MED", "AVG", "STD", "NUM")
M64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


SCENARIOS = {
    # name: world size, scores, gather, kernels, samples, reports, features
    "ws4_all_gather": dict(ws=4, scores=["relative_perf_scores", "individual_perf_scores"],
                           gather=True, K=200, S=1000, reports=3, sections=2, missing=True,
                           nccl=True, shuffle=False),
    "ws2_all_nogather": dict(ws=2, scores=["relative_perf_scores", "individual_perf_scores"],
                             gather=False, K=200, S=1000, reports=3, sections=2, missing=True,
                             nccl=True, shuffle=True),
    "ws8_rel_gather": dict(ws=8, scores=["relative_perf_scores"], gather=True, K=200, S=600,
                           reports=3, sections=1, missing=False, nccl=False, shuffle=False),
    "ws4_indiv_nogather": dict(ws=4, scores=["individual_perf_scores"], gather=False, K=120,
                               S=500, reports=4, sections=2, missing=True, nccl=True,
                               shuffle=False),
}


def kernel_name(k: int) -> str:
    return f"kern_{k:04d}_blk_{64 * (1 + k % 4)}_1_1_grid_{1 + k % 13}_1_1"


def straggler_of(ws: int, t: int) -> int:
    """The straggler rank of report t (the slowest GPU moves between reports)."""
    return (1 + t) % ws


def report_seed(t: int) -> int:
    return 0x5EED ^ (0x1000 * (t + 1))


def kernels_of(sc: dict, r: int, t: int) -> List[int]:
    ks = list(range(sc["K"]))
    if sc["missing"] and t == 1:
        ks = [k for k in ks if (k + r) % 7 != 0]   # some kernels absent on some ranks
    return ks


def section_timings(sc: dict, r: int, t: int, s: int) -> List[float]:
    """CPU section timings in ms (as Detector records perf_counter deltas * 1e-6)."""
    n = 3 + (r + t + s) % 5 + (1 if s == 0 else 0) * 10
    base = 5.0 + 3.0 * s
    slow = 1.3 if r == straggler_of(sc["ws"], t) else 1.0
    out = []
    for i in range(n):
        u = splitmix64(report_seed(t) ^ (r << 20) ^ (s << 12) ^ i) >> 11
        out.append(base * slow * (1.0 + 0.1 * (u / float(1 << 53))))
    if sc["sections"] > 1 and s == 1 and r == sc["ws"] - 1 and t == 0:
        out = [out[0]]  # n == 1 -> STD NaN (straggler.py:191-193)
    return out


def build_rank_inputs(sc: dict, r: int, t: int, gen_matrix: Callable, stats_fn: Callable,
                      section_fn: Callable):
    """Returns (section_summaries, kernel_summaries) of rank r for report t.
    gen_matrix(R, K, S, seed, straggler) -> uint32 [R][K][S];
    stats_fn(uint32 ns[S]) -> (num, min, max, med, avg, std) with float32 values;
    section_fn(list of ms floats) -> dict of the six stats (torch semantics)."""
    ws, K, S = sc["ws"], sc["K"], sc["S"]
    strag = np.zeros(ws, np.uint8)
    strag[straggler_of(ws, t)] = 1
    ns = gen_matrix(ws, K, S, report_seed(t), strag)
    kernels: Dict[str, dict] = {}
    for k in kernels_of(sc, r, t):
        num, mn, mx, med, avg, sd = stats_fn(ns[r, k])
        kernels[kernel_name(k)] = dict(MIN=float(mn), MAX=float(mx), MED=float(med),
                                       AVG=float(avg), STD=float(sd), NUM=int(num))
    if sc["nccl"]:
        num, mn, mx, med, avg, sd = stats_fn(ns[r, 0] * np.uint32(ws - r + 1))
        kernels[f"ncclDevKernel_AllReduce_Sum_f32_RING_LL_blk_256_1_1_grid_{ws}_1_1"] = dict(
            MIN=float(mn), MAX=float(mx), MED=float(med), AVG=float(avg), STD=float(sd),
            NUM=int(num))
    if sc["missing"] and t == 2:
        num, mn, mx, med, avg, sd = stats_fn(ns[r, 1])
        kernels[f"rank{r}_only_kernel_blk_32_1_1_grid_1_1_1"] = dict(
            MIN=float(mn), MAX=float(mx), MED=float(med), AVG=float(avg), STD=float(sd),
            NUM=int(num))
    names = list(kernels.keys())
    if sc["shuffle"]:
        names.sort(key=lambda n: splitmix64(hash_str(n) ^ r ^ (t << 8)))
    else:
        names.sort()  # CuptiProfiler::getStats std::map order
    kernels = {n: kernels[n] for n in names}
    sections = {}
    for s in range(sc["sections"]):
        sections[f"section{s}"] = section_fn(section_timings(sc, r, t, s))
    return sections, kernels


def hash_str(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h = ((h ^ b) * 0x100000001B3) & M64
    return h


def summaries_digest(sections: dict, kernels: dict) -> str:
    """sha256 over the exact bits of every summary value, in dict order."""
    h = hashlib.sha256()
    for group in (sections, kernels):
        for name, st in group.items():
            h.update(name.encode())
            for k in STAT_KEYS:
                v = st[k]
                h.update(struct.pack("<q", v) if k == "NUM" else struct.pack("<d", float(v)))
    return h.hexdigest()


def encode_scores(d) -> dict:
    """JSON form of a score mapping: float.hex keeps every bit (NaN -> 'nan')."""
    def enc(x):
        return "nan" if x != x else float(x).hex()
    out = {}
    for k, v in d.items():
        out[str(k)] = {str(r): enc(x) for r, x in v.items()} if isinstance(v, dict) else enc(v)
    return out


def decode_value(s: str) -> float:
    return float("nan") if s == "nan" else float.fromhex(s)


REPORT_FIELDS = ("gpu_relative_perf_scores", "section_relative_perf_scores",
                 "gpu_individual_perf_scores", "section_individual_perf_scores")


def encode_report(rep) -> dict:
    if rep is None:
        return None
    get = (lambda f: rep[f]) if isinstance(rep, dict) else (lambda f: getattr(rep, f))
    out = {f: encode_scores(get(f)) for f in REPORT_FIELDS}
    out["rank_to_node"] = {str(k): v for k, v in get("rank_to_node").items()}
    out["gather_on_rank0"] = bool(get("gather_on_rank0"))
    out["rank"] = get("rank")
    return out


COMPUTE_STATS_CASES: Sequence = (
    # (name, ns samples pushed, ring cap)
    ("n1", [1500], 8192),
    ("n2", [1500, 2500], 8192),
    ("n3_dup", [1000, 1000, 2000], 8192),
    ("n4_even", [3000, 4000, 5000, 6000], 8192),
    ("ring_cap7_21pushes", [1000 * (i + 1) for i in range(21)], 7),
    ("ring_cap4_1to6", [1000 * (i + 1) for i in range(6)], 4),
    ("f32_round_2p24", [2**24 - 1, 2**24, 2**24 + 1, 2**24 + 2, 2**24 + 3], 8192),
    ("div1000_rounding", [1, 3, 7, 999, 1001, 123457, 16777217, 33554431], 8192),
    ("zeros", [0, 0, 0], 8192),
    ("large_u32", [4294967295, 4000000000, 17, 3999999999], 8192),
)
