"""Validate bench.py's host-CPU baseline (oracle/baseline.cpp, kind "port") against the
reference's own per-kernel path compiled from /root/reference (oracle/_ref/libnvrx_ref.so,
ref_matrix_stats: CircularBuffer pushes + computeStats), on the same inputs and cores, in THIS
container (oracle/_ref never leaves it).  SURVEY 8(d): the port must run within +-20 % of the
reference's per-core rate.  Writes profiles/r02/cpu_baseline_validation.json."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

FIELDS = ("num", "min", "max", "med", "avg", "std")
L = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libnvrx_ref.so"))
P, i64 = ctypes.c_void_p, ctypes.c_int64
L.ref_matrix_stats.argtypes = [P, i64, i64, i64, i64, i64, P, P, P, P, P, P, ctypes.c_int]


def ref_stats(flat, nseg, S, cap, threads):
    out = {f: np.empty(nseg, np.int32 if f == "num" else np.float32) for f in FIELDS}
    L.ref_matrix_stats(flat.ctypes.data, nseg, S, 0, S, cap, *[out[f].ctypes.data for f in FIELDS],
                       threads)
    return out


rows = []
cores = len(os.sched_getaffinity(0))
for (R, K, S, label) in ((4, 2048, 10000, "configs[1] rows: 2048 kernels x 10,000 pushed, 8192 kept"),
                         (32, 2048, 1024, "configs[2] rows: 2048 kernels x 1024")):
    ns = O.gen_matrix(R, K, S)
    flat = np.ascontiguousarray(ns.reshape(-1))
    nseg, keep = R * K, min(S, 8192)
    for threads in (1, cores):
        t = time.perf_counter()
        a = ref_stats(flat, nseg, S, 8192, threads)
        t_ref = time.perf_counter() - t
        t = time.perf_counter()
        b = O.matrix_stats(flat, nseg, S, 0, S, 8192, nthreads=threads, route="baseline")
        t_port = time.perf_counter() - t
        same = all(np.array_equal(a[f].view(np.uint32), b[f].view(np.uint32)) for f in FIELDS)
        rows.append(dict(workload=f"{R} {label}", threads=threads,
                         reference_samples_per_s=nseg * keep / t_ref,
                         port_samples_per_s=nseg * keep / t_port,
                         port_over_reference=t_ref / t_port, bit_identical=same))
        print(rows[-1])
doc = dict(method="oracle/_ref ref_matrix_stats (the reference CuptiProfiler.cpp computeStats + "
                  "CircularBuffer compiled from /root/reference by oracle/Makefile) vs "
                  "oracle/baseline.cpp (route 'baseline'), same inputs and thread counts, this "
                  "container's CPUs", cpu=os.uname().machine, cores=cores, rows=rows)
os.makedirs(os.path.join(ROOT, "profiles", "r02"), exist_ok=True)
json.dump(doc, open(os.path.join(ROOT, "profiles", "r02", "cpu_baseline_validation.json"), "w"), indent=1)
