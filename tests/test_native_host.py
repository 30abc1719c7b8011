"""The C ABI from a native C11 host: tests/native/abi_host.c, compiled with
gcc -std=c11 -Wall -Wextra -pedantic -Werror against include/nvrx_straggler.h and linked to
libnvrx_hip.so, runs INTEGRATION.md section 3's strided statistics + nvrx_scores sequence and the
nvrx_profiler_* lifecycle with no Python in the process (cupti_module_py.cpp:33-54 is the binding it
stands in for); its outputs are checked here against the oracle.

CPU: the header compiles as C11 (and C++17) on its own, and the host compiles.
GPU: the prebuilt host runs (built by tests/native/Makefile from __graft_entry__.build(), never inside
a test); NUM/MIN/MAX/MED bit-exact and scores within 1e-6 of the oracle; the profiler's EXACT
statistics of the pushed records bit-exact in every field, name-sorted, the ring of 7 kept."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
HOST = os.path.join(ROOT, "tests", "native", "abi_host")
STRICT_C = ["-std=c11", "-Wall", "-Wextra", "-pedantic", "-Werror"]


def test_header_compiles_as_c11_and_cpp17(tmp_path):
    hdr = os.path.join(INC, "nvrx_straggler.h")
    subprocess.run(["gcc", *STRICT_C, "-fsyntax-only", "-x", "c", hdr], check=True)
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-pedantic", "-Werror", "-fsyntax-only",
                    "-x", "c++", hdr], check=True)


def test_native_host_compiles(tmp_path):
    src = os.path.join(ROOT, "tests", "native", "abi_host.c")
    subprocess.run(["gcc", *STRICT_C, "-D__HIP_PLATFORM_AMD__", "-isystem", "/opt/rocm/include",
                    "-I", INC, "-c", src, "-o", str(tmp_path / "abi_host.o")], check=True)


class _Reader:
    def __init__(self, path):
        self.buf, self.pos = open(path, "rb").read(), 0

    def take(self, dtype, n):
        a = np.frombuffer(self.buf, dtype=dtype, count=n, offset=self.pos)
        self.pos += a.nbytes
        return a


@pytest.mark.gpu
def test_native_host_matches_oracle(tmp_path):
    assert os.path.exists(HOST), "tests/native/abi_host not built (make -C tests/native)"
    out = tmp_path / "abi_host.bin"
    r = subprocess.run([HOST, str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    rd = _Reader(out)
    R, K, S, cap = (int(x) for x in rd.take(np.int64, 4))
    ns = rd.take(np.uint32, R * K * S)
    g = {f: rd.take(np.int32 if f == "num" else np.float32, R * K)
         for f in ("num", "min", "max", "med", "avg", "std")}
    gpu_rel, gpu_ind = rd.take(np.float64, R), rd.take(np.float64, R)
    srel, sind = rd.take(np.uint8, R), rd.take(np.uint8, R)
    err = int(rd.take(np.int32, 1)[0])
    st = O.matrix_stats(ns, R * K, S, 0, S, cap)
    for f in ("num", "min", "max", "med"):
        assert np.array_equal(g[f].view(np.int32), st[f].view(np.int32)), f
    # NVRX_STATS_FAST: the exact mean / std rounded once, so within the reference's own f32
    # accumulation error of it (sequential sums over 1024 samples: ~1.5e-6 seen), and within
    # one rounding of the exact mean of the retained f32 microsecond values
    for f in ("avg", "std"):
        np.testing.assert_allclose(g[f], st[f], rtol=1e-5, atol=0)
    us = O.ns_to_us(ns.reshape(R * K, S)[:, S - cap:]).astype(np.float64)
    np.testing.assert_allclose(g["avg"], us.mean(axis=1), rtol=2.5e-7, atol=0)
    gr, gi = O.scores(st["num"].reshape(R, K), st["med"].reshape(R, K), st["avg"].reshape(R, K))
    np.testing.assert_allclose(gpu_rel, gr, rtol=1e-6, atol=0)
    np.testing.assert_allclose(gpu_ind, gi, rtol=1e-6, atol=0)
    assert np.array_equal(srel, O.stragglers(gr, 0.8)) and srel.sum() == 1 and srel[5] == 1
    assert np.array_equal(sind, O.stragglers(gi, 0.8))
    assert err == 0

    # B: the profiler handle (EXACT mode: every field bit-exact, CuptiProfiler.cpp:44-74)
    n, nk = (int(x) for x in rd.take(np.int64, 2))
    recs = rd.take(np.uint32, 2 * n).reshape(n, 2)
    slot_names = [bytes(rd.take(np.uint8, 96)).rstrip(b"\0").decode() for _ in range(nk)]
    slots = rd.take(np.uint32, nk)
    p = {f: rd.take(np.int32 if f == "num" else np.float32, nk)
         for f in ("num", "min", "max", "med", "avg", "std")}
    sorted_names = [bytes(rd.take(np.uint8, 96)).rstrip(b"\0").decode() for _ in range(nk)]
    assert rd.pos == len(rd.buf)
    assert sorted_names == sorted(slot_names)                    # std::map order of getStats
    assert [slot_names[s] for s in slots] == sorted_names
    want = O.records_stats(recs, np.array([0, n], np.int64), nk, cap=7)
    for f in ("num", "min", "max", "med", "avg", "std"):
        assert np.array_equal(p[f].view(np.int32), want[f][slots].view(np.int32)), f
    assert sorted(p["num"].tolist()) == [1, 5, 7]                # 21 pushes into a ring of 7
