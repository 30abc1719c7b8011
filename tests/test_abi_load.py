"""CPU: the C-ABI library loads without a GPU and exports every symbol the header declares."""
import ctypes
import os
import re

import pytest

from nvidia_resiliency_ext.straggler import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nvrx_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    lib = ctypes.CDLL(_native.LIB_PATH)
    names = _declared("nvrx_straggler.h")
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    names = _declared("nvrx_straggler.h")
    assert sorted(_native.SIGNATURES) == names


def test_lib_loads_and_reports_abi():
    L = _native.lib()
    assert L.nvrx_abi_version() == _native.ABI_VERSION == 6
    cnt = ctypes.c_int(-1)
    # no HIP device in the CPU container: the call succeeds (0 devices) or reports HIP error
    rc = L.nvrx_device_count(ctypes.byref(cnt))
    assert rc in (0, _native.NVRX_ERR_HIP)


def test_argument_errors_raise_runtime_error_without_gpu():
    # host-side checks run before any launch: a bad mode is rejected with a message
    soa = _native.StatsSoA(1, 1, 1, 1, 1, 1)
    rc = _native.lib().nvrx_segment_stats_strided(1, 1, 8, 0, 8, 0, 9, ctypes.byref(soa), None, 0,
                                                  None)
    assert rc == _native.NVRX_ERR_INVALID
    assert b"mode" in _native.lib().nvrx_last_error()
    with pytest.raises(RuntimeError, match="mode"):
        _native.check(rc, "x")


def test_synth_header_symbols_exported():
    lib = ctypes.CDLL(os.path.join(os.path.dirname(_native.LIB_PATH), "libnvrx_synth.so"))
    for n in _declared("nvrx_synth.h"):
        assert hasattr(lib, n), n


def test_capture_counters_without_capture():
    # the cost accounting of the live capture: all zero while no tool is configured
    c = _native.CaptureCounters()
    assert _native.lib().nvrx_capture_stats(ctypes.byref(c)) == 0
    assert (c.callbacks, c.dispatches, c.flushes, c.callback_ns) == (0, 0, 0, 0)
    assert (c.enqueues_counted, c.counted_flushes, c.flush_timeouts, c.delivery) == (0, 0, 0, -1)
    # the C struct and the ctypes mirror agree on the layout (two int32 at the end)
    assert ctypes.sizeof(c) == 16 * 8 + 2 * 4 + 6 * 8
    assert _native.lib().nvrx_capture_stats(None) == _native.NVRX_ERR_INVALID
