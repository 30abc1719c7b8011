"""GPU: the lane classes' ns -> us conversion (nvrx::ns_to_us_narrow: an f32 product corrected by
two FMAs, nvrx_common.h) equals the reference statement `(float)ns / 1000.0f`
(CuptiProfiler.cpp:187, an IEEE f32 division) for EVERY duration key below NVRX_KEY_WIDE
(3,758,096,384 keys), on the hardware's own instructions -- through a test-only code object
(tests/native/us_conversion.hip) that calls the product function."""
import ctypes
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tests", "native", "us_conversion.hsaco")


def test_f32_conversion_equals_ieee_division_for_every_narrow_key():
    assert os.path.exists(PROBE), "build first: make -C tests/native (__graft_entry__.build())"
    hip = ctypes.CDLL("libamdhip64.so")
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(mod), PROBE.encode()) == 0
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"nvrx_us_conversion_probe") == 0
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    a_bad = ctypes.c_void_p(bad.data_ptr())
    params = (ctypes.c_void_p * 1)(ctypes.cast(ctypes.byref(a_bad), ctypes.c_void_p))
    hip.hipModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [
        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = hip.hipModuleLaunchKernel(fn, 16384, 1, 1, 256, 1, 1, 0, stream, params, None)
    assert rc == 0, rc
    torch.cuda.synchronize()
    assert int(bad.item()) == 0, f"{int(bad.item())} keys differ from (float)ns / 1000.0f"
    hip.hipModuleUnload(mod)
