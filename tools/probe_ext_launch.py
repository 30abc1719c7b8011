"""Probe (not a test): which hipExtModuleLaunchKernel forms the runtime accepts for the
test-only code object tests/native/grid_probe.hsaco, with a global size that is / is not a
multiple of the workgroup size."""
import ctypes
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
hip = ctypes.CDLL("libamdhip64.so")
hip.hipGetErrorString.restype = ctypes.c_char_p
buf = torch.zeros(1024, dtype=torch.int32, device="cuda")
mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
print("load", hip.hipModuleLoad(ctypes.byref(mod), os.path.join(ROOT, "tests/native/grid_probe.hsaco").encode()))
print("getfn", hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"nvrx_grid_probe"))
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
a_out, a_n = ctypes.c_void_p(buf.data_ptr()), ctypes.c_uint32(1000)
params = (ctypes.c_void_p * 2)(ctypes.cast(ctypes.byref(a_out), ctypes.c_void_p),
                               ctypes.cast(ctypes.byref(a_n), ctypes.c_void_p))
hip.hipExtModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [
    ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
    ctypes.c_void_p, ctypes.c_uint32]
hip.hipModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [
    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
for g in (1024, 1000):
    rc = hip.hipExtModuleLaunchKernel(fn, g, 1, 1, 256, 1, 1, 0, stream, params, None, None, None, 0)
    print("ext params", g, rc, hip.hipGetErrorString(rc))
    rc = hip.hipExtModuleLaunchKernel(fn, g, 1, 1, 256, 1, 1, 0, stream, params, None, 0, 0, 0)
    print("ext params (events 0)", g, rc, hip.hipGetErrorString(rc))
rc = hip.hipModuleLaunchKernel(fn, 4, 1, 1, 256, 1, 1, 0, stream, params, None)
print("module params", rc, hip.hipGetErrorString(rc))
torch.cuda.synchronize()
print(buf[:8].tolist(), buf[995:1001].tolist())
