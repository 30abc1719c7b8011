// Test-only code object (not product code): a kernel launched through hipExtModuleLaunchKernel
// with a global work size that is not a multiple of the workgroup size, so the live capture's
// composite key must count the partial last block as CUPTI's gridX does (CuptiProfiler.cpp:185).
#include <hip/hip_runtime.h>

extern "C" __global__ void nvrx_grid_probe(unsigned* out, unsigned n) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i;
}

// A device spin of `iters` dependent FMAs per thread (~0.5 ns each at the shader clock): a kernel of
// known length for the capture's duration checks, launched through hipExtModuleLaunchKernel with
// start / stop events (the runtime may then give the packet a completion signal of its own).
extern "C" __global__ void nvrx_spin_alu(float* out, unsigned iters) {
    float x = (float)threadIdx.x;
    for (unsigned i = 0; i < iters; ++i) x = x * 0.999999f + 1e-6f;
    if (x == -1.0f) out[threadIdx.x] = x;  // never true: keeps the loop
}
