// Test-only code object (not product code): a kernel launched through hipExtModuleLaunchKernel
// with a global work size that is not a multiple of the workgroup size, so the live capture's
// composite key must count the partial last block as CUPTI's gridX does (CuptiProfiler.cpp:185).
#include <hip/hip_runtime.h>

extern "C" __global__ void nvrx_grid_probe(unsigned* out, unsigned n) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i;
}
