// Test-only code object (not product code): the product's ns -> us conversion
// (nvrx::ns_to_us_narrow, nvrx_common.h, used per sample by the lane classes) against the
// reference statement `(float)ns / 1000.0f` (CuptiProfiler.cpp:187, an IEEE f32 division) for
// every key below NVRX_KEY_WIDE; bad[0] counts mismatching keys.
#include "nvrx_common.h"

extern "C" __global__ void nvrx_us_conversion_probe(unsigned long long* bad) {
    unsigned long long miss = 0;
    const unsigned stride = gridDim.x * blockDim.x;
    for (unsigned ns = blockIdx.x * blockDim.x + threadIdx.x; ns < NVRX_KEY_WIDE; ns += stride)
        miss += __float_as_uint((float)ns / 1000.0f) != __float_as_uint(nvrx::ns_to_us_narrow(ns));
    if (miss) atomicAdd(bad, miss);
}
