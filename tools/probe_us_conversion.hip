// Exhaustive check of the ns -> us conversion over every key below NVRX_KEY_WIDE on the GPU
// (not product code): A = (float)ns / 1000.0f (IEEE f32 division: the reference's
// CuptiProfiler.cpp:187 statement), B = the f64 form the kernels use (nvrx_common.h
// ns_to_us_narrow), C = an f32-only form (a product and two FMAs).  Prints the mismatch counts.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void conv_probe(unsigned long long* bad) {
    unsigned long long ab = 0, ac = 0;
    const unsigned stride = gridDim.x * blockDim.x;
    for (unsigned ns = blockIdx.x * blockDim.x + threadIdx.x; ns < 0xE0000000u; ns += stride) {
        const float f = (float)ns;
        const float a = f / 1000.0f;
        const float b = (float)((double)f * (1.0 / 1000.0));
        float q = f * 0.001f;
        const float r = __builtin_fmaf(-q, 1000.0f, f);
        q = __builtin_fmaf(r, 0.001f, q);
        ab += __float_as_uint(a) != __float_as_uint(b);
        ac += __float_as_uint(a) != __float_as_uint(q);
        if (ns > 0xE0000000u - stride) break;
    }
    atomicAdd(&bad[0], ab);
    atomicAdd(&bad[1], ac);
}

int main() {
    unsigned long long* d;
    unsigned long long h[2] = {0, 0};
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    (void)hipMemset(d, 0, sizeof(h));
    hipLaunchKernelGGL(conv_probe, dim3(256 * 64), dim3(256), 0, 0, d);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("{\"keys\": %u, \"div_vs_f64_form\": %llu, \"div_vs_f32_fma_form\": %llu}\n", 0xE0000000u, h[0], h[1]);
    return 0;
}
