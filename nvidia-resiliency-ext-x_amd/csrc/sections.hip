// sections.hip -- statistics of user-section CPU timings (gfx950).
//
// Replaces Detector._get_section_summaries (straggler/straggler.py:171-197), which runs
// torch on the host over each section's deque of elapsed ms (float64):
//   MIN, MAX, MED = torch.median (the LOWER median, s[(n-1)/2]), AVG = mean,
//   STD = unbiased (n-1) standard deviation, NaN when n == 1, NUM = n.
// One 256-thread workgroup per section: values staged in LDS, bitonic sort (+inf
// padding), then order statistics; mean / variance by a fixed-order tree over the
// sorted values (float64; torch's own summation order is not specified, so AVG/STD
// match to ~1e-16 relative, MIN/MAX/MED exactly).  Sections longer than 16384 timings
// (CustomSection.max_elapseds_len raised by the user) are sorted the same way in a device
// scratch buffer by a 1024-thread workgroup.
#include <algorithm>
#include "nvrx_common.h"
#include "nvrx_internal.h"

namespace nvrx {

// The statistics of one section, every thread of the block: s (LDS, or this block's
// device scratch) gets the values padded with +inf to a power of two and sorted.
template <int NT>
__device__ __forceinline__ void section_body(const double* __restrict__ vals, const int64_t* off,
                                             int64_t sec, double* s, double* red, int32_t* num,
                                             double* mn, double* mx, double* med, double* avg,
                                             double* sd) {
    const int64_t b = off[sec];
    const int n = (int)(off[sec + 1] - b);
    const int tid = threadIdx.x;
    if (n <= 0) {
        if (tid == 0) {
            const double q = __builtin_nan("");
            num[sec] = 0;
            mn[sec] = mx[sec] = med[sec] = avg[sec] = sd[sec] = q;
        }
        return;
    }
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int i = tid; i < np2; i += NT) s[i] = i < n ? vals[b + i] : __builtin_inf();
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < np2; i += NT) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const double x = s[i], y = s[ixj];
                    const bool up = (i & k) == 0;
                    if (up ? (x > y) : (x < y)) {
                        s[i] = y;
                        s[ixj] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    // mean: per-thread strided partial sums, then a fixed tree
    double acc = 0.0;
    for (int i = tid; i < n; i += NT) acc += s[i];
    red[tid] = acc;
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
        if (tid < w) red[tid] = red[tid] + red[tid + w];
        __syncthreads();
    }
    const double mean = red[0] / (double)n;
    __syncthreads();
    double q = 0.0;
    for (int i = tid; i < n; i += NT) {
        const double d = s[i] - mean;
        q += d * d;
    }
    red[tid] = q;
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
        if (tid < w) red[tid] = red[tid] + red[tid + w];
        __syncthreads();
    }
    if (tid == 0) {
        num[sec] = n;
        mn[sec] = s[0];
        mx[sec] = s[n - 1];
        med[sec] = s[(n - 1) / 2];
        avg[sec] = mean;
        sd[sec] = n > 1 ? __builtin_sqrt(red[0] / (double)(n - 1)) : __builtin_nan("");
    }
}

template <int NMAX>
__global__ __launch_bounds__(256) void section_stats_kernel(const double* __restrict__ vals,
                                                            const int64_t* __restrict__ off,
                                                            int32_t* num, double* mn, double* mx,
                                                            double* med, double* avg, double* sd) {
    __shared__ double s[NMAX];
    __shared__ double red[256];
    section_body<256>(vals, off, blockIdx.x, s, red, num, mn, mx, med, avg, sd);
}

// sections longer than the LDS holds: the block's own slice of a device scratch buffer
// (np2 doubles per section); global stores are visible to the block after __syncthreads
__global__ __launch_bounds__(1024) void section_stats_global_kernel(
    const double* __restrict__ vals, const int64_t* __restrict__ off, double* work, int64_t np2,
    int32_t* num, double* mn, double* mx, double* med, double* avg, double* sd) {
    __shared__ double red[1024];
    section_body<1024>(vals, off, blockIdx.x, work + (int64_t)blockIdx.x * np2, red, num, mn, mx,
                       med, avg, sd);
}

hipError_t section_stats(const double* vals, const int64_t* off, int64_t nsec, int64_t max_len,
                         int32_t* num, double* mn, double* mx, double* med, double* avg,
                         double* sd, hipStream_t st) {
    if (nsec <= 0) return hipSuccess;
    if (max_len <= 1024)
        hipLaunchKernelGGL(section_stats_kernel<1024>, dim3((unsigned)nsec), dim3(256), 0, st, vals,
                           off, num, mn, mx, med, avg, sd);
    else if (max_len <= 8192)
        hipLaunchKernelGGL(section_stats_kernel<8192>, dim3((unsigned)nsec), dim3(256), 0, st, vals,
                           off, num, mn, mx, med, avg, sd);
    else if (max_len <= 16384)
        hipLaunchKernelGGL(section_stats_kernel<16384>, dim3((unsigned)nsec), dim3(256), 0, st, vals,
                           off, num, mn, mx, med, avg, sd);
    else {
        if (max_len > ((int64_t)1 << 30)) return hipErrorInvalidValue;
        int64_t np2 = 1;
        while (np2 < max_len) np2 <<= 1;
        // sections are sized by the longest one, so the scratch is bounded by launching a chunk
        // of sections at a time (at least one): <= 256 MiB unless one section needs more
        const int64_t per = std::max<int64_t>(1, ((int64_t)256 << 20) / (np2 * (int64_t)sizeof(double)));
        const int64_t chunk = std::min(nsec, per);
        void* work = nullptr;
        hipError_t e = scratch_alloc(&work, (size_t)(chunk * np2) * sizeof(double), st);
        if (e != hipSuccess) return e;
        for (int64_t c0 = 0; c0 < nsec && e == hipSuccess; c0 += chunk) {
            const int64_t m = std::min(chunk, nsec - c0);
            hipLaunchKernelGGL(section_stats_global_kernel, dim3((unsigned)m), dim3(1024), 0, st, vals,
                               off + c0, (double*)work, np2, num + c0, mn + c0, mx + c0, med + c0,
                               avg + c0, sd + c0);
            e = hipGetLastError();
        }
        const hipError_t f = hipFreeAsync(work, st);  // on the error path too
        return e != hipSuccess ? e : f;
    }
    return hipGetLastError();
}

}  // namespace nvrx
