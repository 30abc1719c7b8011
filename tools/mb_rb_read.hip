// mb_rb_read.hip -- how the bucketing kernel's pass-1 read layout affects HBM throughput on the
// configs[3] record streams (16,384 streams x 47,482 records of 8 B, one 16-wave workgroup per
// stream, one workgroup per CU): (a) chunked -- wave w reads its own contiguous 1/16 of the
// stream, RB pairs per lane in flight (the shipped layout); (b) interleaved -- the 16 waves sweep
// the stream together, wave w taking every 16th 1 KB step; both count slots into LDS (the pass-1
// work), so only the address order differs.
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/mb_rb_read tools/mb_rb_read.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int64_t NSTREAM = 16384, NREC = 47482, NSLOT = 2048, W = 16, RB = 16;

template <bool INTERLEAVED>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(1, 4)))
void pass1(const u32x4* recs, unsigned* out) {
    __shared__ unsigned cnt[NSLOT];
    for (int s = threadIdx.x; s < NSLOT; s += blockDim.x) cnt[s] = 0u;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t np = NREC / 2;  // pairs per stream (NREC even)
    const u32x4* q = recs + blockIdx.x * np;
    const auto count = [&](const u32x4& w) {
        atomicAdd(&cnt[w.x & (NSLOT - 1)], 1u);
        atomicAdd(&cnt[w.z & (NSLOT - 1)], 1u);
    };
    if (!INTERLEAVED) {
        const int64_t per = (np + W - 1) / W;
        const int64_t lo = per * wave, hi = lo + per < np ? lo + per : np;
        for (int64_t i = lo + lane; i < hi; i += 64 * RB) {
            u32x4 w[RB];
#pragma unroll
            for (int u = 0; u < RB; ++u) w[u] = i + 64 * u < hi ? __builtin_nontemporal_load(q + i + 64 * u) : u32x4{0, 0, 0, 0};
#pragma unroll
            for (int u = 0; u < RB; ++u) count(w[u]);
        }
    } else {
        for (int64_t b = (int64_t)wave * 64 + lane; b < np; b += 64 * W * RB) {
            u32x4 w[RB];
#pragma unroll
            for (int u = 0; u < RB; ++u) {
                const int64_t i = b + (int64_t)u * 64 * W;
                w[u] = i < np ? __builtin_nontemporal_load(q + i) : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < RB; ++u) count(w[u]);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = cnt[blockIdx.x & (NSLOT - 1)];
}

__global__ void init(u32x4* recs, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const unsigned h = (unsigned)(i * 2654435761u);
        recs[i] = u32x4{h >> 21, 1000u + (h & 0xFFFF), (h * 40503u) >> 21, 2000u + (h >> 16)};
    }
}

int main() {
    const size_t bytes = (size_t)NSTREAM * NREC * 8;
    u32x4* recs;
    unsigned* out;
    if (hipMalloc(&recs, bytes) != hipSuccess || hipMalloc(&out, NSTREAM * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(init, dim3(4096), dim3(256), 0, 0, recs, (int64_t)(bytes / 16));
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const size_t lds = 160 * 1024 - 16 * 1024;  // one workgroup per CU, as the bucketing kernel
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 2; ++mode) {
            auto k = mode ? (const void*)pass1<true> : (const void*)pass1<false>;
            (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            auto launch = [&] {
                if (mode) hipLaunchKernelGGL(pass1<true>, dim3(NSTREAM), dim3(64 * W), lds, 0, recs, out);
                else hipLaunchKernelGGL(pass1<false>, dim3(NSTREAM), dim3(64 * W), lds, 0, recs, out);
            };
            launch();
            (void)hipEventRecord(a);
            for (int i = 0; i < 5; ++i) launch();
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            ms /= 5;
            printf("%-12s %.3f ms  %.0f GB/s\n", mode ? "interleaved" : "chunked", ms, bytes / (ms * 1e6));
        }
    }
    return hipDeviceSynchronize() != hipSuccess;
}
