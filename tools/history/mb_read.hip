// mb_read.hip -- HBM read ceiling on MI355X for the configs[1] workload shape (64 x 2048 rows of
// 10,000 u32, the last 8192 of each row read): the stats kernel's pattern (one wave per 32 KB
// segment, 32 x 16-B loads per lane in flight) against alternatives.  Prints GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -o mb_read tools/mb_read.hip && ./mb_read
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

constexpr int64_t ROWS = 64 * 2048, STRIDE = 10000, KEEP = 8192, BEGIN = STRIDE - KEEP;

__device__ __forceinline__ unsigned wmin(unsigned v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, (unsigned)__shfl_xor((int)v, o));
    return v;
}

// (a) the stats kernel's pattern: one wave per row segment, PL x 16-B loads per lane (64 lanes x
//     16 B per instruction), NV = PL / 4 instructions in flight per lane
template <int PL, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W)))
void seg_wave(const uint32_t* ns, unsigned* out) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * 4 + wave;
    if (s >= ROWS) return;
    const uint32_t* p = ns + s * STRIDE + BEGIN;
    const uintptr_t pa = (uintptr_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)pa), hi = __builtin_amdgcn_readfirstlane((unsigned)(pa >> 32));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, KEEP * 4, 0x00020000);
    unsigned m = 0xFFFFFFFFu;
    for (int base = 0; base < KEEP * 4; base += PL * 64 * 4) {
        unsigned v[PL];
#pragma unroll
        for (int j = 0; j < PL / 4; ++j) {
            const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, base + j * 1024, 2);
            v[4 * j] = q.x, v[4 * j + 1] = q.y, v[4 * j + 2] = q.z, v[4 * j + 3] = q.w;
        }
#pragma unroll
        for (int i = 0; i < PL; ++i) m = min(m, v[i]);
    }
    m = wmin(m);
    if (lane == 0) out[s] = m;
}

// (b) flat grid-stride over the same byte ranges: every thread UNR 16-B loads in flight
template <int UNR>
__global__ __launch_bounds__(256) void flat(const uint32_t* ns, unsigned* out, int64_t nvec) {
    const int64_t per_row = KEEP / 4;  // 16-B vectors per row segment
    unsigned m = 0xFFFFFFFFu;
    const int64_t G = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += G * UNR) {
        u32x4 q[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int64_t k = i + u * G;
            const int64_t row = k / per_row, c = k - row * per_row;
            q[u] = k < nvec ? __builtin_nontemporal_load((const u32x4*)(ns + row * STRIDE + BEGIN) + c) : u32x4{~0u, ~0u, ~0u, ~0u};
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) m = min(m, min(min(q[u].x, q[u].y), min(q[u].z, q[u].w)));
    }
    m = wmin(m);
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = m;
}

template <class F>
float timeit(F&& f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    uint32_t* ns;
    unsigned* out;
    CK(hipMalloc(&ns, ROWS * STRIDE * 4));
    CK(hipMalloc(&out, 1 << 24));
    CK(hipMemset(ns, 0x11, ROWS * STRIDE * 4));
    const double bytes = (double)ROWS * KEEP * 4;
    const int reps = 20;
    const dim3 g((unsigned)((ROWS + 3) / 4)), blk(256);
    struct V {
        const char* name;
        float ms;
    };
    float t;
    t = timeit([&] { hipLaunchKernelGGL((seg_wave<128, 3>), g, blk, 0, 0, ns, out); }, reps);
    printf("seg_wave PL128 W3 (stats kernel pattern): %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((seg_wave<64, 4>), g, blk, 0, 0, ns, out); }, reps);
    printf("seg_wave PL64 W4 (2 passes):             %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
    t = timeit([&] { hipLaunchKernelGGL((seg_wave<32, 8>), g, blk, 0, 0, ns, out); }, reps);
    printf("seg_wave PL32 W8 (4 passes):             %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
    const int64_t nvec = ROWS * (KEEP / 4);
    for (int bpc : {4, 8, 16}) {
        const unsigned blocks = 256u * bpc;
        t = timeit([&] { hipLaunchKernelGGL((flat<8>), dim3(blocks), blk, 0, 0, ns, out, nvec); }, reps);
        printf("flat grid-stride UNR8 %2d blocks/CU:       %.3f ms  %.0f GB/s\n", bpc, t, bytes / t / 1e6);
        t = timeit([&] { hipLaunchKernelGGL((flat<16>), dim3(blocks), blk, 0, 0, ns, out, nvec); }, reps);
        printf("flat grid-stride UNR16 %2d blocks/CU:      %.3f ms  %.0f GB/s\n", bpc, t, bytes / t / 1e6);
    }
    CK(hipFree(ns));
    CK(hipFree(out));
    return 0;
}
