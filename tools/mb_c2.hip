// mb_c2.hip -- HBM read ceiling for the configs[2] bytes (4096 x 2048 segments of 1024 u32,
// 34.4 GB, contiguous): the statistics kernels' access patterns with a trivial reduction.
//   (a) one wave per 4 KB segment (4 x 16-B loads per lane), 8 waves / SIMD
//   (b) one wave per G consecutive segments, one after another (the group kernel's pattern)
//   (c) as (b) with the next segment's loads issued before the current one is reduced
//   (d) flat grid-stride 16-B sweep
// and for the configs[1] bytes (64 x 2048 rows of 10,000 u32, the last 8192 of each read):
//   (e) one wave per 32 KB row segment (the PL = 128 kernel's pattern, 3 waves / SIMD)
//   (f) P waves per row segment, each 32/P KB (P = 2, 4, 8)
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/mb_c2 tools/mb_c2.hip && tools/build/mb_c2
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

constexpr int64_t NSEG = 4096LL * 2048, LEN = 1024;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const uint32_t* p) {
    const uintptr_t pa = (uintptr_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)pa);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(pa >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, LEN * 4, 0x00020000);
}
__device__ __forceinline__ void load4(const uint32_t* p, u32x4 (&q)[4]) {
    const auto r = rsrc_of(p);
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, j * 1024, 2);
}
__device__ __forceinline__ unsigned red(const u32x4 (&q)[4]) {
    unsigned m = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) m ^= q[j].x + q[j].y + q[j].z + q[j].w;
    return m;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8)))
void per_segment(const uint32_t* ns, unsigned* out) {
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= NSEG) return;
    u32x4 q[4];
    load4(ns + s * LEN, q);
    const unsigned m = red(q);
    if (m == 0x12345678u) out[s] = m;
}

template <bool PREFETCH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8)))
void grouped(const uint32_t* ns, unsigned* out, int G) {
    const int64_t s0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * G;
    if (s0 >= NSEG) return;
    unsigned m = 0;
    u32x4 q[4];
    load4(ns + s0 * LEN, q);
    for (int j = 0; j < G; ++j) {
        if (PREFETCH) {
            u32x4 w[4];
            load4(ns + (s0 + (j + 1 < G ? j + 1 : j)) * LEN, w);
            m ^= red(q);
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = w[k];
        } else {
            if (j) load4(ns + (s0 + j) * LEN, q);
            m ^= red(q);
        }
    }
    if (m == 0x12345678u) out[s0] = m;
}

__global__ __launch_bounds__(256) void sweep(const u32x4* ns, int64_t n16, unsigned* out) {
    unsigned m = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const u32x4 v = __builtin_nontemporal_load(ns + i);
        m ^= v.x + v.y + v.z + v.w;
    }
    if (m == 0x12345678u) out[0] = m;
}

constexpr int64_t ROWS1 = 64 * 2048, STRIDE1 = 10000, KEEP1 = 8192, BEGIN1 = STRIDE1 - KEEP1;

// P waves per row: wave w of the row reads samples [w * KEEP1 / P, (w + 1) * KEEP1 / P)
template <int P, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W)))
void row_split(const uint32_t* ns, unsigned* out) {
    constexpr int PL = 128 / P;  // samples per lane
    const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t row = g / P;
    const int part = (int)(g % P);
    if (row >= ROWS1) return;
    const int lane = threadIdx.x & 63;
    const uint32_t* p = ns + row * STRIDE1 + BEGIN1 + part * (KEEP1 / P);
    const uintptr_t pa = (uintptr_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)pa);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(pa >> 32));
    const auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, KEEP1 / P * 4, 0x00020000);
    unsigned v[PL];
#pragma unroll
    for (int j = 0; j < PL / 4; ++j) {
        const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, j * 1024, 2);
        v[4 * j] = q.x, v[4 * j + 1] = q.y, v[4 * j + 2] = q.z, v[4 * j + 3] = q.w;
    }
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < PL; ++i) m ^= v[i];
    if (m == 0x12345678u) out[g] = m;
}

// (g) 4 waves per row (PLW = 32) plus ITER x 32 dependent VALU per wave after the loads (a
//     stand-in for the statistics), one row per workgroup or (PREF) a persistent workgroup over
//     rows with the next row's loads issued before the current row's "reduction"
template <int ITER, bool PREF, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W)))
void row_compute(const uint32_t* ns, unsigned* out, int64_t rows_per_block) {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    auto load = [&](int64_t row, unsigned (&v)[32]) {
        const uint32_t* p = ns + row * STRIDE1 + BEGIN1 + wave * 2048;
        const uintptr_t pa = (uintptr_t)p;
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)pa);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(pa >> 32));
        const auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 8192, 0x00020000);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, j * 1024, 2);
            v[4 * j] = q.x, v[4 * j + 1] = q.y, v[4 * j + 2] = q.z, v[4 * j + 3] = q.w;
        }
    };
    auto work = [&](const unsigned (&v)[32]) {
        float x = (float)lane;
        for (int k = 0; k < ITER; ++k) {
#pragma unroll
            for (int i = 0; i < 32; ++i) x = __builtin_fmaf(x, 0.999f, __builtin_bit_cast(float, v[i] & 0x3FFFFFFFu));
        }
        return x;
    };
    float acc = 0.0f;
    unsigned v[32];
    if (PREF) {
        load(r0, v);
        for (int64_t j = 0; j < rows_per_block && r0 + j < ROWS1; ++j) {
            unsigned w[32];
            load(r0 + j + 1 < ROWS1 && j + 1 < rows_per_block ? r0 + j + 1 : r0 + j, w);
            acc += work(v);
#pragma unroll
            for (int i = 0; i < 32; ++i) v[i] = w[i];
        }
    } else {
        for (int64_t j = 0; j < rows_per_block && r0 + j < ROWS1; ++j) {
            load(r0 + j, v);
            acc += work(v);
        }
    }
    if (acc == 1.2345f) out[blockIdx.x] = 1;
}

int main() {
    const size_t bytes = (size_t)NSEG * LEN * 4;
    uint32_t* ns;
    unsigned* out;
    CK(hipMalloc(&ns, bytes));
    CK(hipMalloc(&out, NSEG * 4));
    CK(hipMemset(ns, 1, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(a);
        const int reps = 10;
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        ms /= reps;
        printf("%-28s %.3f ms  %.0f GB/s\n", name, ms, bytes / (ms * 1e6));
        return 0;
    };
    for (int rep = 0; rep < 2; ++rep) {
        timeit("per_segment", [&] { per_segment<<<NSEG / 4, 256>>>(ns, out); });
        for (int G : {4, 16, 64}) {
            char nm[64];
            snprintf(nm, sizeof nm, "grouped G=%d", G);
            timeit(nm, [&] { grouped<false><<<(NSEG / G + 3) / 4, 256>>>(ns, out, G); });
            snprintf(nm, sizeof nm, "grouped+prefetch G=%d", G);
            timeit(nm, [&] { grouped<true><<<(NSEG / G + 3) / 4, 256>>>(ns, out, G); });
        }
        timeit("sweep 4096x256", [&] { sweep<<<4096, 256>>>((const u32x4*)ns, (int64_t)bytes / 16, out); });
        timeit("sweep 16384x256", [&] { sweep<<<16384, 256>>>((const u32x4*)ns, (int64_t)bytes / 16, out); });
    }
    const double b1 = (double)ROWS1 * KEEP1 * 4;
    auto time1 = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(a);
        const int reps = 50;
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        ms /= reps;
        printf("cfg1 %-23s %.4f ms  %.0f GB/s\n", name, ms, b1 / (ms * 1e6));
    };
    for (int rep = 0; rep < 2; ++rep) {
        time1("row P=1 W3", [&] { row_split<1, 3><<<ROWS1 / 4, 256>>>(ns, out); });
        time1("row P=2 W4", [&] { row_split<2, 4><<<ROWS1 * 2 / 4, 256>>>(ns, out); });
        time1("row P=4 W8", [&] { row_split<4, 8><<<ROWS1 * 4 / 4, 256>>>(ns, out); });
        time1("row P=8 W8", [&] { row_split<8, 8><<<ROWS1 * 8 / 4, 256>>>(ns, out); });
    }
    for (int rep = 0; rep < 2; ++rep) {
        time1("P4 work0", [&] { row_compute<0, false, 8><<<ROWS1, 256>>>(ns, out, 1); });
        time1("P4 work8", [&] { row_compute<8, false, 8><<<ROWS1, 256>>>(ns, out, 1); });
        time1("P4 work16", [&] { row_compute<16, false, 8><<<ROWS1, 256>>>(ns, out, 1); });
        time1("P4 work32", [&] { row_compute<32, false, 8><<<ROWS1, 256>>>(ns, out, 1); });
        for (int rpb : {4, 16}) {
            char nm[64];
            snprintf(nm, sizeof nm, "P4 work8 pref rpb%d W6", rpb);
            time1(nm, [&] { row_compute<8, true, 6><<<ROWS1 / rpb, 256>>>(ns, out, rpb); });
            snprintf(nm, sizeof nm, "P4 work16 pref rpb%d W6", rpb);
            time1(nm, [&] { row_compute<16, true, 6><<<ROWS1 / rpb, 256>>>(ns, out, rpb); });
            snprintf(nm, sizeof nm, "P4 work16 seq rpb%d W8", rpb);
            time1(nm, [&] { row_compute<16, false, 8><<<ROWS1 / rpb, 256>>>(ns, out, rpb); });
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
