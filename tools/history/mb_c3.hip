// mb_c3.hip -- microbenchmark of launch shapes for the strided stats kernel (default C3: 4096 x 2048 x 1024
// u32 samples, one 4 KB segment per wave).  Builds against csrc/segment_kernels.h; every
// variant's outputs are compared bit for bit with the production kernel's.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../nvidia-resiliency-ext-x_amd/csrc
//         mb_c3.hip -o mb_c3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <vector>

#include "segment_kernels.h"
#include "../../include/nvrx_synth.h"

using namespace nvrx;

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__device__ __forceinline__ uint64_t smix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void gen(uint32_t* ns, int64_t nseg, int S, int K) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nseg * S;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t seg = i / S;
    const uint64_t k = (uint64_t)(seg % K);
    const uint64_t base = 2000 + smix(0xBA5E ^ k) % 1998000;
    const uint64_t u = smix(0x5EED ^ (uint64_t)i);
    ns[i] = (uint32_t)(base + (((u >> 32) * (base / 10)) >> 32));
  }
}

// G segments per wave, WPB waves per block; loads of all G segments issued first.
template <int PL, int G, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(G == 1 ? Occ<PL>::W : G == 2 ? 6 : 4)))
void seg_multi(StridedSegs segs, int64_t nseg, nvrx_stats_soa out, ColRef cr) {
    constexpr int NB = Bins<PL>::NB;
    __shared__ __attribute__((aligned(16))) unsigned lds_hist[WPB * NB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned* hist = lds_hist + wave * NB;
    const int64_t s0 = ((int64_t)blockIdx.x * WPB + wave) * G;
    unsigned v[G][PL];
    const uint32_t* p[G];
    int n[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if (s0 + g < nseg) {
            segs.get(s0 + g, p[g], n[g]);
            issue_loads<PL>(p[g], n[g], v[g]);
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if (s0 + g >= nseg) return;
        int m0;
        unsigned x0;
        finish_loads<PL, true>(p[g], n[g], v[g], m0, x0);
        fast_body<PL, true>(v[g], n[g], m0, x0, s0 + g, hist, out, cr);
    }
}

// G segments per wave through lean_body, all G segments' loads issued first
template <int PL, int G, int WPB, int OCC>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(OCC)))
void lean_multi(StridedSegs segs, int64_t nseg, nvrx_stats_soa out, ColRef cr) {
    constexpr int NB = Bins<PL>::NB;
    __shared__ __attribute__((aligned(16))) unsigned lds_hist[WPB * NB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned* hist = lds_hist + wave * NB;
    const int64_t s0 = ((int64_t)blockIdx.x * WPB + wave) * G;
    unsigned v[G][PL];
    const uint32_t* p[G];
    int n[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if (s0 + g < nseg) {
            segs.get(s0 + g, p[g], n[g]);
            issue_loads<PL>(p[g], n[g], v[g]);
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if (s0 + g >= nseg) return;
        int m0;
        unsigned x0;
        finish_loads<PL, true>(p[g], n[g], v[g], m0, x0);
        lean_body<PL>(v[g], n[g], x0, s0 + g, hist, out, cr);
    }
}

// persistent: each wave walks segments w, w + W, ... with the next segment's loads in flight
template <int PL, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(6)))
void seg_persist(StridedSegs segs, int64_t nseg, nvrx_stats_soa out, ColRef cr) {
    constexpr int NB = Bins<PL>::NB;
    __shared__ __attribute__((aligned(16))) unsigned lds_hist[WPB * NB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned* hist = lds_hist + wave * NB;
    const int64_t W = (int64_t)gridDim.x * WPB;
    int64_t s = (int64_t)blockIdx.x * WPB + wave;
    if (s >= nseg) return;
    unsigned a[PL], b[PL];
    const uint32_t* p;
    int n;
    segs.get(s, p, n);
    issue_loads<PL>(p, n, a);
    for (;;) {
        const int64_t sn = s + W;
        const uint32_t* pn = p;
        int nn = n;
        if (sn < nseg) {
            segs.get(sn, pn, nn);
            issue_loads<PL>(pn, nn, b);
        }
        int m0;
        unsigned x0;
        finish_loads<PL, true>(p, n, a, m0, x0);
        fast_body<PL, true>(a, n, m0, x0, s, hist, out, cr);
        if (sn >= nseg) return;
#pragma unroll
        for (int i = 0; i < PL; ++i) a[i] = b[i];
        s = sn;
        p = pn;
        n = nn;
    }
}

// persistent lean waves, next segment's loads in flight while the current one is reduced
template <int PL, int WPB, int OCC>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(OCC)))
void lean_persist(StridedSegs segs, int64_t nseg, nvrx_stats_soa out, ColRef cr) {
    constexpr int NB = Bins<PL>::NB;
    __shared__ __attribute__((aligned(16))) unsigned lds_hist[WPB * NB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned* hist = lds_hist + wave * NB;
    const int64_t W = (int64_t)gridDim.x * WPB;
    int64_t s = (int64_t)blockIdx.x * WPB + wave;
    if (s >= nseg) return;
    unsigned a[PL], b[PL];
    const uint32_t* p;
    int n;
    segs.get(s, p, n);
    issue_loads<PL>(p, n, a);
    for (;;) {
        const int64_t sn = s + W;
        const uint32_t* pn = p;
        int nn = n;
        if (sn < nseg) {
            segs.get(sn, pn, nn);
            issue_loads<PL>(pn, nn, b);
        }
        int m0;
        unsigned x0;
        finish_loads<PL, true>(p, n, a, m0, x0);
        lean_body<PL>(a, n, x0, s, hist, out, cr);
        if (sn >= nseg) return;
#pragma unroll
        for (int i = 0; i < PL; ++i) a[i] = b[i];
        s = sn;
        p = pn;
        n = nn;
    }
}

// streaming ceiling at this granularity: load the 4 KB segment, one store per segment
template <int PL, int WPB>
__global__ __launch_bounds__(64 * WPB) void read_only(StridedSegs segs, int64_t nseg, unsigned* out) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t s = (int64_t)blockIdx.x * WPB + wave;
    if (s >= nseg) return;
    const uint32_t* p;
    int n;
    segs.get(s, p, n);
    unsigned v[PL];
    issue_loads<PL>(p, n, v);
    unsigned m = v[0];
#pragma unroll
    for (int i = 1; i < PL; ++i) m = min(m, v[i]);
    m = wave_min_u32(m);
    if (lane_id() == 0) out[s] = m;
}

template <int WPB>
__global__ __launch_bounds__(64 * WPB) void empty_k(int64_t nseg, unsigned* out) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t s = (int64_t)blockIdx.x * WPB + wave;
    if (s < nseg && lane_id() == 0) out[s] = (unsigned)s;
}

struct Soa {
    void* mem;
    nvrx_stats_soa soa;
    Soa(int64_t n) {
        CK(hipMalloc(&mem, (size_t)n * 24));
        char* b = (char*)mem;
        soa = nvrx_stats_soa{(int32_t*)b, (float*)(b + 4 * n), (float*)(b + 8 * n), (float*)(b + 12 * n),
                             (float*)(b + 16 * n), (float*)(b + 20 * n)};
    }
};

template <class F>
float timeit(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

template <int PL>
int run(int64_t R, int64_t K, bool prod_data, int reps) {
    const int S = 64 * PL;
    const int64_t nseg = R * K;
    uint32_t* ns;
    CK(hipMalloc(&ns, (size_t)nseg * S * 4));
    if (prod_data) {  // the production generator (libnvrx_synth.so)
        if (nvrx_synth_matrix(ns, R, K, K, nullptr, S, 0x5EED, 0xBA5E, nullptr, nullptr) != 0) return 1;
        std::printf("data: nvrx_synth_matrix R=%ld K=%ld S=%d\n", (long)R, (long)K, S);
    } else {
        gen<<<65536, 256>>>(ns, nseg, S, (int)K);
        std::printf("data: local gen R=%ld K=%ld S=%d\n", (long)R, (long)K, S);
    }
    CK(hipDeviceSynchronize());
    StridedSegs segs{ns, S, 0, S, 8192};
    ColRef cr{nullptr, nullptr, 1, 1.0};
    Soa ref(nseg), got(nseg);
    unsigned* scratch;
    CK(hipMalloc(&scratch, (size_t)nseg * 4));
    const double gb = (double)nseg * S * 4 / 1e9;
    std::vector<char> h0((size_t)nseg * 24), h1((size_t)nseg * 24);
    auto report = [&](const char* name, float ms, bool check) {
        const char* verdict = "";
        if (check) {
            CK(hipMemcpy(h0.data(), ref.mem, h0.size(), hipMemcpyDeviceToHost));
            CK(hipMemcpy(h1.data(), got.mem, h1.size(), hipMemcpyDeviceToHost));
            verdict = h0 == h1 ? "bit-exact" : "MISMATCH";
            if (h0 != h1) {
                // per field: differing segments; for the float fields the largest relative diff
                for (int f = 0; f < 6; ++f) {
                    size_t nd = 0;
                    double rel = 0.0;
                    for (int64_t k = 0; k < nseg; ++k) {
                        const size_t i = ((size_t)f * nseg + k) * 4;
                        if (std::memcmp(&h0[i], &h1[i], 4) == 0) continue;
                        ++nd;
                        if (f > 0) {
                            float a, b;
                            std::memcpy(&a, &h0[i], 4);
                            std::memcpy(&b, &h1[i], 4);
                            const double r = std::fabs((double)a - (double)b) / std::fabs((double)a);
                            if (r > rel) rel = r;
                        }
                    }
                    if (nd) std::printf("  field %d: %zu segments differ, max rel %.3g\n", f, nd, rel);
                }
            }
            CK(hipMemset(got.mem, 0xFF, h1.size()));
        }
        std::printf("%-28s %8.3f ms %6.2f TB/s %s\n", name, ms, gb / ms, verdict);
        std::fflush(stdout);
    };
    const unsigned g4 = (unsigned)((nseg + 3) / 4);
    for (int rep = 0; rep < 4; ++rep) {
        report("v0 fast_body", timeit([&] {
                   hipLaunchKernelGGL((seg_stats_fast_kernel<PL, true, StridedSegs>), dim3(g4), dim3(256), 0, 0, segs, nseg, ref.soa, cr);
               }, reps), false);
        report("v4 lean_body", timeit([&] {
                   hipLaunchKernelGGL((seg_stats_lean_kernel<PL, StridedSegs>), dim3(g4), dim3(256), 0, 0, segs, nseg, got.soa, cr);
               }, reps), true);
        if (PL <= 32) {
            report("m2o8 lean 2 seg/wave occ8", timeit([&] {
                       hipLaunchKernelGGL((lean_multi<PL, 2, 4, 8>), dim3((unsigned)((nseg + 7) / 8)), dim3(256), 0, 0, segs, nseg, got.soa, cr);
                   }, reps), true);
            report("m2o6 lean 2 seg/wave occ6", timeit([&] {
                       hipLaunchKernelGGL((lean_multi<PL, 2, 4, 6>), dim3((unsigned)((nseg + 7) / 8)), dim3(256), 0, 0, segs, nseg, got.soa, cr);
                   }, reps), true);
            report("m4o4 lean 4 seg/wave occ4", timeit([&] {
                       hipLaunchKernelGGL((lean_multi<PL, 4, 4, 4>), dim3((unsigned)((nseg + 15) / 16)), dim3(256), 0, 0, segs, nseg, got.soa, cr);
                   }, reps), true);
        }
    }
    report("read-only", timeit([&] {
               hipLaunchKernelGGL((read_only<PL, 4>), dim3(g4), dim3(256), 0, 0, segs, nseg, scratch);
           }, reps), false);
    CK(hipFree(ns));
    CK(hipFree(ref.mem));
    CK(hipFree(got.mem));
    CK(hipFree(scratch));
    return 0;
}

int main(int argc, char** argv) {
    // mb_c3 [R] [s|l] [PL] [reps]: R ranks x 2048 kernels x 64*PL samples
    const int64_t R = argc > 1 ? atoll(argv[1]) : 4096, K = 2048;
    const bool prod = !(argc > 2 && argv[2][0] == 'l');
    const int pl = argc > 3 ? atoi(argv[3]) : 16;
    const int reps = argc > 4 ? atoi(argv[4]) : 5;
    if (pl == 16) return run<16>(R, K, prod, reps);
    if (pl == 32) return run<32>(R, K, prod, reps);
    if (pl == 64) return run<64>(R, K, prod, reps);
    if (pl == 128) return run<128>(R, K, prod, reps);
    return 2;
}
