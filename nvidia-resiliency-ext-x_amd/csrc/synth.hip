// synth.hip -- TEST / BENCH INFRASTRUCTURE (libnvrx_synth.so): device generator of the
// synthetic integer-ns duration matrix, bit-identical to oracle/nvrx_oracle.c.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nvrx_synth.h"

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// one thread per 4 consecutive samples of one (r, kk) row; grid-stride over rows*vectors
__global__ void synth_matrix_kernel(uint32_t* out, int64_t R, int64_t K_local, int64_t K_global,
                                    const int64_t* kmap, int64_t s_push, uint64_t seed,
                                    uint64_t seed2, const uint8_t* straggler) {
    const int64_t total = R * K_local * s_push;
    for (int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; e < total;
         e += (int64_t)gridDim.x * blockDim.x * 4) {
        const int64_t row = e / s_push;
        int64_t i = e - row * s_push;
        const int64_t r = row / K_local;
        const int64_t kk = row - r * K_local;
        const int64_t k = kmap ? kmap[kk] : kk;
        const uint64_t base = 2000ull + splitmix64(seed2 ^ (uint64_t)k) % 1998000ull;
        const bool strag = straggler && straggler[r];
        for (int t = 0; t < 4; ++t) {
            const int64_t ee = e + t;
            if (ee >= total) break;
            int64_t rr = row, ii = i + t;
            uint64_t b = base;
            int64_t kg = k, rk = r;
            bool st = strag;
            if (ii >= s_push) {  // crossed into the next row (s_push not a multiple of 4)
                rr = ee / s_push;
                ii = ee - rr * s_push;
                rk = rr / K_local;
                const int64_t kl = rr - rk * K_local;
                kg = kmap ? kmap[kl] : kl;
                b = 2000ull + splitmix64(seed2 ^ (uint64_t)kg) % 1998000ull;
                st = straggler && straggler[rk];
            }
            const uint64_t u = splitmix64(seed ^ (((uint64_t)rk * (uint64_t)K_global + (uint64_t)kg) *
                                                      (uint64_t)s_push + (uint64_t)ii));
            uint64_t ns = b + (((u >> 32) * (b / 10ull)) >> 32);
            if (st) ns = ns * 13ull / 10ull;
            out[ee] = (uint32_t)ns;
        }
    }
}

// record streams: out[r*N + j] = {slot[j], ns(r, slot[j], occ[j])}, the occ[j]-th push of
// kernel slot[j] on rank r (same sample hash as the matrix with S_push = s_push)
__global__ void synth_records_kernel(uint32_t* out, int64_t R, int64_t N, const uint32_t* slot,
                                     const uint32_t* kglob, const uint32_t* occ, int64_t K,
                                     int64_t s_push, uint64_t seed, uint64_t seed2,
                                     const uint8_t* straggler) {
    const int64_t total = R * N;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / N;
        const int64_t j = e - r * N;
        const uint64_t k = kglob ? kglob[j] : slot[j];
        const uint64_t base = 2000ull + splitmix64(seed2 ^ k) % 1998000ull;
        const uint64_t u = splitmix64(seed ^ (((uint64_t)r * (uint64_t)K + k) * (uint64_t)s_push +
                                              (uint64_t)occ[j]));
        uint64_t ns = base + (((u >> 32) * (base / 10ull)) >> 32);
        if (straggler && straggler[r]) ns = ns * 13ull / 10ull;
        out[2 * e] = slot[j];
        out[2 * e + 1] = (uint32_t)ns;
    }
}

}  // namespace

extern "C" int nvrx_synth_records(uint32_t* out, int64_t R, int64_t N, const uint32_t* slot,
                                  const uint32_t* kglob, const uint32_t* occ, int64_t K,
                                  int64_t s_push, uint64_t seed, uint64_t seed2,
                                  const uint8_t* straggler, void* stream) {
    if (!out || !slot || !occ || R < 0 || N < 0) return -1;
    const int64_t total = R * N;
    if (total == 0) return 0;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(synth_records_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, out, R, N, slot, kglob, occ, K, s_push, seed, seed2,
                       straggler);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int nvrx_synth_matrix(uint32_t* out, int64_t R, int64_t K_local, int64_t K_global,
                                 const int64_t* kmap, int64_t s_push, uint64_t seed,
                                 uint64_t seed2, const uint8_t* straggler, void* stream) {
    if (!out || R < 0 || K_local < 0 || s_push < 0) return -1;
    const int64_t total = R * K_local * s_push;
    if (total == 0) return 0;
    int64_t blocks = (total / 4 + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(synth_matrix_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, out, R, K_local, K_global, kmap, s_push, seed, seed2,
                       straggler);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
