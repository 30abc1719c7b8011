// segment_ragged_kernels.h -- the length-class kernels of segment_ragged.hip, shared by the
// translation units that instantiate them (segment_ragged*.hip: split so that the heavy
// template instantiations -- 128-sample sorting networks, PL = 64/128 wave bodies -- compile
// in parallel).  See segment_ragged.hip for the algorithm.
#pragma once
#include <algorithm>
#include <mutex>

#include "segment_kernels.h"

namespace nvrx {
namespace ragged {
namespace {  // internal linkage: every translation unit keeps its own copy

int cu_count();  // CUs of the current device (below)


constexpr int CLS_THREADS = 1024;
constexpr int CLS_MAX_BLOCKS = 1024;
// segment lengths loaded per thread before any is classified: a block's chunk is tens of
// thousands of segments, and one dependent load per 1024 of them left both passes
// latency-bound (configs[3]: 153 + 118 us for 33.5 M segments)
#ifndef NVRX_CLS_BATCH  // build-time tuning constant
#define NVRX_CLS_BATCH 8
#endif
constexpr int CLS_BATCH = NVRX_CLS_BATCH;
static_assert(CLS_BATCH >= 1 && CLS_BATCH < 16 && 4 * NCLASS <= 64, "4-bit packed class counts per batch");


// pass 1: per-block class counts (bcnt[b][c]); empty segments are written here
__global__ __launch_bounds__(CLS_THREADS) void classify_count_kernel(
    RaggedSegs segs, int64_t nseg, int64_t chunk, int aligned16, int exact, int full_n, uint32_t* bcnt,
    nvrx_stats_soa out) {
    const ColRef cr{nullptr, nullptr, 1, 1.0};  // column references: kernel_ref afterwards
    __shared__ uint32_t lcnt[NCLASS];
    if (threadIdx.x < NCLASS) lcnt[threadIdx.x] = 0u;
    __syncthreads();
    const int64_t lo = (int64_t)blockIdx.x * chunk;
    const int64_t hi = min(nseg, lo + chunk);
    // per-lane class counters in registers (no LDS traffic per segment), one wave reduction
    // and one LDS add per class at the end
    unsigned mine[NCLASS];
#pragma unroll
    for (int c = 0; c < NCLASS; ++c) mine[c] = 0u;
    for (int64_t b = lo; b < hi; b += CLS_THREADS * CLS_BATCH) {
        int n[CLS_BATCH];
#pragma unroll
        for (int j = 0; j < CLS_BATCH; ++j) {
            const int64_t s = b + j * CLS_THREADS + threadIdx.x;
            n[j] = s < hi ? segs.kept_len(s) : -1;
        }
        // the batch's class counts packed 4 bits per class in one 64-bit word (one shift and
        // add per segment instead of a compare and add per class), unpacked once per batch
        uint64_t pk = 0;
#pragma unroll
        for (int j = 0; j < CLS_BATCH; ++j) {
            const int64_t s = b + j * CLS_THREADS + threadIdx.x;
            if (n[j] == 0) {
                write_empty(out, s);
                cr.miss(s);
            } else if (n[j] > 0) {  // n < 0: reduced elsewhere (or past the chunk)
                pk += 1ull << (4 * seg_class(n[j], aligned16 != 0, exact != 0, full_n));
            }
        }
#pragma unroll
        for (int c = 0; c < NCLASS; ++c) mine[c] += (uint32_t)(pk >> (4 * c)) & 15u;
    }
#pragma unroll
    for (int c = 0; c < NCLASS; ++c) {
        const unsigned w = wave_sum_u32(mine[c]);
        if (lane_id() == 0 && w) atomicAdd(&lcnt[c], w);
    }
    __syncthreads();
    if (threadIdx.x < NCLASS) bcnt[(int64_t)blockIdx.x * NCLASS + threadIdx.x] = lcnt[threadIdx.x];
}

// pass 2 (one block): boff[b][c] = start of class c + blocks before b; cls[c] = {start, count}
__global__ __launch_bounds__(CLS_MAX_BLOCKS) void classify_scan_kernel(uint32_t* bcnt, int nblocks,
                                                                       uint32_t* cls) {
    __shared__ uint32_t wsum[CLS_MAX_BLOCKS / 64];
    const int b = threadIdx.x;
    const int w = b >> 6;
    uint32_t start = 0;
    for (int c = 0; c < NCLASS; ++c) {
        const uint32_t v = b < nblocks ? bcnt[(int64_t)b * NCLASS + c] : 0u;
        const uint32_t incl = wave_incl_scan_u32(v);
        if (lane_id() == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (int j = 0; j < CLS_MAX_BLOCKS / 64; ++j) {
            before += j < w ? wsum[j] : 0u;
            all += wsum[j];
        }
        if (b < nblocks) bcnt[(int64_t)b * NCLASS + c] = start + before + incl - v;
        if (b == 0) {
            cls[2 * c] = start;
            cls[2 * c + 1] = all;
        }
        start += all;
        __syncthreads();
    }
}

// pass 3: scatter segment ids into the class-ordered list
__global__ __launch_bounds__(CLS_THREADS) void classify_scatter_kernel(
    RaggedSegs segs, int64_t nseg, int64_t chunk, int aligned16, int exact, int full_n, const uint32_t* boff,
    uint32_t* list) {
    __shared__ uint32_t lcnt[NCLASS];
    __shared__ uint32_t lbase[NCLASS];
    if (threadIdx.x < NCLASS) {
        lcnt[threadIdx.x] = 0u;
        lbase[threadIdx.x] = boff[(int64_t)blockIdx.x * NCLASS + threadIdx.x];
    }
    __syncthreads();
    const int64_t lo = (int64_t)blockIdx.x * chunk;
    const int64_t hi = min(nseg, lo + chunk);
    for (int64_t b = lo; b < hi; b += CLS_THREADS * CLS_BATCH) {
        int n[CLS_BATCH];
#pragma unroll
        for (int j = 0; j < CLS_BATCH; ++j) {
            const int64_t s = b + j * CLS_THREADS + threadIdx.x;
            n[j] = s < hi ? segs.kept_len(s) : -1;
        }
#pragma unroll
        for (int j = 0; j < CLS_BATCH; ++j) {  // the same order as the counting pass
            const int64_t s = b + j * CLS_THREADS + threadIdx.x;
            const int cls = n[j] > 0 ? seg_class(n[j], aligned16 != 0, exact != 0, full_n) : -1;
            const uint32_t r = wave_class_add(lcnt, cls);
            if (cls >= 0) list[lbase[cls] + r] = (uint32_t)s;
        }
    }
}

// ---------------------------------------------------------------- lane classes
template <int N>
struct LaneOcc {
    static constexpr int W = N >= 128 ? 2 : N >= 64 ? 4 : N >= 32 ? 6 : 8;
};

// The shortest segment of a lane class (seg_class): n <= 8, then (N/2, N].
template <int N>
struct LaneMin {
    static constexpr int n = N >= 16 ? N / 2 + 1 : 1;
};

// Segments per lane per step: each takes a chain of three dependent loads (list entry,
// descriptor, samples), so the shortest class runs B chains side by side.
template <int N>
struct LaneBatch {
    static constexpr int B = N <= 8 ? 4 : N <= 16 ? 2 : 1;  // 2 for N = 32: 189 -> 214 us (configs[3])
};

// One lane per segment of 1..N samples.  u32 -> f32 us is monotone, so sorting the
// integer ns sorts the floats computeStats sorts; then CuptiProfiler.cpp:53-71.
template <int N>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LaneOcc<N>::W)))
void seg_stats_lane_kernel(RaggedSegs segs, const uint32_t* list, const uint32_t* cls,
                           int aligned16, nvrx_stats_soa out) {
    const ColRef cr{nullptr, nullptr, 1, 1.0};  // column references: kernel_ref afterwards
    constexpr int B = LaneBatch<N>::B;
    // 32-bit list indices (a 64-bit loop cost lane<8> 315 -> 372 us); the host keeps the
    // segment count below 2^32 - 2^26, so i + B * G never wraps
    const uint32_t start = cls[0], cnt = cls[1];
    const uint32_t G = gridDim.x * 256u;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < cnt; i += B * G) {
        int64_t s[B];
        const uint32_t* p[B];
        int n[B];
#pragma unroll
        for (int b = 0; b < B; ++b) s[b] = i + b * G < cnt ? (int64_t)list[start + i + b * G] : -1;
#pragma unroll
        for (int b = 0; b < B; ++b) {
            n[b] = 0;
            p[b] = nullptr;
            if (s[b] >= 0) segs.get(s[b], p[b], n[b]);  // 1 <= n <= N
        }
        unsigned v[B][N];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            if (aligned16) {
                const u32x4* q = (const u32x4*)p[b];
#pragma unroll
                for (int j = 0; j < N / 4; ++j) {
                    u32x4 w = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
                    if (4 * j < n[b]) w = q[j];
                    v[b][4 * j + 0] = w.x;
                    v[b][4 * j + 1] = w.y;
                    v[b][4 * j + 2] = w.z;
                    v[b][4 * j + 3] = w.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < N; ++j) v[b][j] = j < n[b] ? p[b][j] : 0xFFFFFFFFu;
            }
        }
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (s[b] >= 0) lane_stats<N, LaneMin<N>::n>(v[b], n[b], s[b], out, cr);
    }
}

// ---------------------------------------------------------------- wave / workgroup classes
// One wave per segment over a class list.  Waves take chunks of CH consecutive list
// entries (static round robin; CH shrinks when the class is small so every wave gets
// work); lanes 0..CH-1 fetch the chunk's segment descriptors in one coalesced access, so
// per segment the only dependent memory access is the data itself -- and for PL <= 16
// (short segments, few registers) the next segment's loads are issued before the
// current one is reduced.
template <int PL>
struct ListPrefetch {
    static constexpr bool on = PL <= 16;
};
template <int PL>
struct ListKeepBin {  // level-0 bins in registers while they fit beside the prefetch buffer
    static constexpr bool on = PL <= 8;
};
template <int PL>
struct ListGroup {  // one epilogue per chunk (emit_lane): the short classes, whose chunks are long
    static constexpr bool on = PL <= 8;
};
#ifndef NVRX_LIST4_OCC  // build-time tuning constants: waves per SIMD of list<4> / list<8>
#define NVRX_LIST4_OCC 8
#endif
#ifndef NVRX_LIST8_OCC
#define NVRX_LIST8_OCC 7
#endif
template <int PL>
struct ListOcc {  // the prefetch buffer costs PL more VGPRs, the chunk's results nine
    static constexpr int W = PL == 16 ? 6 : PL == 8 ? NVRX_LIST8_OCC : PL == 4 ? NVRX_LIST4_OCC : OccV<PL, false>::W;
};
#ifndef NVRX_LIST_CHUNK  // build-time tuning constant (tools/build_variant.sh)
#define NVRX_LIST_CHUNK 16
#endif
constexpr int LIST_CHUNK = NVRX_LIST_CHUNK;
// results are held one per lane and the wide-key flags in a 32-bit mask
static_assert(LIST_CHUNK >= 1 && LIST_CHUNK <= 32, "NVRX_LIST_CHUNK must be in [1, 32]");

template <int PL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ListOcc<PL>::W)))
void seg_stats_list_kernel(RaggedSegs segs, const uint32_t* list, const uint32_t* cls,
                           nvrx_stats_soa out) {
    const ColRef cr{nullptr, nullptr, 1, 1.0};  // column references: kernel_ref afterwards
    constexpr int NB = Bins<PL>::NB;
    __shared__ __attribute__((aligned(16))) unsigned lds_hist[4 * NB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id();
    unsigned* hist = lds_hist + wave * NB;
    const uint32_t start = cls[0], cnt = cls[1];
    const uint32_t G = gridDim.x * 4u;
    const uint32_t CH = max(1u, min((uint32_t)LIST_CHUNK, cnt / (4u * G)));
    for (uint32_t c0 = (blockIdx.x * 4u + wave) * CH; c0 < cnt; c0 += G * CH) {
        const int m = (int)min(CH, cnt - c0);
        uint32_t sid = 0, plo = 0, phi = 0;
        int nn = 0;
        if (lane < m) {
            sid = list[start + c0 + lane];
            const uint32_t* p;
            segs.get(sid, p, nn);
            plo = (uint32_t)(uintptr_t)p;
            phi = (uint32_t)((uintptr_t)p >> 32);
        }
        auto desc = [&](int j, int64_t& s, const uint32_t*& p, int& n) {
            s = (uint32_t)__builtin_amdgcn_readlane((int)sid, j);
            p = (const uint32_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)phi, j) << 32) |
                                  (uint32_t)__builtin_amdgcn_readlane((int)plo, j));
            n = __builtin_amdgcn_readlane(nn, j);
        };
        int64_t s;
        const uint32_t* p;
        int n;
        desc(0, s, p, n);
        // the chunk's results, segment j in lane j (lane j already holds its id and length):
        // one epilogue per chunk, lane-parallel (emit_lane), instead of one per segment
        unsigned a_mn = 0, a_mx = 0, a_k0 = 0, a_k1 = 0, a_c = 0, a_sdlo = 0, a_sdhi = 0, a_sqlo = 0,
                 a_sqhi = 0;
        uint32_t wide = 0;
        const auto keep = [&](int j, const LeanOut<PL>& r) {
            const uint64_t sdb = sd_bits(r.sd);
            const uint64_t sqb = (uint64_t)__double_as_longlong(r.sq);
            const bool mine = lane == j;
            a_mn = mine ? r.mn : a_mn;
            a_mx = mine ? r.mx : a_mx;
            a_k0 = mine ? r.mn + r.d0 : a_k0;
            a_k1 = mine ? r.mn + r.d1 : a_k1;
            a_c = mine ? r.c : a_c;
            a_sdlo = mine ? (uint32_t)sdb : a_sdlo;
            a_sdhi = mine ? (uint32_t)(sdb >> 32) : a_sdhi;
            a_sqlo = mine ? (uint32_t)sqb : a_sqlo;
            a_sqhi = mine ? (uint32_t)(sqb >> 32) : a_sqhi;
            if (r.mx >= NVRX_KEY_WIDE) wide |= 1u << j;
        };
        unsigned v[PL];
        if (ListPrefetch<PL>::on) {
            issue_loads<PL>(p, n, v);
            for (int j = 0; j < m; ++j) {
                // unconditional prefetch (the last one re-reads the current segment): a load
                // under a branch would make the waitcnt at the join cover it
                int64_t s2;
                const uint32_t* p2;
                int n2;
                desc(j + 1 < m ? j + 1 : j, s2, p2, n2);
                unsigned w[PL];
                issue_loads<PL>(p2, n2, w);
                int m0;
                unsigned x0;
                finish_loads<PL, false>(p, n, v, m0, x0);
                const LeanOut<PL> r = lean_core<PL, false, ListKeepBin<PL>::on>(v, n, m0, x0, hist);
                if (ListGroup<PL>::on) {
                    keep(j, r);
                } else {
                    emit_stats(out, s, n, r.mn, r.mx, r.d0, r.d1, (double)r.sd, r.sq, r.c, cr);
                    if (r.mx >= NVRX_KEY_WIDE) wide_moments(p, n, s, out);
                }
#pragma unroll
                for (int i = 0; i < PL; ++i) v[i] = w[i];
                s = s2;
                p = p2;
                n = n2;
            }
        } else {
            for (int j = 0; j < m; ++j) {
                if (j) desc(j, s, p, n);
                int m0;
                unsigned x0;
                load_segment<PL, false>(p, n, v, m0, x0);
                const LeanOut<PL> r = lean_core<PL, false, ListKeepBin<PL>::on>(v, n, m0, x0, hist);
                if (ListGroup<PL>::on) {
                    keep(j, r);
                } else {
                    emit_stats(out, s, n, r.mn, r.mx, r.d0, r.d1, (double)r.sd, r.sq, r.c, cr);
                    if (r.mx >= NVRX_KEY_WIDE) wide_moments(p, n, s, out);
                }
            }
        }
        if (ListGroup<PL>::on && lane < m)
            emit_lane(out, (int64_t)sid, nn, a_mn, a_mx, a_k0, a_k1,
                      sd_value<PL>(((uint64_t)a_sdhi << 32) | a_sdlo),
                      __longlong_as_double((long long)(((uint64_t)a_sqhi << 32) | a_sqlo)), a_c, cr);
        while (wide) {  // keys of >= 3.76 s: the decoded moments (rare)
            const int j = __builtin_ffs(wide) - 1;
            wide &= wide - 1;
            desc(j, s, p, n);
            wide_moments(p, n, s, out);
        }
    }
}

// FULL classes (seg_class C_F16..C_F128: exactly 64 * PL samples, 16-B aligned, FAST): the
// configs[1] group kernel's body over a class list -- each wave takes LIST_FULL_GROUP consecutive
// list entries, lanes 0..m-1 fetch their ids in one access, every segment runs the unmasked
// lean_core, and segment j's results wait in lane j for one lane-parallel epilogue.
#ifndef NVRX_LIST_FULL_GROUP  // build-time tuning constant
#define NVRX_LIST_FULL_GROUP 4
#endif
template <int PL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(Occ<PL>::W)))
void seg_stats_list_full_kernel(RaggedSegs segs, const uint32_t* list, const uint32_t* cls,
                                nvrx_stats_soa out) {
    const ColRef cr{nullptr, nullptr, 1, 1.0};  // column references: kernel_ref afterwards
    constexpr int NB = Bins<PL>::NB;
    constexpr uint32_t G = NVRX_LIST_FULL_GROUP;
    __shared__ __attribute__((aligned(16))) unsigned lds_hist[4 * NB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id();
    unsigned* hist = lds_hist + wave * NB;
    const uint32_t start = cls[0], cnt = cls[1];
    const uint32_t W = gridDim.x * 4u;
    for (uint32_t c0 = (blockIdx.x * 4u + wave) * G; c0 < cnt; c0 += W * G) {
        const int m = (int)min(G, cnt - c0);
        const uint32_t sid = lane < m ? list[start + c0 + lane] : 0u;
        unsigned a_mn = 0, a_mx = 0, a_k0 = 0, a_k1 = 0, a_c = 0, a_sdlo = 0, a_sdhi = 0, a_sqlo = 0,
                 a_sqhi = 0;
        uint32_t wide = 0;
        int n = 0;
        for (int j = 0; j < m; ++j) {
            const int64_t s = (uint32_t)__builtin_amdgcn_readlane((int)sid, j);
            const uint32_t* p;
            segs.get(s, p, n);  // n == 64 * PL (the class)
            unsigned v[PL];
            int m0;
            unsigned x0;
            load_segment<PL, true>(p, n, v, m0, x0);
            const LeanOut<PL> r = lean_core<PL>(v, n, 0, x0, hist);
            const uint64_t sqb = (uint64_t)__double_as_longlong(r.sq);
            const uint64_t sdb = sd_bits(r.sd);
            const bool mine = lane == j;
            a_mn = mine ? r.mn : a_mn;
            a_mx = mine ? r.mx : a_mx;
            a_k0 = mine ? r.mn + r.d0 : a_k0;
            a_k1 = mine ? r.mn + r.d1 : a_k1;
            a_c = mine ? r.c : a_c;
            a_sdlo = mine ? (uint32_t)sdb : a_sdlo;
            a_sdhi = mine ? (uint32_t)(sdb >> 32) : a_sdhi;
            a_sqlo = mine ? (uint32_t)sqb : a_sqlo;
            a_sqhi = mine ? (uint32_t)(sqb >> 32) : a_sqhi;
            if (r.mx >= NVRX_KEY_WIDE) wide |= 1u << j;
        }
        if (lane < m)
            emit_lane(out, (int64_t)sid, n, a_mn, a_mx, a_k0, a_k1,
                      sd_value<PL>(((uint64_t)a_sdhi << 32) | a_sdlo),
                      __longlong_as_double((long long)(((uint64_t)a_sqhi << 32) | a_sqlo)), a_c, cr);
        while (wide) {  // keys of >= 3.76 s: the decoded moments (rare)
            const int j = __builtin_ffs(wide) - 1;
            wide &= wide - 1;
            const int64_t s = (uint32_t)__builtin_amdgcn_readlane((int)sid, j);
            const uint32_t* p;
            segs.get(s, p, n);
            wide_moments(p, n, s, out);
        }
    }
}

template <int PL>
void launch_list_full(const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                      const nvrx_stats_soa& out, hipStream_t st) {
    const unsigned blocks = (unsigned)(cu_count() * Occ<PL>::W);
    hipLaunchKernelGGL((seg_stats_list_full_kernel<PL>), dim3(blocks), dim3(256), 0, st, segs, list, cls, out);
}

template <int NMAX>
__global__ __launch_bounds__(256) void seg_stats_exact_list_kernel(RaggedSegs segs,
                                                                   const uint32_t* list,
                                                                   const uint32_t* cls,
                                                                   nvrx_stats_soa out) {
    const ColRef cr{nullptr, nullptr, 1, 1.0};  // column references: kernel_ref afterwards
    __shared__ __attribute__((aligned(16))) float sbuf[NMAX];
    const uint32_t start = cls[0], cnt = cls[1];
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
        const int64_t s = list[start + i];
        const uint32_t* p;
        int n;
        segs.get(s, p, n);
        exact_body<NMAX>(p, n, s, sbuf, out, cr);
    }
}

// rings longer than NVRX_LDS_SEGMENT: exact_global_body over a per-block slice of device scratch
__global__ __launch_bounds__(XG_THREADS) void seg_stats_exact_list_global_kernel(
    RaggedSegs segs, const uint32_t* list, const uint32_t* cls, float* work, int64_t np2,
    nvrx_stats_soa out) {
    const ColRef cr{nullptr, nullptr, 1, 1.0};
    __shared__ __attribute__((aligned(16))) float lds[XG_CHUNK];
    const uint32_t start = cls[0], cnt = cls[1];
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
        const int64_t s = list[start + i];
        const uint32_t* p;
        int n;
        segs.get(s, p, n);
        exact_global_body(p, n, s, work + (int64_t)blockIdx.x * np2, lds, out, cr);
    }
}

int cu_count() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cus[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n <= 0)
            n = 256;
        cus[dev] = n;
    }
    return cus[dev];
}

template <int N>
void launch_lane(const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls, bool aligned16,
                 const nvrx_stats_soa& out, hipStream_t st) {
    const unsigned blocks = (unsigned)(cu_count() * 2 * LaneOcc<N>::W);
    hipLaunchKernelGGL((seg_stats_lane_kernel<N>), dim3(blocks), dim3(256), 0, st, segs, list, cls,
                       aligned16 ? 1 : 0, out);
}

template <int PL>
void launch_list(const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                 const nvrx_stats_soa& out, hipStream_t st) {
    const unsigned blocks = (unsigned)(cu_count() * ListOcc<PL>::W);
    hipLaunchKernelGGL((seg_stats_list_kernel<PL>), dim3(blocks), dim3(256), 0, st, segs, list, cls,
                       out);
}

hipError_t launch_exact_list(const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                             int64_t max_len, const nvrx_stats_soa& out,
                             hipStream_t st) {
    const unsigned cus = (unsigned)cu_count();
    if (max_len <= 1024)
        hipLaunchKernelGGL((seg_stats_exact_list_kernel<1024>), dim3(cus * 8), dim3(256), 0, st, segs,
                           list, cls, out);
    else if (max_len <= 8192)
        hipLaunchKernelGGL((seg_stats_exact_list_kernel<8192>), dim3(cus * 4), dim3(256), 0, st, segs,
                           list, cls, out);
    else if (max_len <= NVRX_LDS_SEGMENT)
        hipLaunchKernelGGL((seg_stats_exact_list_kernel<NVRX_LDS_SEGMENT>), dim3(cus), dim3(256), 0,
                           st, segs, list, cls, out);
    else if (max_len <= NVRX_MAX_SEGMENT) {
        const int64_t np2 = exact_global_np2(max_len), blocks = exact_global_blocks(np2, cus);
        void* work = nullptr;
        hipError_t e = scratch_alloc(&work, (size_t)(blocks * np2) * sizeof(float), st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(seg_stats_exact_list_global_kernel, dim3((unsigned)blocks), dim3(XG_THREADS),
                           0, st, segs, list, cls, (float*)work, np2, out);
        e = hipGetLastError();
        const hipError_t f = hipFreeAsync(work, st);
        return e != hipSuccess ? e : f;
    } else
        return hipErrorInvalidValue;
    return hipSuccess;
}


}  // namespace
}  // namespace ragged

// per-class launches, each defined in the translation unit that instantiates its kernel
void ragged_launch_lane(int n, const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                        bool aligned16, const nvrx_stats_soa& out, hipStream_t st);
void ragged_launch_list(int pl, const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                        const nvrx_stats_soa& out, hipStream_t st);
void ragged_launch_full(int pl, const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                        const nvrx_stats_soa& out, hipStream_t st);
hipError_t ragged_launch_exact(const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                               int64_t max_len, const nvrx_stats_soa& out,
                               hipStream_t st);

}  // namespace nvrx
