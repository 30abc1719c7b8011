// segment_rows.hip -- FAST per-kernel statistics for SHORT segments: 4 segments per wave.
//
// Same results as seg_stats_fast_kernel (segment_stats.hip; reference computeStats,
// straggler/cupti_src/CuptiProfiler.cpp:44-74) for strided segments of <= 16*PL samples,
// but each 16-lane DPP row of a wave owns one segment.  Everything that costs a fixed
// number of instructions per segment -- min/max/sum reductions (row DPP only, no
// readlanes), the histogram scan, candidate ranking, the epilogue's conversions and the
// 24-byte store -- then runs for 4 segments per instruction.  At 1024 samples per segment
// (the 4096-rank config) the one-segment-per-wave kernel spent ~60% of its VALU issue on
// those fixed costs.
//
// Per row: samples in VGPRs (16-B buffer loads, one SRD per wave, row offset in voffset),
// d = x - MIN in place, exact f64 sums, LDS histogram of NB bins per row, bucket location
// by a row-local DPP scan, resolution by (a) adjacent-bucket max/min, (b) width-1 bucket,
// (c) <= 16 candidates compacted with LDS atomics and ranked by compare, or (d) one more
// level inside the bucket.  Rows resolve independently (per-lane state, exec masks).
#include "nvrx_common.h"
#include "nvrx_internal.h"

namespace nvrx {

namespace {

template <int CTRL>
__device__ __forceinline__ unsigned dppr(unsigned x) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double dppr_f64(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const unsigned lo = dppr<CTRL>((unsigned)b), hi = dppr<CTRL>((unsigned)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// results valid in every lane of the 16-lane row
__device__ __forceinline__ unsigned row_min(unsigned v) {
    v = min(v, dppr<0xB1>(v));
    v = min(v, dppr<0x4E>(v));
    v = min(v, dppr<0x141>(v));
    return min(v, dppr<0x140>(v));
}
__device__ __forceinline__ unsigned row_max(unsigned v) {
    v = max(v, dppr<0xB1>(v));
    v = max(v, dppr<0x4E>(v));
    v = max(v, dppr<0x141>(v));
    return max(v, dppr<0x140>(v));
}
__device__ __forceinline__ double row_sum_f64(double v) {
    v = v + dppr_f64<0xB1>(v);
    v = v + dppr_f64<0x4E>(v);
    v = v + dppr_f64<0x141>(v);
    return v + dppr_f64<0x140>(v);
}
__device__ __forceinline__ unsigned row_incl_scan(unsigned v) {
    v += dppr<0x111>(v);
    v += dppr<0x112>(v);
    v += dppr<0x114>(v);
    return v + dppr<0x118>(v);
}
// value of `v` in lane `src` (0..15) of this lane's row
__device__ __forceinline__ unsigned row_get(unsigned v, unsigned src) {
    return (unsigned)__shfl((int)v, (int)((lane_id() & 48) + src));
}
// this row's 16 bits of a wave ballot
__device__ __forceinline__ unsigned row_bits(uint64_t m) {
    return (unsigned)(m >> (lane_id() & 48)) & 0xFFFFu;
}

template <int PL>
struct RowBins {
    static constexpr int NB = (2 * PL < 16) ? 16 : (2 * PL > 256 ? 256 : 2 * PL);  // bins per row
    static constexpr int BPL = NB / 16;                                          // bins per lane
    static constexpr int LOG = NB == 16 ? 4 : NB == 32 ? 5 : NB == 64 ? 6 : NB == 128 ? 7 : 8;
    static_assert((1 << LOG) == NB, "NB must be a power of two");
};

template <int PL>
struct RowOcc {
    static constexpr int W = PL >= 64 ? 3 : PL >= 32 ? 4 : 5;
};

}  // namespace

// Locate, per row, the buckets of relative ranks ta <= tb (per-lane values, uniform in a row).
template <int PL>
__device__ __forceinline__ void row_locate2(const unsigned* hist, unsigned ta, unsigned tb,
                                            unsigned& ba, unsigned& bfa, unsigned& ca,
                                            unsigned& bb, unsigned& bfb, unsigned& cb) {
    constexpr int BPL = RowBins<PL>::BPL;
    const int j = lane_id() & 15;
    unsigned h[BPL];
    unsigned local = 0;
#pragma unroll
    for (int b = 0; b < BPL; ++b) {
        h[b] = hist[j * BPL + b];
        local += h[b];
    }
    const unsigned incl = row_incl_scan(local);
    const unsigned excl = incl - local;
    const unsigned La = __builtin_popcount(row_bits(__ballot(incl <= ta)));
    const unsigned Lb = __builtin_popcount(row_bits(__ballot(incl <= tb)));
    unsigned run = excl, sa = 0, pa = 0, na = 0, sb = 0, pb = 0, nb = 0;
    bool fa = false, fb = false;
#pragma unroll
    for (int b = 0; b < BPL; ++b) {
        const unsigned nxt = run + h[b];
        if (!fa && nxt > ta) {
            fa = true;
            sa = (unsigned)(j * BPL + b);
            pa = run;
            na = h[b];
        }
        if (!fb && nxt > tb) {
            fb = true;
            sb = (unsigned)(j * BPL + b);
            pb = run;
            nb = h[b];
        }
        run = nxt;
    }
    ba = row_get(sa, La);
    bfa = row_get(pa, La);
    ca = row_get(na, La);
    bb = row_get(sb, Lb);
    bfb = row_get(pb, Lb);
    cb = row_get(nb, Lb);
}

struct ColRefRows {
    uint32_t* minbits;
    uint32_t* missing;
    int64_t ncols;
};

// Segment s = base[s*stride + begin + (len - keep) : + keep], keep = min(len, cap);
// requires stride % 4 == 0 (all rows share one 16-byte phase) and keep <= 16*PL.
template <int PL, bool FULL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RowOcc<PL>::W)))
void seg_rows_kernel(const uint32_t* base, int64_t nseg, int64_t stride, int64_t begin,
                     int64_t keep_off, int n, nvrx_stats_soa out, ColRefRows cr) {
    constexpr int NV = PL / 4;
    constexpr int NB = RowBins<PL>::NB;
    constexpr int LOGNB = RowBins<PL>::LOG;
    constexpr int BPL = RowBins<PL>::BPL;
    __shared__ __attribute__((aligned(16))) unsigned lds[4][4][NB];
    __shared__ unsigned cnt[4][4];

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id();
    const int row = lane >> 4;
    const int j = lane & 15;
    const int64_t s0 = ((int64_t)blockIdx.x * 4 + wave) * 4;
    if (s0 >= nseg) return;  // wave-uniform
    const int64_t s = s0 + row;
    const int rows_here = (int)min<int64_t>(4, nseg - s0);
    const bool valid = row < rows_here;
    unsigned* hist = &lds[wave][row][0];

    // ---- HBM -> VGPR: one SRD per wave (base = row 0's aligned start), row in voffset
    const uint32_t* p0 = base + s0 * stride + begin + keep_off;
    const uintptr_t pa = (uintptr_t)p0 & ~(uintptr_t)15;
    const int m0 = FULL ? 0 : (int)(((uintptr_t)p0 & 15) >> 2);
    const int nvec = (n + m0 + 3) >> 2;
    const unsigned pa_lo = __builtin_amdgcn_readfirstlane((unsigned)pa);
    const unsigned pa_hi = __builtin_amdgcn_readfirstlane((unsigned)(pa >> 32));
    const int nbytes = __builtin_amdgcn_readfirstlane(
        (int)((int64_t)(rows_here - 1) * stride * 4 + (int64_t)nvec * 16));
    void* const pbase = (void*)(((uint64_t)pa_hi << 32) | pa_lo);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(pbase, 0, nbytes, 0x00020000);
    const unsigned roff = (unsigned)(row * stride * 4);
    unsigned v[PL];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(roff + (q * 16 + j) * 16), 0, 0);
        v[4 * q + 0] = w.x;
        v[4 * q + 1] = w.y;
        v[4 * q + 2] = w.z;
        v[4 * q + 3] = w.w;
    }
    const int pad = FULL ? 0 : 16 * PL - n;
    unsigned x0 = 0;
    if (!FULL) {
        x0 = valid ? p0[row * stride] : 0u;  // a sample of the row: neutral for min/max
#pragma unroll
        for (int i = 0; i < PL; ++i) {
            const unsigned e = (unsigned)((((i >> 2) * 16 + j) * 4) + (i & 3) - m0);
            v[i] = (e < (unsigned)n) ? v[i] : x0;
        }
    }
    unsigned lmn = v[0], lmx = v[0];
#pragma unroll
    for (int i = 1; i < PL; ++i) {
        lmn = min(lmn, v[i]);
        lmx = max(lmx, v[i]);
    }
    const unsigned mn = row_min(lmn);
    const unsigned mx = row_max(lmx);
#pragma unroll
    for (int i = 0; i < PL; ++i) {
        if (FULL) {
            v[i] -= mn;
        } else {
            const unsigned e = (unsigned)((((i >> 2) * 16 + j) * 4) + (i & 3) - m0);
            v[i] = (e < (unsigned)n) ? v[i] - mn : 0u;
        }
    }
    const unsigned range = mx - mn;
    const int bits = 32 - __clz((int)range);
    int shift = bits > LOGNB ? bits - LOGNB : 0;

#pragma unroll
    for (int b = 0; b < BPL; ++b) hist[j * BPL + b] = 0u;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < PL; ++i) atomicAdd(&hist[v[i] >> shift], 1u);
    __builtin_amdgcn_wave_barrier();
    // pivot: the row's first sample (FULL); masked rows use c = 0 in f64
    const bool pivot = FULL && __ballot(range >= 0x80000000u) == 0;
    const unsigned c = pivot ? row_get(v[0], 0u) : 0u;
    uint64_t sdl;
    double sql;
    if (pivot)
        lane_sums<PL>(v, c, sdl, sql);
    else
        lane_sums_f64<PL>(v, sdl, sql);
    const double sd = row_sum_f64((double)sdl);
    const double sq = row_sum_f64(sql);

    // ---- median selection, rows independently
    const unsigned t0 = (unsigned)(pad + ((n & 1) ? n / 2 : n / 2 - 1));
    const unsigned t1 = (unsigned)(pad + n / 2);
    unsigned wlo = 0, below = 0, d0 = 0, d1 = 0;
    bool done = !valid;
    for (int level = 0; __ballot(!done) != 0; ++level) {
        if (level > 0) {
            if (!done) {
#pragma unroll
                for (int b = 0; b < BPL; ++b) hist[j * BPL + b] = 0u;
            }
            __builtin_amdgcn_wave_barrier();
            if (!done) {
                const unsigned span = (unsigned)NB << shift;  // level > 0: fits in 32 bits
#pragma unroll
                for (int i = 0; i < PL; ++i) {
                    const unsigned q = v[i] - wlo;  // wraps for d < wlo
                    if (q < span) atomicAdd(&hist[q >> shift], 1u);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        unsigned b0 = 0, c0 = 0, n0 = 0, b1 = 0, c1 = 0, n1 = 0;
        row_locate2<PL>(hist, t0 - below, t1 - below, b0, c0, n0, b1, c1, n1);
        // case A: the two middle ranks straddle two buckets
        const bool caseA = !done && b0 != b1;
        if (__ballot(caseA)) {
            unsigned lmax = 0, lmin = 0xFFFFFFFFu;
            if (caseA) {
                const unsigned lo0 = wlo + (b0 << shift), lo1 = wlo + (b1 << shift);
                const unsigned width = 1u << shift;
#pragma unroll
                for (int i = 0; i < PL; ++i) {
                    const unsigned d = v[i];
                    if (d - lo0 < width) lmax = max(lmax, d);
                    if (d - lo1 < width) lmin = min(lmin, d);
                }
            }
            lmax = row_max(lmax);
            lmin = row_min(lmin);
            if (caseA) {
                d0 = lmax;
                d1 = lmin;
                done = true;
            }
        }
        // case B: width-1 bucket -> the value itself
        const bool caseB = !done && shift == 0;
        if (caseB) {
            d0 = d1 = wlo + b0;
            done = true;
        }
        // case C: <= 16 candidates -> compact (LDS atomics) and rank by compare
        const bool caseC = !done && n0 <= 16u;
        if (__ballot(caseC)) {
            if (caseC && j == 0) cnt[wave][row] = 0u;
            __builtin_amdgcn_wave_barrier();
            if (caseC) {
                const unsigned lo0 = wlo + (b0 << shift);
                const unsigned width = 1u << shift;
#pragma unroll
                for (int i = 0; i < PL; ++i) {
                    const unsigned d = v[i];
                    if (d - lo0 < width) {
                        const unsigned pos = atomicAdd(&cnt[wave][row], 1u);
                        hist[pos] = d;  // the row's histogram is consumed
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            const unsigned ci = (caseC && (unsigned)j < n0) ? hist[j] : 0xFFFFFFFFu;
            unsigned rank = 0;
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                const unsigned cj = row_get(ci, (unsigned)jj);
                rank += ((unsigned)jj < n0 && (cj < ci || (cj == ci && jj < j))) ? 1u : 0u;
            }
            const unsigned r0 = t0 - below - c0, r1 = t1 - below - c0;
            const unsigned m0b = row_bits(__ballot(caseC && (unsigned)j < n0 && rank == r0));
            const unsigned m1b = row_bits(__ballot(caseC && (unsigned)j < n0 && rank == r1));
            const unsigned v0 = row_get(ci, (unsigned)(__builtin_ffs((int)m0b) - 1) & 15u);
            const unsigned v1 = row_get(ci, (unsigned)(__builtin_ffs((int)m1b) - 1) & 15u);
            if (caseC) {
                d0 = v0;
                d1 = v1;
                done = true;
            }
        }
        // case D: descend one level into bucket b0
        if (!done) {
            below += c0;
            wlo += b0 << shift;
            shift = shift > LOGNB ? shift - LOGNB : 0;
        }
    }

    if (valid && j == 0) {
        out.num[s] = n;
        out.min[s] = ns_to_us(mn);
        out.max[s] = ns_to_us(mx);
        const float f0 = ns_to_us(mn + d0);
        float med = f0;
        if (!(n & 1)) {
            const float f1 = ns_to_us(mn + d1);
            med = (f0 + f1) / 2;  // f32 add, exact halving (CuptiProfiler.cpp:58)
        }
        out.med[s] = med;
        if (cr.minbits) atomicMin(&cr.minbits[s % cr.ncols], __float_as_uint(med));
        // same formulas as emit_stats (segment_stats.hip)
        const double dn = (double)n;
        const double se = sd - dn * (double)c;
        out.avg[s] = (float)(__builtin_fma((double)mn, dn, sd) / (1000.0 * dn));
        const double var = __builtin_fma(sq, dn, -(se * se));
        out.std[s] = (float)(__builtin_sqrt(var > 0.0 ? var : 0.0) / (1000.0 * dn));
    }
}

template <int PL>
static void launch_rows_pl(const uint32_t* ns, int64_t nseg, int64_t stride, int64_t begin,
                           int64_t keep_off, int keep, bool full, const nvrx_stats_soa& out,
                           const ColRefRows& cr, hipStream_t st) {
    const dim3 grid((unsigned)((nseg + 15) / 16)), block(256);
    if (full)
        hipLaunchKernelGGL((seg_rows_kernel<PL, true>), grid, block, 0, st, ns, nseg, stride, begin,
                           keep_off, keep, out, cr);
    else
        hipLaunchKernelGGL((seg_rows_kernel<PL, false>), grid, block, 0, st, ns, nseg, stride,
                           begin, keep_off, keep, out, cr);
}

// Returns hipErrorNotSupported when the shape does not fit the rows kernel (the caller then
// uses the one-segment-per-wave kernel).
hipError_t segment_stats_rows(const uint32_t* ns, int64_t nseg, int64_t stride, int64_t begin,
                              int64_t len, int64_t cap, const nvrx_stats_soa& out,
                              uint32_t* minbits, uint32_t* missing, int64_t ncols,
                              hipStream_t st) {
    const int64_t keep = (cap > 0 && len > cap) ? cap : len;
    if (keep <= 0 || stride % 4 != 0 || nseg <= 0) return hipErrorNotSupported;
    if (3 * stride * 4 + 16 * 64 * 4 >= ((int64_t)1 << 31)) return hipErrorNotSupported;
    const bool aligned = (((uintptr_t)(ns + begin + (len - keep))) & 15) == 0;
    const int64_t need = aligned ? keep : keep + 3;
    const ColRefRows cr{minbits, missing, ncols > 0 ? ncols : 1};
    const int64_t koff = len - keep;
    const int k = (int)keep;
    if (need <= 16 * 4)
        launch_rows_pl<4>(ns, nseg, stride, begin, koff, k, aligned && keep == 64, out, cr, st);
    else if (need <= 16 * 8)
        launch_rows_pl<8>(ns, nseg, stride, begin, koff, k, aligned && keep == 128, out, cr, st);
    else if (need <= 16 * 16)
        launch_rows_pl<16>(ns, nseg, stride, begin, koff, k, aligned && keep == 256, out, cr, st);
    else if (need <= 16 * 32)
        launch_rows_pl<32>(ns, nseg, stride, begin, koff, k, aligned && keep == 512, out, cr, st);
    else if (need <= 16 * 64)
        launch_rows_pl<64>(ns, nseg, stride, begin, koff, k, aligned && keep == 1024, out, cr, st);
    else
        return hipErrorNotSupported;
    return hipGetLastError();
}

}  // namespace nvrx
