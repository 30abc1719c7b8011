// segment_kernels.h -- device code shared by the segment-statistics launchers
// (segment_stats.hip: strided / one-shot; segment_ragged.hip: length classes).
// See segment_stats.hip for the algorithm.
#pragma once
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "nvrx_common.h"
#include "nvrx_internal.h"

namespace nvrx {

// ---------------------------------------------------------------------------
// Segment addressing
// ---------------------------------------------------------------------------
struct StridedSegs {  // segment s = base[s*stride + begin : + len], last `cap` kept
    const uint32_t* base;
    int64_t stride, begin, len, cap;
    __device__ __forceinline__ void get(int64_t s, const uint32_t*& p, int& n) const {
        int64_t keep = (cap > 0 && len > cap) ? cap : len;
        p = base + s * stride + begin + (len - keep);
        n = (int)keep;
    }
};
struct RaggedSegs {  // segment s = base[off[s] : off[s] + len[s]] (len NULL: off[s+1]), last `cap` kept;
                     // len[s] < 0: skipped (already reduced, e.g. by records_stats)
    const uint32_t* base;
    const int64_t* off;
    const int32_t* lens;
    int64_t cap;
    __device__ __forceinline__ void get(int64_t s, const uint32_t*& p, int& n) const {
        const int64_t b = off[s];
        const int64_t e = lens ? b + lens[s] : off[s + 1];
        const int64_t len = e - b;
        int64_t keep = (cap > 0 && len > cap) ? cap : len;
        p = base + (e - keep);
        n = (int)keep;
    }
    // the retained length alone (no offset load when `lens` is given)
    __device__ __forceinline__ int kept_len(int64_t s) const {
        const int64_t len = lens ? (int64_t)lens[s] : off[s + 1] - off[s];
        return (int)((cap > 0 && len > cap) ? cap : len);
    }
};

// Optional fused per-column reference (segment s = row s / ncols, column s % ncols):
// minbits[c] = atomicMin of the float bits of MED (non-negative floats order like their
// bit patterns), missing[c] |= 1 for an empty segment -- _all_reduce_times'
// MIN-over-ranks with the -1 => NaN rule (reporting.py:255-296), done in the epilogue.
struct ColRef {
    uint32_t* minbits;
    uint32_t* missing;
    int64_t ncols;
    double inv;  // 1.0 / ncols
    // s % ncols without a 64-bit integer divide: the f64 quotient is off by at most one
    // for s < 2^52
    __device__ __forceinline__ int64_t col(int64_t s) const {
        int64_t q = (int64_t)((double)s * inv);
        int64_t r = s - q * ncols;
        if (r < 0) r += ncols;
        if (r >= ncols) r -= ncols;
        return r;
    }
    __device__ __forceinline__ void add(int64_t s, float med) const {
        if (minbits) atomicMin(&minbits[col(s)], __float_as_uint(med));
    }
    __device__ __forceinline__ void miss(int64_t s) const {
        if (minbits) atomicOr(&missing[col(s)], 1u);
    }
};

// ---------------------------------------------------------------------------
// Length classes of ragged segments (segment_ragged.hip).  Class lists: cls[2c] = first list entry of class c, cls[2c+1] = its
// count.
// ---------------------------------------------------------------------------
namespace ragged {
enum : int {
    C_T8 = 0, C_T16, C_T32, C_T64, C_T128,    // lane classes
    C_W4, C_W8, C_W16, C_W32, C_W64, C_W128,  // wave classes (PL)
    C_X,                                      // workgroup (EXACT kernel)
    C_F,                                      // FAST, exactly full_n = 64 * PL samples, 16-B aligned
    NCLASS
};

// need = retained samples + misalignment slack a wave would have to hold.  Every class is a
// power-of-two length range, so the class is ceil(log2) of the length, offset: lane classes
// 1..8 / 9..16 / ... / 65..128, then wave classes of need 129..256 (PL 4) ... 4097..8192 (PL 128).
// full_n (0: none) -- the longest retained length when it is 64 * PL samples for a PL of 16..128
// and the segments start on 16-B boundaries (FAST): segments of exactly that length, the rings
// that overflowed (the hot kernels of a live report, configs[3]'s hottest slot), are the FULL
// class -- no lane masks, and the grouped lane-parallel epilogue (seg_stats_list_full_kernel).
__device__ __forceinline__ int seg_class(int n, bool aligned16, bool exact, int full_n) {
    if (n <= 128) {
        const int l = 32 - __clz(n - 1);  // ceil(log2 n); 0 for n = 1
        return l <= 3 ? C_T8 : l - 3;     // 4..7 -> C_T16..C_T128
    }
    if (exact) return C_X;
    if (n == full_n) return C_F;
    const int need = aligned16 ? n : n + 3;
    const int l = 32 - __clz(need - 1);  // 8..13 -> C_W4..C_W128
    return l <= 13 ? l - 3 : C_X;
}
static_assert(C_T16 == 1 && C_T128 == 4 && C_W4 == 5 && C_W128 == 10 && C_X == 11 && C_F == 12,
              "class order");
// the FULL length of a launch (seg_class): keep if it is 64 * PL for PL in 16..128, else 0
inline int full_len(int64_t keep, bool aligned16, bool exact) {
    return (!exact && aligned16 && (keep == 1024 || keep == 2048 || keep == 4096 || keep == 8192)) ? (int)keep : 0;
}

// Wave-aggregated class counting: one LDS atomic per distinct class present in the
// wave (leader = lowest lane); returns this lane's rank among same-class lanes plus the
// class's previous count.  cls < 0: lane does not take part.
__device__ __forceinline__ uint32_t wave_class_add(uint32_t* lcnt, int cls) {
    uint64_t pending = __ballot(cls >= 0);
    uint32_t mine = 0;
    while (pending) {
        const int leader = __builtin_ffsll(pending) - 1;
        const int c = __builtin_amdgcn_readlane(cls, leader);
        const uint64_t grp = __ballot(cls == c) & pending;
        uint32_t base = 0;
        if (lane_id() == leader) base = atomicAdd(&lcnt[c], (uint32_t)__popcll(grp));
        base = __builtin_amdgcn_readlane(base, leader);
        if (cls == c) mine = base + mbcnt(grp);
        pending &= ~grp;
    }
    return mine;
}
}  // namespace ragged

// The class kernels over class-ordered segment lists (segment_ragged.hip): keep = the
// longest retained segment; classes it rules out are not launched.
hipError_t ragged_launch_classes(const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                                 int64_t keep, bool aligned16, bool exact, const nvrx_stats_soa& out,
                                 hipStream_t st);

__device__ __forceinline__ void write_empty(const nvrx_stats_soa& o, int64_t s) {
    // KernelStats() default: num_calls 0, every float NaN (CuptiProfiler.h:39-45)
    const float q = __builtin_nanf("");
    o.num[s] = 0;
    o.min[s] = q;
    o.max[s] = q;
    o.med[s] = q;
    o.avg[s] = q;
    o.std[s] = q;
}

// Epilogue of the FAST kernels, lane-parallel: lanes 0-3 convert MIN, MAX, s[t0], s[t1]
// in one ns_to_us, lanes 0/1 form avg and std from one f64 divide; lane 0 stores.
//   sd = sum(d), sq = sum((d - c)^2) over the n samples, d = x - MIN.
//   avg = (n MIN + sd) / (1000 n)               (numerator exact in f64)
//   std = sqrtf(f32((n sq - (sd - n c)^2) / (1000 n)^2))  (population std, CuptiProfiler.cpp:66-70)
// num / dd from the hardware reciprocal refined by two Newton steps and one residual
// correction (~1e-16 relative; emit_stats and the group epilogue share it, so both round alike)
__device__ __forceinline__ double quot_f64(double num, double dd) {
    double rc = __builtin_amdgcn_rcp(dd);
    rc = __builtin_fma(rc, __builtin_fma(-dd, rc, 1.0), rc);
    rc = __builtin_fma(rc, __builtin_fma(-dd, rc, 1.0), rc);
    double q = num * rc;
    return __builtin_fma(__builtin_fma(-dd, q, num), rc, q);
}

__device__ __forceinline__ void emit_stats(const nvrx_stats_soa& o, int64_t s, int n,
                                           unsigned mn, unsigned mx, unsigned d0, unsigned d1,
                                           double sd, double sq, unsigned c, const ColRef& cr) {
    const int lane = lane_id();
    const unsigned x = lane == 0 ? mn : lane == 1 ? mx : lane == 2 ? mn + d0 : mn + d1;
    const float f = mx < NVRX_KEY_WIDE ? ns_to_us_narrow(x) : ns_to_us(x);  // wave-uniform
    const float fmn = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, f), 0));
    const float fmx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, f), 1));
    const float f0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, f), 2));
    const float f1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, f), 3));
    // CuptiProfiler.cpp:58: f32 add, exact halving
    const float med = (n & 1) ? f0 : (f0 + f1) / 2;
    const double dn = (double)n;
    const double se = sd - dn * (double)c;  // exact: integers < 2^53
    // lane 0: avg = (n MIN + sd) / (1000 n), rounded once to f32;
    // lane 1: std = sqrt(n sq - se^2) / (1000 n) as the f32 root of the f32-rounded variance
    //         in us^2.
    // The quotient is num times the hardware reciprocal refined by Newton steps (~1e-16
    // relative, so at most a rounding-boundary case off the correctly rounded f32) and the root
    // is the hardware v_sqrt_f32 (~1 ulp): both far inside the FAST bars (2.5e-7 / 1e-6
    // relative), without the f64 divide and correctly rounded sqrt sequences (~20 of ~400 VALU
    // per segment at 1024 samples).
    const double den = 1000.0 * dn;
    const double vq = __builtin_fma(sq, dn, -(se * se));
    const double num = lane == 0 ? __builtin_fma((double)mn, dn, sd) : (vq > 0.0 ? vq : 0.0);
    const double dd = lane == 0 ? den : den * den;
    const double q = quot_f64(num, dd);
    const float r = lane == 0 ? (float)q : __builtin_amdgcn_sqrtf((float)q);
    const float avg = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, r), 0));
    const float sdv = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, r), 1));
    if (lane == 0) {
        o.num[s] = n;
        o.min[s] = fmn;
        o.max[s] = fmx;
        o.med[s] = med;
        o.avg[s] = avg;
        o.std[s] = sdv;
        cr.add(s, med);
    }
}

// emit_stats for one segment per lane (the group epilogues: lane j holds segment s0 + j's
// results); the same arithmetic, so the same bits.  k0 / k1: the middle-rank keys (mn + d0,
// mn + d1).
__device__ __forceinline__ void emit_lane(const nvrx_stats_soa& o, int64_t s, int n, unsigned mn,
                                          unsigned mx, unsigned k0, unsigned k1, double sd,
                                          double sq, unsigned c, const ColRef& cr) {
    const float f0 = ns_to_us(k0), f1 = ns_to_us(k1);
    const float med = (n & 1) ? f0 : (f0 + f1) / 2;  // CuptiProfiler.cpp:58
    const double dn = (double)n;
    const double se = sd - dn * (double)c;
    const double den = 1000.0 * dn;
    const double vq = __builtin_fma(sq, dn, -(se * se));
    o.num[s] = n;
    o.min[s] = ns_to_us(mn);
    o.max[s] = ns_to_us(mx);
    o.med[s] = med;
    o.avg[s] = (float)quot_f64(__builtin_fma((double)mn, dn, sd), den);
    o.std[s] = __builtin_amdgcn_sqrtf((float)quot_f64(vq > 0.0 ? vq : 0.0, den * den));
    cr.add(s, med);
}

// FAST AVG / STD of a segment whose keys reach NVRX_KEY_WIDE (a kernel of 3.76 s or more): the
// integer sums of the bodies do not apply to f32-valued keys, so lane 0 overwrites what
// emit_stats stored with the mean and population std of the decoded f32(ns) values in f64, each
// rounded once to f32 us -- two strided passes over the segment p[0:n) in memory (no register
// arrays: this rare branch must not raise the bodies' register pressure).
__device__ __forceinline__ void wide_moments(const uint32_t* p, int n, int64_t s, const nvrx_stats_soa& o) {
    const int lane = lane_id();
    double a = 0.0;
    for (int i = lane; i < n; i += 64) a += (double)key_to_f32(p[i]);
    const double mean = wave_sum_f64(a) / (double)n;
    double q = 0.0;
    for (int i = lane; i < n; i += 64) {
        const double e = (double)key_to_f32(p[i]) - mean;
        q = __builtin_fma(e, e, q);
    }
    const double var = wave_sum_f64(q) / (double)n;
    if (lane == 0) {
        o.avg[s] = (float)(mean / 1000.0);
        o.std[s] = (float)(__builtin_sqrt(var) / 1000.0);
    }
}

#ifndef NVRX_BINS_PER_SAMPLE_SHORT  // build-time tuning constant: bins per lane-sample, PL <= 8
#define NVRX_BINS_PER_SAMPLE_SHORT 16
#endif
template <int PL>
struct Bins {
    // bins per wave: 16 per lane-sample for short segments (PL <= 16: C3's 1024 samples take
    // 256 bins -- fewer bucket-mates of the median to compact and rank, 3-5 % faster than 128,
    // while 512 was slower), 8 above (PL = 32 was fastest at 256)
    static constexpr int PB = PL <= 8 ? NVRX_BINS_PER_SAMPLE_SHORT * PL : PL <= 16 ? 16 * PL : 8 * PL;
    static constexpr int NB = PB < 64 ? 64 : PB > 512 ? 512 : PB;
    static constexpr int BPL = NB / 64;                     // bins per lane
    static constexpr int LOG = (NB == 64) ? 6 : (NB == 128) ? 7 : (NB == 256) ? 8 : (NB == 512) ? 9 : 10;
    static_assert((1 << LOG) == NB, "NB must be a power of two <= 1024");
};

// Locate the bucket holding relative rank ta in the wave's histogram (one read of the bins):
// bucket index, elements in lower buckets, count of the bucket.  Vector work is the row-wise
// inclusive prefix of the lanes' bin sums (DPP row shifts) and one compare; the row holding ta,
// the lane inside it (ballot), that lane's bins (readlanes) and the walk over them are scalar.
template <int PL>
__device__ __forceinline__ void hist_locate1(const unsigned* hist, unsigned ta, unsigned& ba,
                                             unsigned& bfa, unsigned& ca) {
    constexpr int BPL = Bins<PL>::BPL;
    const int lane = lane_id();
    unsigned h[BPL];
    unsigned local = 0;
#pragma unroll
    for (int j = 0; j < BPL; ++j) {
        h[j] = hist[lane * BPL + j];
        local += h[j];
    }
    unsigned v = local;  // inclusive prefix inside the lane's 16-lane row
    v += dpp<0x111>(v);
    v += dpp<0x112>(v);
    v += dpp<0x114>(v);
    v += dpp<0x118>(v);
    const unsigned t0 = rl(v, 15), t1 = t0 + rl(v, 31), t2 = t1 + rl(v, 47);
    const int row = ta < t0 ? 0 : ta < t1 ? 1 : ta < t2 ? 2 : 3;
    const unsigned rbase = row == 0 ? 0u : row == 1 ? t0 : row == 2 ? t1 : t2;
    const uint64_t before = __ballot(v <= ta - rbase) & (0xFFFFull << (16 * row));
    const int La = min(16 * row + (int)__popcll(before), 63);
    unsigned hs[BPL], loc = 0;
#pragma unroll
    for (int j = 0; j < BPL; ++j) {
        hs[j] = rl(h[j], La);
        loc += hs[j];
    }
    unsigned run = rbase + rl(v, La) - loc;  // elements below lane La's first bin
    ba = (unsigned)(La * BPL + BPL - 1);
    bfa = run;
    ca = 0;
    bool found = false;
#pragma unroll
    for (int j = 0; j < BPL; ++j) {
        const unsigned nxt = run + hs[j];
        if (!found && nxt > ta) {
            found = true;
            ba = (unsigned)(La * BPL + j);
            bfa = run;
            ca = hs[j];
        }
        run = nxt;
    }
}

// Occupancy target per PL: the samples take PL VGPRs; ask the register allocator for
// enough waves per SIMD that HBM latency is covered by other waves' segments.
template <int PL>
struct Occ {
    static constexpr int W = PL >= 128 ? 3 : PL >= 64 ? 4 : PL >= 32 ? 6 : 8;
};
template <int PL, bool FULL>
struct OccV {  // the masked PL=128 variant gets the whole 256-register budget
    static constexpr int W = (!FULL && PL >= 128) ? 2 : Occ<PL>::W;
};

// cache policy of the once-read sample stream (buffer-load aux bits)
#ifndef NVRX_LOAD_AUX
#define NVRX_LOAD_AUX 2  // nt: measured +1.5-2% on C2/C3 over the default policy
#endif

// One wave per segment held in registers (v: 64*PL slots, lane-interleaved in 16-B vectors;
// register i of lane L holds slot e = 256 (i >> 2) + 4 L + (i & 3) - m0).  MIN / MAX by wave
// reductions; d = x - MIN in place; exact sums; MED by radix select on d with a wave-private LDS
// histogram, the median's bucket resolved by candidate compaction and rank-by-compare, or by
// the wrapped extremes of two buckets, or by another level.  Round 3 replaced the masked
// (!FULL) body (fast_body: per-slot masks, f64 squares about 0) with this one.  Per sample:
//   * the exact sum is one 32-bit add when the segment spans < 2^24 ns (64*PL*2^24 < 2^32:
//     no carry chain); wider segments take lane_sums / lane_sums_f64;
//   * the squares are packed f32 (v_pk_add / v_pk_fma on sample pairs: d, c < 2^24 convert
//     exactly, so (float)d - (float)c == (float)(int)(d - c));
//   * when ranks t0, t1 fall in different buckets b0 < b1, s[t0] = max{d < hi(b0)} and
//     s[t1] = min{d >= lo(b1)} come from one wrapped max / min per sample: d - hi (mod 2^32)
//     puts every sample below hi above every sample at or above it, so the wave max of
//     d - hi is the largest sample below hi (likewise the min of d - lo), for any range.
// The wave reductions finish with row_bcast (wave_*_b).
template <int PL>
struct LeanOut {
    // the exact sum of d: an integer for PL <= 16 (the group kernel's epilogue takes it from
    // scalar registers), its (exact) f64 value above
    using Sd = typename std::conditional<(PL <= 16), uint64_t, double>::type;
    unsigned mn, mx, d0, d1, c;  // d0 / d1: the two middle ranks, relative to mn
    Sd sd;
    double sq;
};
// LeanOut::sd through a 64-bit register pair (the group epilogues' lane-held results)
__device__ __forceinline__ uint64_t sd_bits(uint64_t sd) { return sd; }
__device__ __forceinline__ uint64_t sd_bits(double sd) { return (uint64_t)__double_as_longlong(sd); }
template <int PL>
__device__ __forceinline__ double sd_value(uint64_t b) {
    if constexpr (PL <= 16)
        return (double)b;
    else
        return __longlong_as_double((long long)b);
}

// !FULL: a segment of n < 64 * PL samples starting m0 slots into its first 16-byte vector
// (finish_loads set every other slot to x0, sample 0, the pivot: neutral for MIN / MAX, d - c
// = 0 in the squares).  The pad = 64 * PL - n copies of x0 are taken out again where they
// count: pad * c from the exact sum; -pad as the initial count of the pivot's bin at every
// histogram level whose window holds it; and from the candidates of the pivot's bucket (a
// masked compaction, only when the median's bucket is the pivot's).  The wrapped max / min of
// two buckets need nothing: x0 is a sample, so its copies change neither.
// KB: level-0 bins kept in registers (PL more VGPRs).
template <int PL, bool FULL = true, bool KB = (PL <= 16)>
__device__ __forceinline__ LeanOut<PL> lean_core(unsigned (&v)[PL], int n, int m0, unsigned x0,
                                                 unsigned* hist) {
    using Sd = typename LeanOut<PL>::Sd;
    constexpr int NB = Bins<PL>::NB;
    constexpr int LOGNB = Bins<PL>::LOG;
    constexpr int BPL = Bins<PL>::BPL;
    const int lane = lane_id();
    const unsigned pad = FULL ? 0u : (unsigned)(64 * PL - n);
    const int eb = 4 * lane - m0;  // slot of register i: eb + 256 (i >> 2) + (i & 3)
    const auto real = [&](int i) { return FULL || (unsigned)(eb + 256 * (i >> 2) + (i & 3)) < (unsigned)n; };

    unsigned lmn = v[0], lmx = v[0];
#pragma unroll
    for (int i = 1; i < PL; ++i) {
        lmn = min(lmn, v[i]);
        lmx = max(lmx, v[i]);
    }
    const unsigned mn = wave_min_b(lmn);
    const unsigned mx = wave_max_b(lmx);
    const unsigned range = mx - mn;
    // Segments spanning < 2^23 ns (every configs[] shape) hold x = d + B, B = 0x4B000000 = the
    // f32 bits of 2^23: x is then the bit pattern of the float 2^23 + d, so the squares take
    // the registers as they are (no int -> float conversion per sample).  Selection is
    // translation invariant -- the histogram takes bits [shift, shift + LOGNB) of x (those of
    // d: bits(range) <= 23), the walk starts at wlo = B -- and B leaves the results at the end.
    const unsigned B = range < (1u << 23) ? 0x4B000000u : 0u;
    const unsigned off = B - mn;
#pragma unroll
    for (int i = 0; i < PL; ++i) v[i] += off;

    // ---- exact sum + squares about the pivot c (lane_sums order: pairs, groups of 16) ----
    const unsigned cp = x0 - mn;  // the padding's d
    unsigned c = cp;
    Sd sd;
    double acc;
    if (range < (1u << 24)) {
        constexpr int G = PL < 16 ? PL : 16;
        unsigned ls = 0;
        acc = 0.0;
        if (B) {
            // (2^23 + d) - (2^23 + c): both exact in f32, and so is the difference
            const float fc = __builtin_bit_cast(float, B + c);
            const f32x2 cc = {fc, fc};
#pragma unroll
            for (int g = 0; g < PL; g += G) {
                f32x2 q = {0.0f, 0.0f};
#pragma unroll
                for (int i = 0; i < G; i += 2) {
                    ls += v[g + i];
                    ls += v[g + i + 1];
                    const f32x2 e = (f32x2){__builtin_bit_cast(float, v[g + i]),
                                            __builtin_bit_cast(float, v[g + i + 1])} - cc;
                    q = __builtin_elementwise_fma(e, e, q);
                }
                acc += (double)q.x + (double)q.y;
            }
            ls -= (unsigned)PL * B;  // sum d mod 2^32, exact: PL * 2^23 < 2^32
        } else {
            const f32x2 cc = {(float)c, (float)c};
#pragma unroll
            for (int g = 0; g < PL; g += G) {
                f32x2 q = {0.0f, 0.0f};
#pragma unroll
                for (int i = 0; i < G; i += 2) {
                    ls += v[g + i];
                    ls += v[g + i + 1];
                    const f32x2 e = (f32x2){(float)v[g + i], (float)v[g + i + 1]} - cc;
                    q = __builtin_elementwise_fma(e, e, q);
                }
                acc += (double)q.x + (double)q.y;
            }
        }
        if (PL <= 16) {
            // integer reduction: a row of 16 lanes sums to < 16 * 16 * 2^24 = 2^32 (no
            // u32 wrap), the four row sums combine in 64 bits -- exact, as the f64 sum
            unsigned r = ls;
            r += dpp<0xB1>(r);
            r += dpp<0x4E>(r);
            r += dpp<0x141>(r);
            r += dpp<0x140>(r);
            sd = (Sd)(((uint64_t)rl(r, 0) + rl(r, 16)) + ((uint64_t)rl(r, 32) + rl(r, 48)) -
                      (uint64_t)pad * cp);
        } else {
            sd = (Sd)(wave_sum_f64_b((double)ls) - (double)((uint64_t)pad * cp));  // exact
        }
    } else {  // rare: a ring spanning >= 16.7 ms
        uint64_t sdi;
        if (range < 0x80000000u) {
            lane_sums<PL>(v, c, sdi, acc);
        } else {
            c = 0u;
            lane_sums_f64<PL>(v, sdi, acc);
            if (!FULL) acc -= lane == 0 ? (double)pad * ((double)cp * (double)cp) : 0.0;
        }
        sd = (Sd)(wave_sum_f64_b((double)sdi) - (double)((uint64_t)pad * cp));
    }
    const double sq = wave_sum_f64_b(acc);

    // ---- first histogram level ----
    // KEEPBIN (short segments, registers to spare): every sample's level-0 bin stays in a
    // register, so the level-0 candidate test is one compare instead of a subtract, a shift
    // and a compare
    constexpr bool KEEPBIN = KB;
    unsigned hb[KEEPBIN ? PL : 1];
    const int bits = 32 - __clz((int)range);
    int shift = bits > LOGNB ? bits - LOGNB : 0;
    const unsigned xc = B + cp;  // the padding's value
    // the padding's bin starts at -pad: at level 0 bin ubfe(x, shift, LOGNB) (the window is
    // every value; NB << shift may be 2^32), below it [wlo, wlo + NB << shift) if it holds xc
    const auto clear_bins = [&](unsigned wlo_, int shift_, bool level0) {
        const unsigned q = xc - wlo_;
        const unsigned pb = !(!FULL && pad) ? 0xFFFFFFFFu
                            : level0 ? __builtin_amdgcn_ubfe(xc, (unsigned)shift_, (unsigned)LOGNB)
                            : q < ((unsigned)NB << shift_) ? q >> shift_ : 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < BPL; ++j) hist[lane * BPL + j] = (unsigned)(lane * BPL + j) == pb ? 0u - pad : 0u;
    };
    if (FULL) {
#pragma unroll
        for (int j = 0; j < BPL; ++j) hist[lane * BPL + j] = 0u;
    } else {
        clear_bins(B, shift, true);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < PL; ++i) {
        const unsigned h = __builtin_amdgcn_ubfe(v[i], (unsigned)shift, (unsigned)LOGNB);  // d >> shift
        if (KEEPBIN) hb[KEEPBIN ? i : 0] = h;
        atomicAdd(&hist[h], 1u);
    }
    __builtin_amdgcn_wave_barrier();

    const unsigned t0 = (unsigned)((n & 1) ? n / 2 : n / 2 - 1);
    const unsigned t1 = (unsigned)(n / 2);
    unsigned wlo = B, below = 0, d0 = 0, d1 = 0;
    // every level narrows the window by LOGNB bits and shift reaches 0 (an exit) by level
    // ceil(32 / LOGNB): the bound only makes that explicit, so no wave can spin here (round 3's
    // gfx950 hang was a loop of this shape with control flow merged into its exits)
    constexpr int LEVELS = (32 + LOGNB - 1) / LOGNB + 1;
#pragma unroll 1
    for (int level = 0; level < LEVELS; ++level) {
        if (level > 0) {
            if (FULL) {
#pragma unroll
                for (int j = 0; j < BPL; ++j) hist[lane * BPL + j] = 0u;
            } else {
                clear_bins(wlo, shift, false);
            }
            __builtin_amdgcn_wave_barrier();
            const unsigned span = (unsigned)NB << shift;
#pragma unroll
            for (int i = 0; i < PL; ++i) {
                const unsigned q = v[i] - wlo;
                if (q < span) atomicAdd(&hist[q >> shift], 1u);
            }
            __builtin_amdgcn_wave_barrier();
        }
        // rank t1 = t0 or t0 + 1: usually in t0's bucket, so locate t0 alone and t1 only
        // when it lies past that bucket (a wave-uniform branch)
        unsigned b0, c0, n0, b1;
        hist_locate1<PL>(hist, t0 - below, b0, c0, n0);
        if (t1 - below < c0 + n0) {
            b1 = b0;
        } else {
            unsigned c1, n1;
            hist_locate1<PL>(hist, t1 - below, b1, c1, n1);
        }
        if (b0 != b1) {
            const unsigned hi0 = wlo + ((b0 + 1) << shift);
            const unsigned lo1 = wlo + (b1 << shift);
            unsigned a = 0u, z = 0xFFFFFFFFu;
#pragma unroll
            for (int i = 0; i < PL; i += 2) {
                a = max(a, max(v[i] - hi0, v[i + 1] - hi0));
                z = min(z, min(v[i] - lo1, v[i + 1] - lo1));
            }
            d0 = wave_max_b(a) + hi0;
            d1 = wave_min_b(z) + lo1;
            break;
        }
        if (shift == 0) {
            d0 = d1 = wlo + b0;
            break;
        }
        if (n0 <= 64u) {
            // compact the <= 64 candidates of bucket b0 into LDS (the histogram is consumed)
            __builtin_amdgcn_wave_barrier();
            unsigned base = 0;
            const unsigned lo0 = wlo + (b0 << shift);
            const unsigned width = 1u << shift;
            const bool masked = !FULL && pad && xc - lo0 < width;  // the padding is in bucket b0
            if (masked) {
#pragma unroll
                for (int i = 0; i < PL; ++i) {
                    const bool in = v[i] - lo0 < width && real(i);
                    const uint64_t bm = __ballot(in);
                    if (in) hist[base + mbcnt(bm)] = v[i];
                    base += (unsigned)__popcll(bm);
                }
            } else if (KEEPBIN && level == 0) {
#pragma unroll
                for (int i = 0; i < PL; ++i) {
                    const bool in = hb[KEEPBIN ? i : 0] == b0;
                    const uint64_t bm = __ballot(in);
                    if (in) hist[base + mbcnt(bm)] = v[i];
                    base += (unsigned)__popcll(bm);
                }
            } else {
#pragma unroll
                for (int i = 0; i < PL; ++i) {
                    const bool in = v[i] - lo0 < width;
                    const uint64_t bm = __ballot(in);
                    if (in) hist[base + mbcnt(bm)] = v[i];
                    base += (unsigned)__popcll(bm);
                }
            }
            __builtin_amdgcn_wave_barrier();
            const unsigned ci = (lane < (int)n0) ? hist[lane] : 0xFFFFFFFFu;
            unsigned rank = 0;
            if (shift <= 26) {
                // unique keys (candidate - lo0, lane) in one word: rank = keys below mine, one
                // compare per candidate; lanes >= n0 hold the maximum and never count
                const unsigned key = (lane < (int)n0) ? ((ci - lo0) << 6) | (unsigned)lane : 0xFFFFFFFFu;
                for (int j = 0; j < (int)n0; j += 4) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) rank += (rl(key, j + u) < key) ? 1u : 0u;
                }
            } else {
                for (int j = 0; j < (int)n0; ++j) {
                    const unsigned cj = __builtin_amdgcn_readlane(ci, j);
                    rank += (cj < ci || (cj == ci && j < lane)) ? 1u : 0u;
                }
            }
            const unsigned r0 = t0 - below - c0, r1 = t1 - below - c0;
            const int L0 = __builtin_ffsll(__ballot(lane < (int)n0 && rank == r0)) - 1;
            const int L1 = __builtin_ffsll(__ballot(lane < (int)n0 && rank == r1)) - 1;
            d0 = __builtin_amdgcn_readlane(ci, L0);
            d1 = __builtin_amdgcn_readlane(ci, L1);
            break;
        }
        below += c0;
        wlo += b0 << shift;
        shift = shift > LOGNB ? shift - LOGNB : 0;
    }
    return LeanOut<PL>{mn, mx, d0 - B, d1 - B, c, sd, sq};
}

template <int PL>
__device__ __forceinline__ unsigned lean_body(unsigned (&v)[PL], int n, unsigned x0, int64_t s,
                                          unsigned* hist, const nvrx_stats_soa& out,
                                          const ColRef& cr) {
    const LeanOut<PL> r = lean_core<PL>(v, n, 0, x0, hist);
    emit_stats(out, s, n, r.mn, r.mx, r.d0, r.d1, (double)r.sd, r.sq, r.c, cr);
    return r.mx;
}

// HBM -> VGPR in two steps, so a caller can issue the next segment's loads before it
// reduces the current one.  issue_loads: the segment p[0:n) into v (64*PL slots, see
// lean_core) with 16-byte buffer loads from the 16-B aligned base below p; the descriptor
// is built from wave-uniform (readfirstlane'd) inputs so the loads issue back to back (no
// waterfall); lanes past the segment fall outside the descriptor's range (the hardware
// returns 0).  finish_loads (after the loads landed): m0 = p's offset in its 16-B vector
// (in samples), x0 = sample 0 (lane 0's slot m0: no extra memory access); !FULL sets the
// slots outside the segment to x0 (a sample: neutral for MIN/MAX).
template <int PL>
__device__ __forceinline__ void issue_loads(const uint32_t* p, int n, unsigned (&v)[PL]) {
    constexpr int NV = PL / 4;
    const int lane = lane_id();
    const uintptr_t pa = (uintptr_t)p & ~(uintptr_t)15;
    const int m0 = (int)(((uintptr_t)p & 15) >> 2);
    const int nvec = (n + m0 + 3) >> 2;
    const unsigned pa_lo = __builtin_amdgcn_readfirstlane((unsigned)pa);
    const unsigned pa_hi = __builtin_amdgcn_readfirstlane((unsigned)(pa >> 32));
    const int nbytes = __builtin_amdgcn_readfirstlane(nvec * 16);
    void* const pbase = (void*)(((uint64_t)pa_hi << 32) | pa_lo);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(pbase, 0, nbytes, 0x00020000);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane * 16, j * 1024, NVRX_LOAD_AUX);
        v[4 * j + 0] = q.x;
        v[4 * j + 1] = q.y;
        v[4 * j + 2] = q.z;
        v[4 * j + 3] = q.w;
    }
}

template <int PL, bool FULL>
__device__ __forceinline__ void finish_loads(const uint32_t* p, int n, unsigned (&v)[PL], int& m0,
                                             unsigned& x0) {
    const int lane = lane_id();
    m0 = FULL ? 0 : (int)(((uintptr_t)p & 15) >> 2);
    const unsigned e0 = m0 == 0 ? v[0] : m0 == 1 ? v[1] : m0 == 2 ? v[2] : v[3];
    x0 = __builtin_amdgcn_readlane(e0, 0);
    // a masked-class segment that happens to fill the wave exactly (configs[3]: every ring at
    // cap = 8192) needs no masking (wave-uniform test)
    if (!FULL && (n != 64 * PL || m0 != 0)) {
#pragma unroll
        for (int i = 0; i < PL; ++i) {
            const unsigned e = (unsigned)(((i >> 2) * 64 + lane) * 4 + (i & 3) - m0);
            v[i] = (e < (unsigned)n) ? v[i] : x0;
        }
    }
}

template <int PL, bool FULL>
__device__ __forceinline__ void load_segment(const uint32_t* p, int n, unsigned (&v)[PL], int& m0,
                                             unsigned& x0) {
    issue_loads<PL>(p, n, v);
    finish_loads<PL, FULL>(p, n, v, m0, x0);
}

// FULL: the host guarantees every segment holds exactly 64*PL samples starting on a
// 16-byte boundary, so no lane needs masking.  !FULL: per-element masks (branch-free).
template <int PL, bool FULL, class Segs>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OccV<PL, FULL>::W)))
void seg_stats_fast_kernel(Segs segs, int64_t nseg, nvrx_stats_soa out, ColRef cr) {
    constexpr int NB = Bins<PL>::NB;
    __shared__ __attribute__((aligned(16))) unsigned lds_hist[4 * NB];

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id();
    const int64_t s = (int64_t)blockIdx.x * 4 + wave;
    if (s >= nseg) return;  // wave-uniform; the kernel has no workgroup barrier
    unsigned* hist = lds_hist + wave * NB;

    const uint32_t* p;
    int n;
    segs.get(s, p, n);
    if (n <= 0) {  // n < 0: segment reduced elsewhere (records_stats), outputs untouched
        if (n == 0 && lane == 0) {
            write_empty(out, s);
            cr.miss(s);
        }
        return;
    }

    unsigned v[PL];
    int m0;
    unsigned x0;
    load_segment<PL, FULL>(p, n, v, m0, x0);
    const LeanOut<PL> r = lean_core<PL, FULL>(v, n, m0, x0, hist);
    emit_stats(out, s, n, r.mn, r.mx, r.d0, r.d1, (double)r.sd, r.sq, r.c, cr);
    // keys of >= 3.76 s take the decoded moments (rare, wave-uniform)
    if (r.mx >= NVRX_KEY_WIDE) wide_moments(p, n, s, out);
}

// FULL segments only (64*PL samples each, 16-B aligned): lean_body.
template <int PL, class Segs>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(Occ<PL>::W)))
void seg_stats_lean_kernel(Segs segs, int64_t nseg, nvrx_stats_soa out, ColRef cr) {
    constexpr int NB = Bins<PL>::NB;
    __shared__ __attribute__((aligned(16))) unsigned lds_hist[4 * NB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t s = (int64_t)blockIdx.x * 4 + wave;
    if (s >= nseg) return;
    unsigned* hist = lds_hist + wave * NB;
    const uint32_t* p;
    int n;
    segs.get(s, p, n);
    unsigned v[PL];
    int m0;
    unsigned x0;
    load_segment<PL, true>(p, n, v, m0, x0);
    if (lean_body<PL>(v, n, x0, s, hist, out, cr) >= NVRX_KEY_WIDE) wide_moments(p, n, s, out);
}

// FULL segments (configs[1] / configs[2]): each wave reduces `group` consecutive segments one
// after another and keeps what lean_core returns for segment s0 + j in lane j (one compare and
// nine selects), so the epilogue -- the unit conversions, the f64 quotients and the root, the
// stores -- runs once per group, lane-parallel with coalesced stores, instead of once per
// segment on one busy lane (~55 VALU, half of them f64).  Same arithmetic as emit_stats, so the
// same bits.  Groups of up to 8 (lean_group): the sweep on configs[2] in DESIGN.md section 3.1.
#ifndef NVRX_GROUP_WAVES  // waves per workgroup of the group kernel (build-time tuning constant)
#define NVRX_GROUP_WAVES 4
#endif
template <int PL, class Segs>
__global__ __launch_bounds__(64 * NVRX_GROUP_WAVES) __attribute__((amdgpu_waves_per_eu(Occ<PL>::W)))
void seg_stats_lean_group_kernel(Segs segs, int64_t nseg, int group, nvrx_stats_soa out, ColRef cr) {
    constexpr int NB = Bins<PL>::NB;
    __shared__ __attribute__((aligned(16))) unsigned lds_hist[NVRX_GROUP_WAVES * NB];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id();
    const int64_t s0 = ((int64_t)blockIdx.x * NVRX_GROUP_WAVES + wave) * group;
    if (s0 >= nseg) return;
    const int cnt = (int)(nseg - s0 < group ? nseg - s0 : group);
    unsigned* hist = lds_hist + wave * NB;
    unsigned a_mn = 0, a_mx = 0, a_k0 = 0, a_k1 = 0, a_c = 0, a_sdlo = 0, a_sdhi = 0, a_sqlo = 0, a_sqhi = 0;
    uint64_t wide = 0;
    int n = 0;
    for (int j = 0; j < cnt; ++j) {
        const uint32_t* p;
        segs.get(s0 + j, p, n);
        unsigned v[PL];
        int m0;
        unsigned x0;
        load_segment<PL, true>(p, n, v, m0, x0);
        const LeanOut<PL> r = lean_core<PL>(v, n, 0, x0, hist);
        const uint64_t sqb = (uint64_t)__double_as_longlong(r.sq);
        const bool mine = lane == j;  // one compare, nine selects
        a_mn = mine ? r.mn : a_mn;
        a_mx = mine ? r.mx : a_mx;
        a_k0 = mine ? r.mn + r.d0 : a_k0;
        a_k1 = mine ? r.mn + r.d1 : a_k1;
        a_c = mine ? r.c : a_c;
        const uint64_t sdb = sd_bits(r.sd);
        a_sdlo = mine ? (uint32_t)sdb : a_sdlo;
        a_sdhi = mine ? (uint32_t)(sdb >> 32) : a_sdhi;
        a_sqlo = mine ? (uint32_t)sqb : a_sqlo;
        a_sqhi = mine ? (uint32_t)(sqb >> 32) : a_sqhi;
        if (r.mx >= NVRX_KEY_WIDE) wide |= 1ull << j;
    }
    if (lane < cnt)
        emit_lane(out, s0 + lane, n, a_mn, a_mx, a_k0, a_k1,
                  sd_value<PL>(((uint64_t)a_sdhi << 32) | a_sdlo),
                  __longlong_as_double((long long)(((uint64_t)a_sqhi << 32) | a_sqlo)), a_c, cr);
    while (wide) {  // keys of >= 3.76 s: the decoded moments (rare)
        const int j = __builtin_ffsll(wide) - 1;
        wide &= wide - 1;
        const uint32_t* p;
        segs.get(s0 + j, p, n);
        wide_moments(p, n, s0 + j, out);
    }
}

// Batcher's odd-even merge sort over N registers (N a power of two) as a compile-time list of
// compare-exchanges -- v_min/v_max pairs, no LDS, no branches: 19 / 63 / 191 / 543 / 1471 of them
// for N = 8 / 16 / 32 / 64 / 128, against the bitonic network's 24 / 80 / 240 / 672 / 1792.
template <int N>
struct OemNet {
    template <class F>
    static constexpr void walk(F&& f) {
        for (int p = 1; p < N; p += p)
            for (int k = p; k > 0; k /= 2)
                for (int j = k % p; j + k < N; j += k + k)
                    for (int i = 0; i < k && i + j + k < N; ++i)
                        if ((i + j) / (p + p) == (i + j + k) / (p + p)) f(i + j, i + j + k);
    }
    static constexpr int count() {
        int c = 0;
        walk([&](int, int) { ++c; });
        return c;
    }
    static constexpr int NC = count();
    short a[NC], b[NC];
    constexpr OemNet() : a(), b() {
        int c = 0;
        walk([&](int x, int y) {
            a[c] = (short)x;
            b[c] = (short)y;
            ++c;
        });
    }
};
// compare-exchanges [LO, HI) of the network, split in halves down to single ones, so every
// register index is a constant expression (a loop over the table left 128-register networks
// with runtime indices: the array went to scratch)
template <int N, int LO, int HI>
__device__ __forceinline__ void net_range(unsigned (&v)[N]) {
    if constexpr (HI - LO == 1) {
        constexpr OemNet<N> net{};
        constexpr int a = net.a[LO], b = net.b[LO];
        const unsigned x = v[a], y = v[b];
        v[a] = min(x, y);
        v[b] = max(x, y);
    } else if constexpr (HI - LO > 1) {
        net_range<N, LO, (LO + HI) / 2>(v);
        net_range<N, (LO + HI) / 2, HI>(v);
    }
}
template <int N>
__device__ __forceinline__ void sort_net(unsigned (&v)[N]) {
    net_range<N, 0, OemNet<N>::NC>(v);
}

constexpr int pow2_ceil(int m) {
    int p = 1;
    while (p < m) p += p;
    return p;
}
// v[idx] for a runtime idx known to lie in the compile-time range [LO, HI] (any register of the
// range otherwise): a multiplexer tree on the bits of idx - LO, one v_cndmask per candidate,
// instead of a compare and a select per register.
template <int LO, int HI, int N>
__device__ __forceinline__ unsigned pick(const unsigned (&v)[N], int idx) {
    constexpr int P = pow2_ceil(HI - LO + 1);
    unsigned t[P];
#pragma unroll
    for (int j = 0; j < P; ++j) t[j] = v[LO + j <= HI ? LO + j : HI];
    const unsigned k = (unsigned)(idx - LO);
#pragma unroll
    for (int w = P, bit = 1; w > 1; w >>= 1, bit += bit) {
        const bool hi = (k & (unsigned)bit) != 0u;
#pragma unroll
        for (int j = 0; j < w / 2; ++j) t[j] = hi ? t[2 * j + 1] : t[2 * j];
    }
    return t[0];
}

// One segment of n samples per LANE, NMIN <= n <= N (v: the n samples in slots [0, n) in any
// order, slots >= n ignored; a length class guarantees NMIN, so slots below it need no masks).
// u32 -> f32 us is monotone, so sorting the integer ns sorts the floats computeStats sorts; then
// CuptiProfiler.cpp:53-71 statement by statement (sequential f32 sums over the sorted samples)
// -- every field bit-exact.
template <int N, int NMIN = 1>
__device__ __forceinline__ void lane_stats(unsigned (&v)[N], int n, int64_t s,
                                           const nvrx_stats_soa& out, const ColRef& cr) {
    static_assert(NMIN >= 1 && NMIN <= N, "NMIN in [1, N]");
#pragma unroll
    for (int j = NMIN; j < N; ++j) v[j] = j < n ? v[j] : 0xFFFFFFFFu;  // sentinels sort last
    sort_net<N>(v);
    float acc = 0.0f;
    // keys of 3.76 s and more (rare) are decoded; the wave takes the plain conversion unless
    // one of its lanes holds such a key
    const bool wide = __ballot(pick<NMIN - 1, N - 1>(v, n - 1) >= NVRX_KEY_WIDE) != 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const float f = wide ? ns_to_us(v[j]) : ns_to_us_narrow(v[j]);
        v[j] = __float_as_uint(f);
        acc = (j < NMIN || j < n) ? acc + f : acc;  // accumulate(sorted, 0.0f): sequential f32
    }
    // s[n-1], s[n/2] and s[n/2 - 1] (the latter read only for even n >= 2)
    const float fmin = __uint_as_float(v[0]);
    const float fmax = __uint_as_float(pick<NMIN - 1, N - 1>(v, n - 1));
    const float f1 = __uint_as_float(pick<NMIN / 2, N / 2>(v, n / 2));
    const float f0 = __uint_as_float(pick<(NMIN / 2 > 0 ? NMIN / 2 - 1 : 0), N / 2 - 1>(v, n / 2 - 1));
    const float med = (n & 1) ? f1 : (f0 + f1) / 2;
    const float avg = acc / (float)n;
    float sq = 0.0f;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const float t = __uint_as_float(v[j]) - avg;
        sq = (j < NMIN || j < n) ? sq + t * t : sq;
    }
    out.num[s] = n;
    out.min[s] = fmin;
    out.max[s] = fmax;
    out.med[s] = med;
    out.avg[s] = avg;
    out.std[s] = (float)__builtin_sqrt((double)(sq / (float)n));  // sqrtf, correctly rounded
    cr.add(s, med);
}

// ---------------------------------------------------------------------------
// EXACT mode: one 256-thread workgroup per segment, bitonic sort in LDS.
// ---------------------------------------------------------------------------
// Block-wide body: the segment p[0:n), n >= 1, into sbuf[NMAX] (LDS), sorted, then the
// reference's statistics statement by statement.  Every thread of the block calls it.
template <int NMAX>
__device__ __forceinline__ void exact_body(const uint32_t* p, int n, int64_t s, float* sbuf,
                                           const nvrx_stats_soa& out, const ColRef& cr) {
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int i = threadIdx.x; i < np2; i += blockDim.x)
        sbuf[i] = (i < n) ? ns_to_us(p[i]) : __builtin_inff();
    __syncthreads();
    // bitonic sort, ascending (+inf padding sorts last)
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < np2; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const float a = sbuf[i], b = sbuf[ixj];
                    const bool up = (i & k) == 0;
                    if (up ? (a > b) : (a < b)) {
                        sbuf[i] = b;
                        sbuf[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) {
        // CuptiProfiler.cpp:53-71, statement by statement
        const float mnv = sbuf[0], mxv = sbuf[n - 1];
        float med;
        if (n % 2 == 0)
            med = (sbuf[n / 2 - 1] + sbuf[n / 2]) / 2;
        else
            med = sbuf[n / 2];
        float acc = 0.0f;
        for (int i = 0; i < n; ++i) acc = acc + sbuf[i];
        const float avg = acc / (float)n;
        float sqs = 0.0f;
        for (int i = 0; i < n; ++i) {
            const float t = sbuf[i] - avg;
            sqs = sqs + t * t;
        }
        // sqrtf, correctly rounded: f64 sqrt then one rounding to f32 is exact for sqrt
        const float sd = (float)__builtin_sqrt((double)(sqs / (float)n));
        out.num[s] = n;
        out.min[s] = mnv;
        out.max[s] = mxv;
        out.med[s] = med;
        cr.add(s, med);
        out.avg[s] = avg;
        out.std[s] = sd;
    }
    __syncthreads();  // sbuf is reused by the block's next segment
}

template <int NMAX, class Segs>
__global__ __launch_bounds__(256) void seg_stats_exact_kernel(Segs segs, int64_t nseg,
                                                              nvrx_stats_soa out, ColRef cr) {
    __shared__ __attribute__((aligned(16))) float sbuf[NMAX];
    const int64_t s = blockIdx.x;
    if (s >= nseg) return;
    const uint32_t* p;
    int n;
    segs.get(s, p, n);
    if (n <= 0) {  // n < 0: reduced elsewhere
        if (n == 0 && threadIdx.x == 0) {
            write_empty(out, s);
            cr.miss(s);
        }
        return;
    }
    exact_body<NMAX>(p, n, s, sbuf, out, cr);
}

// ---------------------------------------------------------------------------
// Rings longer than the LDS holds (statsMaxLenPerKernel > NVRX_LDS_SEGMENT; the reference's
// CircularBuffer takes any capacity, CuptiProfiler.h:49-51).  One 1024-thread workgroup per
// segment sorts its samples in a slice `g` of a device scratch buffer (np2 floats): the bitonic
// stages whose partner distance j reaches XG_CHUNK run in global memory; for every k the stages
// below it stay inside aligned XG_CHUNK blocks, which are sorted in LDS.  The sequential f32 sums
// of computeStats then run on one lane over the sorted samples staged through LDS chunk by
// chunk -- the same statements, so every field is bit-exact.  Global stores are visible to the
// block after __syncthreads (one workgroup, one CU).
// ---------------------------------------------------------------------------
#define XG_CHUNK 8192
#define XG_THREADS 1024
__device__ __forceinline__ void bitonic_step(float* b, int i, int j, int k) {
    const int ixj = i ^ j;
    if (ixj > i) {
        const float a = b[i], c = b[ixj];
        if (((i & k) == 0) ? (a > c) : (a < c)) {
            b[i] = c;
            b[ixj] = a;
        }
    }
}

__device__ __forceinline__ void exact_global_body(const uint32_t* p, int n, int64_t s, float* g,
                                                  float* lds, const nvrx_stats_soa& out,
                                                  const ColRef& cr) {
    int np2 = XG_CHUNK;
    while (np2 < n) np2 <<= 1;
    for (int i = threadIdx.x; i < np2; i += XG_THREADS) g[i] = (i < n) ? ns_to_us(p[i]) : __builtin_inff();
    __syncthreads();
    // the stages of k <= XG_CHUNK, one aligned chunk at a time in LDS; then, for every larger k,
    // the global stages (j >= XG_CHUNK) and the remaining ones per chunk in LDS.  The direction
    // bit (i & k) is taken on the global index.
    for (int k = 2; k <= np2; k <<= 1) {
        if (k <= XG_CHUNK && k != 2) continue;  // k = 2 .. XG_CHUNK all run on the first visit
        const int kmax = k == 2 ? XG_CHUNK : k;
        int j = k >> 1;
        if (k > XG_CHUNK) {
            for (; j >= XG_CHUNK; j >>= 1) {  // partners XG_CHUNK or more apart: global memory
                for (int i = threadIdx.x; i < np2; i += XG_THREADS) bitonic_step(g, i, j, k);
                __syncthreads();
            }
        }
        for (int c0 = 0; c0 < np2; c0 += XG_CHUNK) {
            for (int i = threadIdx.x; i < XG_CHUNK; i += XG_THREADS) lds[i] = g[c0 + i];
            __syncthreads();
            for (int kk = k; kk <= kmax; kk <<= 1) {
                for (int jj = (kk == k ? j : kk >> 1); jj > 0; jj >>= 1) {
                    for (int i = threadIdx.x; i < XG_CHUNK; i += XG_THREADS) {
                        const int ixj = i ^ jj;
                        if (ixj > i) {
                            const float a = lds[i], c = lds[ixj];
                            if ((((c0 + i) & kk) == 0) ? (a > c) : (a < c)) {
                                lds[i] = c;
                                lds[ixj] = a;
                            }
                        }
                    }
                    __syncthreads();
                }
            }
            for (int i = threadIdx.x; i < XG_CHUNK; i += XG_THREADS) g[c0 + i] = lds[i];
            __syncthreads();
        }
    }
    // CuptiProfiler.cpp:53-71, statement by statement; the sums stage the sorted samples in LDS
    float acc = 0.0f;
    for (int c0 = 0; c0 < n; c0 += XG_CHUNK) {
        const int m = min(XG_CHUNK, n - c0);
        for (int i = threadIdx.x; i < m; i += XG_THREADS) lds[i] = g[c0 + i];
        __syncthreads();
        if (threadIdx.x == 0)
            for (int i = 0; i < m; ++i) acc = acc + lds[i];
        __syncthreads();
    }
    const float avg = acc / (float)n;  // meaningful on thread 0 only (the others never summed)
    float sqs = 0.0f;
    for (int c0 = 0; c0 < n; c0 += XG_CHUNK) {
        const int m = min(XG_CHUNK, n - c0);
        for (int i = threadIdx.x; i < m; i += XG_THREADS) lds[i] = g[c0 + i];
        __syncthreads();
        if (threadIdx.x == 0)
            for (int i = 0; i < m; ++i) {
                const float t = lds[i] - avg;
                sqs = sqs + t * t;
            }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float med = (n % 2 == 0) ? (g[n / 2 - 1] + g[n / 2]) / 2 : g[n / 2];
        out.num[s] = n;
        out.min[s] = g[0];
        out.max[s] = g[n - 1];
        out.med[s] = med;
        cr.add(s, med);
        out.avg[s] = avg;
        out.std[s] = (float)__builtin_sqrt((double)(sqs / (float)n));
    }
    __syncthreads();  // g and lds are reused by the block's next segment
}

// segments s0 + blockIdx.x (a chunk of the batch: the scratch holds one slice per block)
template <class Segs>
__global__ __launch_bounds__(XG_THREADS) void seg_stats_exact_global_kernel(
    Segs segs, int64_t s0, int64_t nseg, float* work, int64_t np2, nvrx_stats_soa out, ColRef cr) {
    __shared__ __attribute__((aligned(16))) float lds[XG_CHUNK];
    const int64_t s = s0 + blockIdx.x;
    if (s >= nseg) return;
    const uint32_t* p;
    int n;
    segs.get(s, p, n);
    if (n <= 0) {
        if (n == 0 && threadIdx.x == 0) {
            write_empty(out, s);
            cr.miss(s);
        }
        return;
    }
    exact_global_body(p, n, s, work + (int64_t)blockIdx.x * np2, lds, out, cr);
}

// scratch for the global path: np2 floats per block, bounded to ~256 MiB (at least one block)
static inline int64_t exact_global_np2(int64_t max_len) {
    int64_t np2 = XG_CHUNK;
    while (np2 < max_len) np2 <<= 1;
    return np2;
}
static inline int64_t exact_global_blocks(int64_t np2, int64_t want) {
    const int64_t per = std::max<int64_t>(1, ((int64_t)256 << 20) / (np2 * (int64_t)sizeof(float)));
    return std::max<int64_t>(1, std::min(want, per));
}

// ---------------------------------------------------------------------------
// Host-side launchers shared by segment_stats.hip and segment_ragged.hip
// ---------------------------------------------------------------------------
// col_ref: [min med bits | missing] per column, initialised to (+inf, 0) on `st` by one
// kernel (a launch that HIP graph capture records like any other; template: defined once
// across the translation units that include this header)
template <int U = 0>
__global__ void colref_init_kernel(uint32_t* col_ref, int64_t ncols) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 2 * ncols) col_ref[i] = i < ncols ? 0x7F800000u : 0u;
}
static inline hipError_t make_colref(uint32_t* col_ref, int64_t ncols, hipStream_t st, ColRef& cr,
                                     bool ready = false) {
    cr = ColRef{nullptr, nullptr, 1, 1.0};
    if (!col_ref || ncols <= 0) return hipSuccess;
    cr = ColRef{col_ref, col_ref + ncols, ncols, 1.0 / (double)ncols};
    if (ready) return hipSuccess;  // NVRX_STATS_COLREF_READY: initialised by the caller
    hipLaunchKernelGGL(colref_init_kernel<0>, dim3((unsigned)((2 * ncols + 255) / 256)), dim3(256), 0,
                       st, col_ref, ncols);
    return hipGetLastError();
}

// segments per wave of the group kernel: up to NVRX_LEAN_GROUP_MAX while the grid keeps >= 32768 waves
// Segments per wave of the group kernel: configs[2] statistics interleaved on one box
// (tools/build_variant.sh + tools/gpu_r03_variants.sh, profiles/r03/group_size/): 4 / 6 / 8 / 12
// / 32 / 64 per wave 5.70 / 5.87 / 5.57 / 5.78 / 6.04 / 5.87 ms (round-start library 6.00 ms);
// a prefetch of the next segment's loads (80 VGPRs, 6 waves / SIMD) 5.90-5.94 at 64.  A build
// constant, so A/B builds can override it.
#ifndef NVRX_LEAN_GROUP_MAX
#define NVRX_LEAN_GROUP_MAX 8
#endif
// one segment's results per lane, wide-key flags in a 64-bit mask
static_assert(NVRX_LEAN_GROUP_MAX >= 1 && NVRX_LEAN_GROUP_MAX <= 64, "NVRX_LEAN_GROUP_MAX in [1, 64]");
#ifndef NVRX_LEAN_GROUP_PL_MAX  // FULL segments of up to 64 * this many samples take the group kernel
#define NVRX_LEAN_GROUP_PL_MAX 128
#endif
#ifndef NVRX_LEAN_GROUP_WAVES  // build-time tuning constant: the fewest waves a grouped grid keeps
#define NVRX_LEAN_GROUP_WAVES 32768
#endif
static inline int lean_group(int64_t nseg) {
    const int64_t g = nseg / NVRX_LEAN_GROUP_WAVES;
    return g < 1 ? 1 : g > NVRX_LEAN_GROUP_MAX ? NVRX_LEAN_GROUP_MAX : (int)g;
}

template <int PL, class Segs>
static void launch_pl(const Segs& segs, int64_t nseg, bool full, const nvrx_stats_soa& out,
                      const ColRef& cr, hipStream_t st) {
    const dim3 grid((unsigned)((nseg + 3) / 4)), block(256);
    // FULL: unmasked lean_core with the group epilogue (one segment per wave above
    // NVRX_LEAN_GROUP_PL_MAX, a build-time choice); otherwise the masked lean_core
    if (full) {
        if constexpr (PL <= NVRX_LEAN_GROUP_PL_MAX) {
            const int g = lean_group(nseg);
            const int64_t waves = (nseg + g - 1) / g;
            hipLaunchKernelGGL((seg_stats_lean_group_kernel<PL, Segs>),
                               dim3((unsigned)((waves + NVRX_GROUP_WAVES - 1) / NVRX_GROUP_WAVES)),
                               dim3(64 * NVRX_GROUP_WAVES), 0, st, segs, nseg, g, out, cr);
        } else {
            hipLaunchKernelGGL((seg_stats_lean_kernel<PL, Segs>), grid, block, 0, st, segs, nseg, out, cr);
        }
    } else {
        hipLaunchKernelGGL((seg_stats_fast_kernel<PL, false, Segs>), grid, block, 0, st, segs, nseg, out, cr);
    }
}

// need = samples + alignment slack a wave must hold; picks the smallest PL.  `full`
// (every segment exactly 64*PL samples, 16-B aligned) selects the unmasked variant.
template <class Segs>
static hipError_t launch_fast(const Segs& segs, int64_t nseg, int64_t need, int64_t exact_len,
                              const nvrx_stats_soa& out, const ColRef& cr, hipStream_t st) {
    if (need <= 64 * 4)
        launch_pl<4>(segs, nseg, exact_len == 64 * 4, out, cr, st);
    else if (need <= 64 * 8)
        launch_pl<8>(segs, nseg, exact_len == 64 * 8, out, cr, st);
    else if (need <= 64 * 16)
        launch_pl<16>(segs, nseg, exact_len == 64 * 16, out, cr, st);
    else if (need <= 64 * 32)
        launch_pl<32>(segs, nseg, exact_len == 64 * 32, out, cr, st);
    else if (need <= 64 * 64)
        launch_pl<64>(segs, nseg, exact_len == 64 * 64, out, cr, st);
    else if (need <= 64 * 128)
        launch_pl<128>(segs, nseg, exact_len == 64 * 128, out, cr, st);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

template <class Segs>
static hipError_t launch_exact(const Segs& segs, int64_t nseg, int64_t max_len,
                               const nvrx_stats_soa& out, const ColRef& cr, hipStream_t st) {
    const dim3 grid((unsigned)nseg), block(256);
    if (max_len <= 1024)
        hipLaunchKernelGGL((seg_stats_exact_kernel<1024, Segs>), grid, block, 0, st, segs, nseg, out, cr);
    else if (max_len <= 8192)
        hipLaunchKernelGGL((seg_stats_exact_kernel<8192, Segs>), grid, block, 0, st, segs, nseg, out, cr);
    else if (max_len <= NVRX_LDS_SEGMENT)
        hipLaunchKernelGGL((seg_stats_exact_kernel<NVRX_LDS_SEGMENT, Segs>), grid, block, 0, st, segs, nseg, out, cr);
    else if (max_len <= NVRX_MAX_SEGMENT) {
        // longer rings: device scratch, the batch in chunks of blocks (one slice each)
        const int64_t np2 = exact_global_np2(max_len), chunk = exact_global_blocks(np2, nseg);
        void* work = nullptr;
        hipError_t e = scratch_alloc(&work, (size_t)(chunk * np2) * sizeof(float), st);
        if (e != hipSuccess) return e;
        for (int64_t s0 = 0; s0 < nseg && e == hipSuccess; s0 += chunk) {
            hipLaunchKernelGGL((seg_stats_exact_global_kernel<Segs>), dim3((unsigned)std::min(chunk, nseg - s0)),
                               dim3(XG_THREADS), 0, st, segs, s0, nseg, (float*)work, np2, out, cr);
            e = hipGetLastError();
        }
        const hipError_t f = hipFreeAsync(work, st);  // on the error path too
        return e != hipSuccess ? e : f;
    } else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace nvrx
