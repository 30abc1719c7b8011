// records_resident.hip -- record streams -> per-(stream, slot) statistics in ONE pass over HBM
// (gfx950).  FAST-mode nvrx_records_stats for streams that fit on chip.
//
// Replaces, per rank, the reference's record loop and rings (CuptiProfiler.cpp:168-203,
// CircularBuffer.h:53-69: the LAST `cap` pushes of every key) followed by getStats /
// computeStats (CuptiProfiler.cpp:44-74, 136-146).  records.hip + the ragged class kernels
// do the same in three memory passes (stream in, buckets out, buckets in again); here one
// workgroup holds its whole stream on chip and never writes the buckets:
//
//   load   : the stream -> VGPRs, RR_PPL 16-byte record pairs per lane (8 waves x 64 lanes x
//            47 pairs = 48,128 records; a CU's register file is 512 KiB and the stream takes
//            376 KiB of it), every load issued before the first is consumed;
//   count  : LDS histogram of slots (no-return LDS atomics from the registers);
//   scan   : keep = min(count, cap), buckets laid out in slot order, each padded to 4 records
//            (16-byte aligned LDS reads), counts / seg_len written;
//   groups : consecutive slot ranges whose buckets fit the LDS stage (configs[3]: 2);
//            per group
//     place: every register-held record of the group's slots takes a returning LDS atomic
//            cursor and lands in the stage (order inside a bucket is free: computeStats
//            sorts); records of a slot that overflowed its ring are placed in push order by
//            wave 0 walking the stream (it keeps the LAST `cap`);
//     stats: buckets of <= RR_LANE_MAX records one lane each (lane_stats: computeStats
//            statement by statement, every field bit-exact), longer ones one wave each
//            from LDS through a dynamic queue (lds_wave_stats: NUM/MIN/MAX/MED bit-exact by
//            radix select, AVG/STD the FAST-mode exact mean / std rounded once, as the
//            segment kernels' emit_stats).
// HBM traffic: 8 B per record in, 24 B of statistics + 8 B of counts / lengths per (stream,
// slot) out -- against 8 + 4 + 4 (+ re-reads) per record for bucket + class kernels.
// A stream longer than the register capacity takes the same steps with its records re-read
// from memory at each pass (correct for any length; configs[3] never needs it).
#include "segment_kernels.h"

// Timing ablations for tools/rr_bench.hip only (never in the library build): NVRX_AB_RR bit
// 1 = skip the wave-path statistics, 2 = skip the lane-path statistics, 4 = skip placement,
// 8 = skip counting.
#ifndef NVRX_AB_RR
#define NVRX_AB_RR 0
#endif
#ifdef RR_DEBUG
#define RR_TRACE(...) do { if (blockIdx.x == 0 && threadIdx.x == 0) printf(__VA_ARGS__); } while (0)
// progress words in host-mapped memory, polled by tools/rr_debug.hip while the kernel runs:
// [wave] = last phase reached by wave `wave` of block 0, [8 + wave] = a value of that phase
__device__ uint32_t* rr_dbg_ptr;
#define RR_MARK(phase, val) do { if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && rr_dbg_ptr) { \
    rr_dbg_ptr[threadIdx.x >> 6] = (phase); rr_dbg_ptr[8 + (threadIdx.x >> 6)] = (val); __threadfence_system(); } } while (0)
#else
#define RR_TRACE(...) do {} while (0)
#define RR_MARK(phase, val) do {} while (0)
#endif

namespace nvrx {

constexpr int RR_WAVES = 8;
constexpr int RR_THREADS = 64 * RR_WAVES;
constexpr int RR_PPL = 47;  // record pairs (16 B) per lane held in VGPRs: 188 of 256
constexpr int64_t RR_CAPACITY = (int64_t)RR_PPL * 2 * RR_THREADS;
constexpr int RR_LANE_MAX = 16;    // buckets of up to this many records: one lane each
constexpr int RR_LANE_FINAL = 64;  // ... in the last group (the stream's registers freed)
constexpr int RR_SLOT_BITS = 13;   // register keys: bucket start << 13 | slot (nslots < 8192)
constexpr int RR_NB = 256;       // histogram bins per wave (Bins<16>, hist_locate1<16>)
constexpr uint32_t RR_OVF = 0x80000000u;
constexpr size_t RR_LDS = 160 * 1024 - 256;  // one workgroup per CU takes the whole LDS

// LDS words of everything but the stage
__host__ __device__ __forceinline__ int64_t rr_fixed_words(int64_t nslots) {
    return ((4 * nslots + 3) & ~(int64_t)3) + RR_WAVES * RR_NB;
}
int64_t records_resident_stage(int64_t nslots) {
    const int64_t w = (int64_t)(RR_LDS / 4) - rr_fixed_words(nslots);
    return w > 0 ? (w & ~(int64_t)3) : 0;
}

// Element-wise walk of seg[0:n) (LDS, 16-B aligned) by one wave: lane L takes elements
// 4L..4L+3 of every 256-element block.  The loop is wave-uniform (every lane runs every
// block; f gets a validity flag), so ballots inside f see the whole wave.
template <class F>
__device__ __forceinline__ void lds_walk(const uint32_t* seg, int n, F&& f) {
    const int lane = lane_id();
    for (int b = 0; b < n; b += 256) {
        const int i = b + lane * 4;
        u32x4 q = {0u, 0u, 0u, 0u};
        if (i < n) q = *(const u32x4*)(seg + i);
        f(q.x, i < n);
        f(q.y, i + 1 < n);
        f(q.z, i + 2 < n);
        f(q.w, i + 3 < n);
    }
}

// One wave: FAST statistics of seg[0:n) (n >= 1) held in LDS -- lean_body's algorithm with the
// samples re-read from LDS at every pass instead of held in registers (the registers hold the
// record stream).  hist: this wave's RR_NB words of LDS.  Returns MAX (a key).
__device__ __forceinline__ unsigned lds_wave_stats(const uint32_t* seg, int n, int64_t g, uint32_t* hist,
                                            const nvrx_stats_soa& out) {
    constexpr int LOGNB = 8;
    constexpr int BPL = RR_NB / 64;
    const int lane = lane_id();
    unsigned lmn = 0xFFFFFFFFu, lmx = 0u;
    lds_walk(seg, n, [&](unsigned x, bool ok) {
        if (ok) {
            lmn = min(lmn, x);
            lmx = max(lmx, x);
        }
    });
    const unsigned mn = wave_min_b(lmn);
    const unsigned mx = wave_max_b(lmx);
    const unsigned range = mx - mn;
    RR_MARK(100, n);
    // exact sum of d = x - MIN; squares about a pivot c (a sample) in f64; c = 0 once the
    // range reaches 2^31 (d - c must be a signed 32-bit value)
    unsigned c = seg[0] - mn;
    if (range >= 0x80000000u) c = 0u;
    const int bits = 32 - __clz((int)range);
    int shift = bits > LOGNB ? bits - LOGNB : 0;
#pragma unroll
    for (int j = 0; j < BPL; ++j) hist[lane * BPL + j] = 0u;
    __builtin_amdgcn_wave_barrier();
    unsigned slo = 0, shi = 0;
    double acc = 0.0;
    const bool wide = range >= 0x80000000u;
    lds_walk(seg, n, [&](unsigned x, bool ok) {
        if (ok) {
            const unsigned d = x - mn;
            unsigned cy;
            slo = __builtin_addc(slo, d, 0u, &cy);
            shi += cy;
            const double e = wide ? (double)d : (double)(int)(d - c);
            acc = __builtin_fma(e, e, acc);
            atomicAdd(&hist[d >> shift], 1u);
        }
    });
    __builtin_amdgcn_wave_barrier();
    const double sd = wave_sum_f64_b((double)(((uint64_t)shi << 32) | slo));
    const double sq = wave_sum_f64_b(acc);
    RR_MARK(101, shift);

    const unsigned t0 = (unsigned)((n & 1) ? n / 2 : n / 2 - 1);
    const unsigned t1 = (unsigned)(n / 2);
    unsigned wlo = 0, below = 0, d0 = 0, d1 = 0;
    for (int level = 0; level < 8; ++level) {  // <= 4 levels of 8 bits (bound: every wave exits)
        RR_MARK(110 + level, wlo);
        if (level > 0) {
#pragma unroll
            for (int j = 0; j < BPL; ++j) hist[lane * BPL + j] = 0u;
            __builtin_amdgcn_wave_barrier();
            const unsigned span = (unsigned)RR_NB << shift;
            lds_walk(seg, n, [&](unsigned x, bool ok) {
                const unsigned q = x - mn - wlo;
                if (ok && q < span) atomicAdd(&hist[q >> shift], 1u);
            });
            __builtin_amdgcn_wave_barrier();
        }
        unsigned b0, c0, n0, b1;
        hist_locate1<16>(hist, t0 - below, b0, c0, n0);
        if (t1 - below < c0 + n0) {
            b1 = b0;
        } else {
            unsigned c1, n1;
            hist_locate1<16>(hist, t1 - below, b1, c1, n1);
        }
        if (b0 != b1) {  // ranks t0, t1 in different buckets: the nearest samples across
            const unsigned hi0 = wlo + ((b0 + 1) << shift);
            const unsigned lo1 = wlo + (b1 << shift);
            unsigned a = 0u, z = 0xFFFFFFFFu;
            lds_walk(seg, n, [&](unsigned x, bool ok) {
                if (ok) {
                    const unsigned d = x - mn;
                    a = max(a, d - hi0);
                    z = min(z, d - lo1);
                }
            });
            d0 = wave_max_b(a) + hi0;
            d1 = wave_min_b(z) + lo1;
            break;
        }
        if (shift == 0) {
            d0 = d1 = wlo + b0;
            break;
        }
        if (n0 <= 64u) {  // <= 64 candidates: compact into LDS, rank by compares
            __builtin_amdgcn_wave_barrier();
            const unsigned lo0 = wlo + (b0 << shift);
            const unsigned width = 1u << shift;
            unsigned base = 0;
            lds_walk(seg, n, [&](unsigned x, bool ok) {
                const unsigned d = x - mn;
                const bool in = ok && d - lo0 < width;
                const uint64_t bm = __ballot(in);
                if (in) hist[base + mbcnt(bm)] = d;
                base += (unsigned)__popcll(bm);
            });
            __builtin_amdgcn_wave_barrier();
            const unsigned ci = (lane < (int)n0) ? hist[lane] : 0xFFFFFFFFu;
            unsigned rank = 0;
            if (shift <= 26) {  // unique keys (candidate - lo0, lane) in one word
                const unsigned key = (lane < (int)n0) ? ((ci - lo0) << 6) | (unsigned)lane : 0xFFFFFFFFu;
                for (int j = 0; j < (int)n0; ++j) rank += (rl(key, j) < key) ? 1u : 0u;
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
    emit_stats(out, g, n, mn, mx, d0, d1, sd, sq, c, ColRef{});
    return mx;
}

// Keys of >= 3.76 s in a wave-path bucket (rare): lane 0 overwrites AVG / STD with the mean and
// population std of the decoded f32(ns) values in f64, each rounded once (the integer sums of
// lds_wave_stats do not apply to f32-valued keys).  A separate call after lds_wave_stats
// returns: placed inside it, after its median search, the branch hung the wave (gfx950 build of
// ROCm 7.2: control flow merged into the search loop's exits).
__device__ __noinline__ void lds_wide_moments(const uint32_t* seg, int n, int64_t g, const nvrx_stats_soa& out) {
    const int lane = lane_id();
    double a = 0.0;
    for (int i = lane; i < n; i += 64) a += (double)key_to_f32(seg[i]);
    const double mean = wave_sum_f64(a) / (double)n;
    double q = 0.0;
    for (int i = lane; i < n; i += 64) {
        const double e = (double)key_to_f32(seg[i]) - mean;
        q = __builtin_fma(e, e, q);
    }
    const double var = wave_sum_f64(q) / (double)n;
    if (lane == 0) {
        out.avg[g] = (float)(mean / 1000.0);
        out.std[g] = (float)(__builtin_sqrt(var) / 1000.0);
    }
}

template <int N, int NMIN>
__device__ __forceinline__ void lane_bucket(const uint32_t* b, int keep, int64_t g, const nvrx_stats_soa& out) {
    unsigned v[N];
#pragma unroll
    for (int j = 0; j < N; j += 4) {
        u32x4 q = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        if (j == 0 || j < keep) q = *(const u32x4*)(b + j);  // inside the padded bucket
        v[j] = q.x;
        v[j + 1] = q.y;
        v[j + 2] = q.z;
        v[j + 3] = q.w;
    }
    lane_stats<N, NMIN>(v, keep, g, out, ColRef{});
}

__global__ __launch_bounds__(RR_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
void records_resident_kernel(const nvrx_record* __restrict__ recs, const int64_t* __restrict__ rec_off,
                             int64_t nslots, int64_t cap, int64_t stg, int32_t* seg_len,
                             int32_t* counts, nvrx_stats_soa out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* cnt = lds;                   // [nslots] pushes per slot
    uint32_t* st = lds + nslots;           // [nslots] bucket start (stream layout) | RR_OVF
    uint32_t* cur = lds + 2 * nslots;      // [nslots] placement cursor / walk occurrence
    uint32_t* wlist = lds + 3 * nslots;    // [nslots] the group's wave-path slots
    uint32_t* hists = lds + ((4 * nslots + 3) & ~(int64_t)3);  // [RR_WAVES][RR_NB]
    uint32_t* stage = hists + RR_WAVES * RR_NB;                 // [stg] the group's buckets
    __shared__ uint32_t wtot[2][RR_WAVES];
    __shared__ uint32_t sh_next, sh_wl, sh_q, sh_total, sh_ta, sh_ovf;

    const int64_t t = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int wave = tid >> 6;
    uint32_t* hist = hists + wave * RR_NB;
    const int64_t r0 = rec_off[t], r1 = rec_off[t + 1];
    const int64_t n = r1 - r0;
    const nvrx_record* rs = recs + r0;
    const bool resident = n <= RR_CAPACITY;
    const uint32_t ns32 = (uint32_t)nslots;

    // ---- load: pair p = u * RR_THREADS + tid covers records 2p - o, 2p + 1 - o, read from the
    // 16-byte aligned address at or below the stream start; the buffer descriptor bounds the
    // reads (lanes past the end get zeros), indices outside [0, n) are marked invalid
    u32x4 w[RR_PPL];
    const int o = (int)(((uintptr_t)rs >> 3) & 1);
    if (resident) {
        const uintptr_t qa = (uintptr_t)(rs - o);
        const int64_t np = (n + o + 1) >> 1;
        const unsigned lo32 = __builtin_amdgcn_readfirstlane((unsigned)qa);
        const unsigned hi32 = __builtin_amdgcn_readfirstlane((unsigned)(qa >> 32));
        void* const pb = (void*)(((uint64_t)hi32 << 32) | lo32);
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(pb, 0, __builtin_amdgcn_readfirstlane((int)(np * 16)), 0x00020000);
#pragma unroll
        for (int u = 0; u < RR_PPL; ++u)
            w[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (u * RR_THREADS + tid) * 16, 0, NVRX_LOAD_AUX);
    }
    for (int64_t s = tid; s < nslots; s += RR_THREADS) cnt[s] = 0u;
    if (tid == 0) sh_ovf = 0u;
    RR_TRACE("rr: block 0 n=%ld resident=%d o=%d\n", (long)n, (int)resident, o);
    RR_MARK(1, (uint32_t)n);
    __syncthreads();

    // ---- count: branch-free -- an invalid record adds to this lane's own word of the wave's
    // histogram area (idle until the statistics, which clear it first)
    uint32_t* const dummy = hist + lane;
    if (resident) {
#pragma unroll
        for (int u = 0; u < RR_PPL; ++u) {
            const int64_t i0 = 2 * (int64_t)(u * RR_THREADS + tid) - o;
            if (!(i0 >= 0 && i0 < n && w[u].x < ns32)) w[u].x = 0xFFFFFFFFu;
            if (!(i0 + 1 < n && w[u].z < ns32)) w[u].z = 0xFFFFFFFFu;
            if (NVRX_AB_RR & 8) continue;
            atomicAdd(w[u].x != 0xFFFFFFFFu ? cnt + w[u].x : dummy, 1u);
            atomicAdd(w[u].z != 0xFFFFFFFFu ? cnt + w[u].z : dummy, 1u);
        }
    } else {
        for (int64_t i = tid; i < n; i += RR_THREADS) {
            const uint32_t s = rs[i].slot;
            if (s < ns32) atomicAdd(&cnt[s], 1u);
        }
    }
    __syncthreads();

    // ---- scan over slots: padded keeps laid out in two tiers -- tier A (keep > RR_LANE_FINAL)
    // first, tier B (the buckets a lane reduces) after it, slot order inside a tier, each bucket
    // padded to 4 records.  Tier B starts an LDS group of its own, so when it fits one stage it
    // is the LAST group, reduced after the last placement has freed the stream's registers
    // (lane classes up to 64 records there).  Each wave scans its own chunk of slots: chunk
    // totals first, then each wave from the preceding totals.
    const auto keep_of = [&](uint32_t c) { return (cap > 0 && c > (uint32_t)cap) ? (uint32_t)cap : c; };
    const auto tier_b = [](uint32_t keep) { return keep <= (uint32_t)RR_LANE_FINAL; };
    const int64_t chunk = ((nslots + RR_WAVES - 1) / RR_WAVES + 63) & ~(int64_t)63;
    const int64_t c_lo = min(nslots, chunk * wave), c_hi = min(nslots, c_lo + chunk);
    {
        uint32_t pa = 0, pb = 0;
        for (int64_t s = c_lo + lane; s < c_hi; s += 64) {
            const uint32_t k = keep_of(cnt[s]);
            const uint32_t p = (k + 3u) & ~3u;
            pa += tier_b(k) ? 0u : p;
            pb += tier_b(k) ? p : 0u;
        }
        pa = wave_sum_u32(pa);
        pb = wave_sum_u32(pb);
        if (lane == 0) {
            wtot[0][wave] = pa;
            wtot[1][wave] = pb;
        }
    }
    __syncthreads();
    {
        uint32_t ca = 0, cb = 0, ta = 0, tb = 0;
        for (int v = 0; v < RR_WAVES; ++v) {
            ca += v < wave ? wtot[0][v] : 0u;
            cb += v < wave ? wtot[1][v] : 0u;
            ta += wtot[0][v];
            tb += wtot[1][v];
        }
        cb += ta;  // tier B follows tier A
        bool ovf = false;
        for (int64_t c0 = c_lo; c0 < c_hi; c0 += 64) {
            const int64_t s = c0 + lane;
            const bool valid = s < c_hi;
            uint32_t c = 0, keep = 0;
            if (valid) {
                c = cnt[s];
                keep = keep_of(c);
            }
            const bool b = tier_b(keep);
            const uint32_t padded = (keep + 3u) & ~3u;
            const uint32_t ia = wave_incl_scan_u32(valid && !b ? padded : 0u);
            const uint32_t ib = wave_incl_scan_u32(valid && b ? padded : 0u);
            if (valid) {
                const uint32_t start = b ? cb + ib - padded : ca + ia - padded;
                const bool o2 = keep != c;
                ovf |= o2;
                st[s] = start | (o2 ? RR_OVF : 0u);
                cur[s] = start | (o2 ? RR_OVF : 0u);  // overflowed: the flag skips the fast placement
                const int64_t g = t * nslots + s;
                counts[g] = (int32_t)c;
                seg_len[g] = (int32_t)keep;
            }
            ca += rl(ia, 63);
            cb += rl(ib, 63);
        }
        if (__ballot(ovf) != 0 && lane == 0) atomicOr(&sh_ovf, 1u);
        if (tid == 0) {
            sh_total = ta + tb;
            sh_ta = ta;
        }
    }
    __syncthreads();
    RR_TRACE("rr: scanned total=%u tierA=%u ovf=%u\n", sh_total, sh_ta, sh_ovf);
    RR_MARK(2, sh_total);
    const auto start_of = [&](int64_t s) { return st[s] & ~RR_OVF; };

    // ---- register keys: (bucket start << RR_SLOT_BITS) | slot, so that a group (a window of
    // bucket starts) is one subtract and compare per record (host: nslots < 2^RR_SLOT_BITS,
    // starts < 2^(32 - RR_SLOT_BITS) for a resident stream)
    if (resident) {
#pragma unroll
        for (int u = 0; u < RR_PPL; ++u) {
            if (w[u].x != 0xFFFFFFFFu) w[u].x = (start_of(w[u].x) << RR_SLOT_BITS) | w[u].x;
            if (w[u].z != 0xFFFFFFFFu) w[u].z = (start_of(w[u].z) << RR_SLOT_BITS) | w[u].z;
        }
    }

    const uint32_t total = sh_total, ta = sh_ta;
    constexpr uint32_t SLOT_MASK = (1u << RR_SLOT_BITS) - 1u;
    // one LDS group: the buckets starting in [P, P + W); last: the final one, whose buckets of
    // RR_LANE_MAX+1 .. RR_LANE_FINAL records are left to the lane pass after the group loop
    // (the stream's registers are dead there; inside the loop they would have to stay live)
    const auto group = [&](bool last, uint32_t P, uint32_t W) {
        const auto place = [&](uint32_t s, uint32_t x) {
            if (start_of(s) - P < W) {
                const uint32_t pos = atomicAdd(&cur[s], 1u);
                if (!(pos & RR_OVF)) stage[pos - P] = x;
            }
        };
        if (NVRX_AB_RR & 4) {
        } else if (resident) {
            // branch-free batches: the cursor atomics of RR_PB pairs are issued back to back (a
            // record outside the group increments this lane's dummy word), then their stores
            // (outside the group / overflowed: this lane's second dummy word)
            constexpr int RR_PB = 4;
            // an opaque copy of the slot mask, made inside the group loop: with a constant mask
            // the compiler proves (key - (P << 13)) & mask == key & mask and hoists the 94 masked
            // keys out of the loop, which spilled the stream's registers
            uint32_t slot_mask = SLOT_MASK;
            asm volatile("" : "+s"(slot_mask));
#pragma unroll
            for (int u0 = 0; u0 < RR_PPL; u0 += RR_PB) {
                uint32_t pos[2 * RR_PB];
                bool in[2 * RR_PB];
#pragma unroll
                for (int k = 0; k < 2 * RR_PB && u0 + k / 2 < RR_PPL; ++k) {
                    const uint32_t key = (k & 1) ? w[u0 + k / 2].z : w[u0 + k / 2].x;
                    // start - P < W  <=>  key - (P << 13) < W << 13 (the slot bits lie below)
                    const uint32_t dk = key - (P << RR_SLOT_BITS);
                    in[k] = dk < (W << RR_SLOT_BITS);  // invalid keys (all ones) never fall inside
                    pos[k] = atomicAdd(in[k] ? cur + (dk & slot_mask) : dummy, 1u);
                }
#pragma unroll
                for (int k = 0; k < 2 * RR_PB && u0 + k / 2 < RR_PPL; ++k) {
                    const uint32_t x = (k & 1) ? w[u0 + k / 2].w : w[u0 + k / 2].y;
                    const bool ok = in[k] && !(pos[k] & RR_OVF);
                    *(ok ? stage + (pos[k] - P) : dummy + 64) = x;
                }
            }
        } else {
            for (int64_t i = tid; i < n; i += RR_THREADS) {
                const nvrx_record r = rs[i];
                if (r.slot < ns32) place(r.slot, r.ns);
            }
        }
        if (sh_ovf) {
            // overflowed slots of the group: wave 0 walks the stream in push order and keeps
            // occurrences >= count - keep (the ring's last `cap`), as records_bucket_kernel
            __syncthreads();
            if (wave == 0) {
                for (int64_t s = lane; s < nslots; s += 64)
                    if ((st[s] & RR_OVF) && start_of(s) - P < W) cur[s] = 0u;
                __builtin_amdgcn_wave_barrier();
                for (int64_t b = 0; b < n; b += 64) {
                    const int64_t i = b + lane;
                    nvrx_record rec = {0xFFFFFFFFu, 0u};
                    if (i < n) rec = rs[i];
                    bool ok = rec.slot < ns32;
                    if (ok) ok = (st[rec.slot] & RR_OVF) && start_of(rec.slot) - P < W;
                    uint64_t pending = __ballot(ok);
                    uint32_t occ = 0;
                    while (pending) {
                        const int leader = __builtin_ffsll(pending) - 1;
                        const uint32_t ls = __builtin_amdgcn_readlane(rec.slot, leader);
                        const uint64_t grp = __ballot(ok && rec.slot == ls) & pending;
                        const uint32_t c0 = cur[ls];
                        if (ok && rec.slot == ls) occ = c0 + mbcnt(grp);
                        __builtin_amdgcn_wave_barrier();
                        if (lane == leader) cur[ls] = c0 + (uint32_t)__popcll(grp);
                        __builtin_amdgcn_wave_barrier();
                        pending &= ~grp;
                    }
                    if (ok) {
                        const uint32_t c = cnt[rec.slot];
                        const uint32_t drop = c - keep_of(c);
                        if (occ >= drop) stage[start_of(rec.slot) - P + (occ - drop)] = rec.ns;
                    }
                }
            }
        }
        __syncthreads();

        // ---- statistics of the group's buckets: short ones one lane each, the rest queued
        const uint32_t lane_max = last ? (uint32_t)RR_LANE_FINAL : (uint32_t)RR_LANE_MAX;
        for (int64_t s = tid; s < nslots; s += RR_THREADS) {
            const uint32_t b = start_of(s);
            const bool mine = b - P < W;
            const uint32_t keep = mine ? keep_of(cnt[s]) : 0u;
            const int64_t g = t * nslots + s;
            const uint32_t* bk = stage + (b - P);
            const bool wave_path = mine && keep > lane_max && !(NVRX_AB_RR & 1);
            if ((NVRX_AB_RR & 2) || !mine) {
            } else if (keep == 0) {
                write_empty(out, g);
            } else if (keep <= 8) {
                lane_bucket<8, 1>(bk, (int)keep, g, out);
            } else if (keep <= 16) {
                lane_bucket<16, 9>(bk, (int)keep, g, out);
            }
        const uint64_t bm = __ballot(wave_path);
            uint32_t base = 0;
            if (lane == __builtin_ffsll(bm) - 1) base = atomicAdd(&sh_wl, (uint32_t)__popcll(bm));
            base = __builtin_amdgcn_readlane(base, __builtin_ffsll(bm | (1ull << 63)) - 1);
            if (wave_path) wlist[base + mbcnt(bm)] = (uint32_t)s;
        }
        __syncthreads();
        const uint32_t nwl = sh_wl;
        RR_MARK(3, nwl);
        RR_TRACE("rr: group [%u, +%u) last=%d: %u wave-path buckets\n", P, W, (int)last, nwl);
        for (;;) {
            uint32_t j = 0;
            if (lane == 0) j = atomicAdd(&sh_q, 1u);
            j = __builtin_amdgcn_readfirstlane(j);
            if (j >= nwl) break;
            const int64_t s = wlist[j];
            const uint32_t* seg = stage + (start_of(s) - P);
            const int kn = (int)keep_of(cnt[s]);
            if (lds_wave_stats(seg, kn, t * nslots + s, hist, out) >= NVRX_KEY_WIDE)
                lds_wide_moments(seg, kn, t * nslots + s, out);
        }
        RR_MARK(4, 0);
        __syncthreads();
    };

    uint32_t P = 0, W = 0;
    for (;;) {
        // the next group boundary: the start of the first bucket (layout order) that does not fit
        // a stage opened at P, and the start of tier B (it opens a group of its own)
        if (tid == 0) {
            sh_next = P < ta ? ta : 0xFFFFFFFFu;
            sh_wl = 0u;
            sh_q = 0u;
        }
        __syncthreads();
        for (int64_t s = tid; s < nslots; s += RR_THREADS) {
            const uint32_t k = keep_of(cnt[s]);
            const uint32_t b = start_of(s);
            if (k > 0 && b >= P && b + ((k + 3u) & ~3u) - P > (uint32_t)stg) atomicMin(&sh_next, b);
        }
        __syncthreads();
        const uint32_t Pn = sh_next;
        const bool last = Pn >= total;
        W = last ? total - P + 1 : Pn - P;  // + 1: empty buckets start at `total` too
        group(last, P, W);
        if (last) break;
        P = Pn;
    }
    // ---- the last group's buckets of RR_LANE_MAX+1 .. RR_LANE_FINAL records, one lane each,
    // still in the stage (tier B: all of them when it fits one stage)
    if (!(NVRX_AB_RR & 2)) {
        for (int64_t s = tid; s < nslots; s += RR_THREADS) {
            const uint32_t b = start_of(s);
            const uint32_t keep = b - P < W ? keep_of(cnt[s]) : 0u;
            if (keep <= (uint32_t)RR_LANE_MAX || keep > (uint32_t)RR_LANE_FINAL) continue;
            const uint32_t* bk = stage + (b - P);
            if (keep <= 32) lane_bucket<32, 17>(bk, (int)keep, t * nslots + s, out);
            else lane_bucket<64, 33>(bk, (int)keep, t * nslots + s, out);
        }
    }
}

hipError_t records_resident_stats(const nvrx_record* recs, const int64_t* rec_off, int64_t nstreams,
                                  int64_t nslots, int64_t cap, int32_t* seg_len, int32_t* counts,
                                  const nvrx_stats_soa& out, hipStream_t st) {
    if (nstreams <= 0 || nslots <= 0) return hipSuccess;
    const int64_t stg = records_resident_stage(nslots);
    if (cap <= 0 || ((cap + 3) & ~(int64_t)3) > stg || nslots >= ((int64_t)1 << RR_SLOT_BITS))
        return hipErrorInvalidValue;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)records_resident_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)RR_LDS);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL(records_resident_kernel, dim3((unsigned)nstreams), dim3(RR_THREADS), RR_LDS, st,
                       recs, rec_off, nslots, cap, stg, seg_len, counts, out);
    return hipGetLastError();
}

}  // namespace nvrx
