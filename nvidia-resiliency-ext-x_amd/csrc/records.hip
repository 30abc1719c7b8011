// records.hip -- kernel-duration record streams -> per-kernel retained segments (gfx950).
//
// Replaces the per-record hot loop of CuptiProfiler::bufferCompleted
// (straggler/cupti_src/CuptiProfiler.cpp:168-203: key lookup, then a push into that
// key's CircularBuffer) and the ring itself (CircularBuffer.h:53-69: keeps the LAST
// `capacity` pushes).  Records stay resident in HBM in push order; at report time each
// stream (one per rank) is bucketed by slot and only the last `cap` records of every
// slot are kept.  computeStats sorts, so order inside a bucket does not change any
// statistic; buckets are still written in push order whenever a slot overflowed.
//
// One workgroup of RB_WAVES waves owns one stream; per-slot counters live in LDS:
//   pass 1: LDS histogram of slots, 16-byte loads = two records per lane: the head of the
//           stream (up to RB_WAVES * RB_REGS * 64 pairs) swept by all waves together (wave w
//           takes every RB_WAVES-th 1 KB step) and held in VGPRs, then each wave's contiguous
//           chunk of the rest (its head kept in the LDS stash);
//   scan  : keep_s = min(count_s, cap), bucket starts padded to 16 B (aligned loads
//           in segment_stats), written to seg_off / seg_len / counts;
//   pass 2: scatter.  Records of slots that did not overflow take LDS atomic cursors
//           (order inside such a bucket is free: computeStats sorts); records of
//           overflowed slots are placed by wave 0 alone, in push order: 64 records per
//           step, same-slot lanes grouped with ballot (leader = lowest lane), occurrence
//           index = cursor + mbcnt(group), kept iff occurrence >= count - keep.
#include <stdlib.h>

#include <algorithm>

#include "segment_kernels.h"

namespace nvrx {

// Per-stream slack for the 16-B padding of every bucket (<= 3 per slot), itself a
// multiple of 4 elements so that every stream base stays 16-byte aligned.
__host__ __device__ __forceinline__ int64_t stream_slack(int64_t nslots) {
    return (3 * nslots + 4 + 3) & ~(int64_t)3;
}
__device__ __forceinline__ int64_t stream_base(const int64_t* rec_off, int64_t t, int64_t nslots) {
    return ((rec_off[t] + 3) & ~(int64_t)3) + t * stream_slack(nslots);
}

// Timing-only ablation builds (tools/build_variant.sh -DNVRX_RB_ABLATE=k; outputs are wrong):
// 1 = stop after pass 1 + the scans, 2 = also skip the staged copy-out and the tiny statistics
// after pass 2, 3 = skip only the tiny statistics, 4 = pass 1's loads without the LDS slot counts,
// then stop, 5 = pass 1 alone (no scans), 6 = pass 1 + the scan's chunk totals, 7 = pass 1 + the
// scans without their global stores.  0 (the library): the whole kernel.
#ifndef NVRX_RB_ABLATE
#define NVRX_RB_ABLATE 0
#endif
// Timing-only probes of an in-place reduction of the hot slots (outputs are
// wrong): NVRX_RB_HOTPASS = k adds k passes over the register head and the LDS stash after the
// scan, each record of local slot < 32 adding one non-returning LDS atomic into a 32 x 256-bin
// histogram (a radix-select level); NVRX_RB_HOTP1 = 1 adds ds_min / ds_max per hot record to
// pass 1 (the slot's MIN / MAX).  Both use the cold-bucket stage as scratch.
#ifndef NVRX_RB_TINY_COPY  // build-time switch: 1 = also write the reduced tiny buckets (and offsets) out
#define NVRX_RB_TINY_COPY 0
#endif
#ifndef NVRX_RB_HOTPASS
#define NVRX_RB_HOTPASS 0
#endif
#ifndef NVRX_RB_HOTP1
#define NVRX_RB_HOTP1 0
#endif

constexpr uint32_t RB_OVF = 0x80000000u;  // start[s] flag: slot s overflowed its ring
// Slots one bucketing pass counts in LDS; a larger slot table is bucketed in passes over
// consecutive slot ranges (each pass re-reads the streams and ignores other slots' records),
// each pass into its own region of out_ns.
constexpr int64_t RB_PASS_SLOTS = NVRX_RECORDS_MAX_LDS / (3 * sizeof(uint32_t));
constexpr int RB_TINY = 8;  // records_stats: buckets this short are reduced by the bucketing kernel

// records [lo, hi) of a stream in 16-byte pairs where the base allows it; f(rec) per record.
// RB_UNROLL independent loads per lane are issued before any is consumed: a wave keeps
// RB_UNROLL KB in flight instead of one (the loop is otherwise latency-bound).
#ifndef NVRX_RB_UNROLL  // build-time tuning constant
#define NVRX_RB_UNROLL 8
#endif
constexpr int RB_UNROLL = NVRX_RB_UNROLL;
template <class F>
__device__ __forceinline__ void for_records(const nvrx_record* rs, int64_t lo, int64_t hi, int lane,
                                            bool pairs, F&& f) {
    if (pairs) {  // lo, hi even; rs 16-B aligned
        const u32x4* q = (const u32x4*)(rs + lo);
        const int64_t np = (hi - lo) >> 1;
        int64_t i = lane;
        for (; i + 64 * (RB_UNROLL - 1) < np; i += 64 * RB_UNROLL) {
            u32x4 w[RB_UNROLL];
#pragma unroll
            for (int u = 0; u < RB_UNROLL; ++u) w[u] = __builtin_nontemporal_load(q + i + 64 * u);
#pragma unroll
            for (int u = 0; u < RB_UNROLL; ++u) {
                f(nvrx_record{w[u].x, w[u].y});
                f(nvrx_record{w[u].z, w[u].w});
            }
        }
        for (; i < np; i += 64) {
            const u32x4 w = q[i];
            f(nvrx_record{w.x, w.y});
            f(nvrx_record{w.z, w.w});
        }
    } else {
        int64_t i = lo + lane;
        for (; i + 64 * (RB_UNROLL - 1) < hi; i += 64 * RB_UNROLL) {
            nvrx_record w[RB_UNROLL];
#pragma unroll
            for (int u = 0; u < RB_UNROLL; ++u) w[u] = rs[i + 64 * u];
#pragma unroll
            for (int u = 0; u < RB_UNROLL; ++u) f(w[u]);
        }
        for (; i < hi; i += 64) f(rs[i]);
    }
}

// record pairs [p_lo, p_hi) of a 16-B aligned pair array, f(pair, index) per pair, with the
// same RB_UNROLL loads in flight per lane as for_records.
template <class F>
__device__ __forceinline__ void for_pairs(const u32x4* q, int64_t p_lo, int64_t p_hi, int lane, F&& f) {
    int64_t i = p_lo + lane;
    for (; i + 64 * (RB_UNROLL - 1) < p_hi; i += 64 * RB_UNROLL) {
        u32x4 w[RB_UNROLL];
#pragma unroll
        for (int u = 0; u < RB_UNROLL; ++u) w[u] = __builtin_nontemporal_load(q + i + 64 * u);
#pragma unroll
        for (int u = 0; u < RB_UNROLL; ++u) f(w[u], i + 64 * u);
    }
    for (; i < p_hi; i += 64) f(q[i], i);
}

// RB_REGS > 0: the next RB_REGS pairs per lane after the LDS stash are also kept, in VGPRs
// (16 B each; with one block per CU the block may take a SIMD register file's worth per
// SIMD), so pass 2 re-reads only what neither holds -- nothing on configs[3] -- and pass 1
// has RB_REGS loads per lane in flight at once.
template <int RB_WAVES, int RB_REGS>
__global__ __launch_bounds__(64 * RB_WAVES) __attribute__((amdgpu_waves_per_eu(1, RB_REGS > 32 ? 1 : RB_REGS > 16 ? 2 : RB_REGS > 0 ? 4 : 8)))
void records_bucket_kernel(
    const nvrx_record* __restrict__ recs, const int64_t* __restrict__ rec_off, int64_t nslots,
    int64_t cap, int force_stable, int64_t* seg_off, int32_t* seg_len, uint32_t* out_ns,
    int32_t* counts, int64_t stash_pairs, int64_t stage_cap, uint32_t cold_max,
    nvrx_stats_soa tiny, uint32_t slot_lo, int64_t seg_stride, int pass, int64_t t0,
    int64_t nstreams_total) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* cnt = lds;                // [nslots] pushes per slot
    uint32_t* cur = lds + nslots;       // [nslots] scatter cursor / occurrence counter
    uint32_t* start = lds + 2 * nslots; // [nslots] bucket start (relative to stream base) | RB_OVF
    // [stage_cap] the first bucket positions of the stream, assembled in LDS and written out
    // with 16-byte stores (stage_cap: a multiple of 4, 0 = off)
    uint32_t* stage = lds + ((3 * nslots + 3) & ~(int64_t)3);
    // [RB_WAVES][stash_pairs] record pairs: the head of every wave's chunk, kept from pass 1
    // for pass 2 (which would otherwise re-read them from the memory side)
    u32x4* stash = (u32x4*)(stage + stage_cap);
    __shared__ uint32_t any_ovf;
    __shared__ uint32_t wtot[3][RB_WAVES];
    const int64_t t = t0 + blockIdx.x;  // this launch's streams: [t0, t0 + gridDim.x)
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const int64_t r0 = rec_off[t], r1 = rec_off[t + 1];
    const nvrx_record* rs = recs + r0;
    const int64_t n = r1 - r0;
    const int64_t base = stream_base(rec_off, t, nslots);
    // a slot table larger than one pass's LDS counters: pass p's buckets follow the regions of
    // passes 0..p-1, each as large as records_bucket_capacity's per-pass term
    const int64_t ns_off = pass == 0 ? 0 :
        (int64_t)pass * (((rec_off[nstreams_total] + 3) & ~(int64_t)3) + nstreams_total * stream_slack(RB_PASS_SLOTS));
    const bool pairs = (((uintptr_t)rs) & 15) == 0;
    // The head of the stream -- up to RB_REGS x 64 x RB_WAVES record pairs -- is held in
    // registers between the passes, the waves sweeping it together (pair (u RB_WAVES + w) 64 +
    // lane in register u of wave w: 1.36 against 1.45 ms for per-wave chunks in the pass-1
    // skeleton on configs[3], tools/mb_rb_read.hip); the rest of the stream is split into
    // per-wave chunks whose heads go to the LDS stash.
    const int64_t rp = pairs ? min(n >> 1, (int64_t)RB_REGS * 64 * RB_WAVES) : 0;  // register pairs
    const u32x4* q = (const u32x4*)rs;
    // wave w's chunk of the rest: [lo, hi), even boundaries
    const int64_t n_rest = n - 2 * rp;
    const int64_t per = ((n_rest + RB_WAVES - 1) / RB_WAVES + 1) & ~(int64_t)1;
    const int64_t lo = 2 * rp + min(n_rest, per * wave), hi = min(n, lo + per);
    const bool wpairs = pairs && ((hi - lo) % 2 == 0);
    // pairs of this wave's chunk held in LDS between the passes (0 when not pair-aligned)
    const int64_t snp = wpairs ? min((hi - lo) >> 1, stash_pairs) : 0;
    u32x4* wstash = stash + wave * stash_pairs;
    const u32x4* wq = (const u32x4*)(rs + lo);
    // pairs [held, np) of the chunk are read again in pass 2
    const int64_t np = wpairs ? (hi - lo) >> 1 : 0;
    const int64_t held = snp;
    u32x4 reg[RB_REGS > 0 ? RB_REGS : 1];

    for (int64_t s = threadIdx.x; s < nslots; s += blockDim.x) {
        cnt[s] = 0u;
        cur[s] = 0u;
    }
    if (threadIdx.x == 0) any_ovf = force_stable ? 1u : 0u;
    __syncthreads();
    uint32_t sink = 0;  // NVRX_RB_ABLATE == 4: the records consumed without the LDS counts
    const auto count = [&](const nvrx_record& r) {
        const uint32_t ls = r.slot - slot_lo;  // this pass's slots: [slot_lo, slot_lo + nslots)
        if (NVRX_RB_ABLATE == 4)
            sink += ls;
        else if (ls < (uint32_t)nslots)
            atomicAdd(&cnt[ls], 1u);
        if (NVRX_RB_HOTP1 && ls < 32u && stage_cap >= 8192) {
            atomicMin(&stage[2 * ls], r.ns);
            atomicMax(&stage[2 * ls + 1], r.ns);
        }
    };
    if (RB_REGS > 0) {  // issued first: their latency overlaps the LDS-stashed head
#pragma unroll
        for (int u = 0; u < RB_REGS; ++u) {
            const int64_t p = ((int64_t)u * RB_WAVES + wave) * 64 + lane;
            reg[u] = p < rp ? __builtin_nontemporal_load(q + p) : u32x4{~0u, 0u, ~0u, 0u};
        }
    }
    for_pairs(wq, 0, snp, lane, [&](const u32x4& w, int64_t p) {
        wstash[p] = w;
        count(nvrx_record{w.x, w.y});
        count(nvrx_record{w.z, w.w});
    });
    if (RB_REGS > 0) {
#pragma unroll
        for (int u = 0; u < RB_REGS; ++u) {
            count(nvrx_record{reg[u].x, reg[u].y});
            count(nvrx_record{reg[u].z, reg[u].w});
        }
    }
    for_records(rs, lo + 2 * (wpairs ? held : 0), hi, lane, wpairs, count);
    __syncthreads();
    if (NVRX_RB_ABLATE == 5) {  // pass 1 alone (no scans)
        if (threadIdx.x == 0 && cnt[0] == 0x12345u) counts[0] = 1;
        return;
    }

    // exclusive scan of padded keeps over slots, every wave on its own chunk of slots (the
    // block's other waves would otherwise wait at the barrier while one wave walks all the
    // slots: with one block per CU that wait was ~1 ms of configs[3]):
    //   (a) chunk totals -> LDS, (b) each wave scans its chunk from the preceding totals.
    // With staging the bucket array is laid out by tier, slot order inside a tier: the tiny
    // buckets (<= RB_TINY records), the other cold ones (<= cold_max, not overflowed), then
    // the rest -- one scan per tier, each carried past the tiers before it.  The first
    // stage_cap positions (tiny and cold buckets) are assembled in LDS and written out with
    // 16-byte stores; see records_bucket for what pays.
    const auto keep_of = [&](uint32_t total) {
        return (cap > 0 && total > (uint32_t)cap) ? (uint32_t)cap : total;
    };
    const bool staging = stage_cap > 0 && !force_stable;
    const auto tier_of = [&](uint32_t total) {
        const uint32_t keep = keep_of(total);
        if (!staging || keep != total || keep > cold_max) return 2;
        return keep <= (uint32_t)RB_TINY ? 0 : 1;
    };
    const int64_t chunk = ((nslots + RB_WAVES - 1) / RB_WAVES + 63) & ~(int64_t)63;
    const int64_t c_lo = min(nslots, chunk * wave), c_hi = min(nslots, c_lo + chunk);
    {
        uint32_t p0 = 0, p1 = 0, p2 = 0;
        for (int64_t s = c_lo + lane; s < c_hi; s += 64) {
            const uint32_t total = cnt[s];
            const uint32_t padded = (keep_of(total) + 3u) & ~3u;
            const int tr = tier_of(total);
            p0 += tr == 0 ? padded : 0u;
            p1 += tr == 1 ? padded : 0u;
            p2 += tr == 2 ? padded : 0u;
        }
        p0 = wave_sum_u32(p0);
        p1 = wave_sum_u32(p1);
        p2 = wave_sum_u32(p2);
        if (lane == 0) {
            wtot[0][wave] = p0;
            wtot[1][wave] = p1;
            wtot[2][wave] = p2;
        }
    }
    __syncthreads();
    if (NVRX_RB_ABLATE == 6) {  // pass 1 + the scan's chunk totals only
        if (threadIdx.x == 0 && wtot[0][0] == 0x12345u) counts[0] = 1;
        return;
    }
    uint32_t cold_total = 0, tiny_end = 0;
    {
        // the tier totals and this wave's carries from the waves' chunk totals: lane w reads
        // wave w's, one wave reduction each (a serial walk over the waves' totals, 16 dependent
        // LDS reads for the last wave and each tier, was ~1/3 of the scan phase)
        const uint32_t w0 = lane < RB_WAVES ? wtot[0][lane] : 0u;
        const uint32_t w1 = lane < RB_WAVES ? wtot[1][lane] : 0u;
        const uint32_t w2 = lane < RB_WAVES ? wtot[2][lane] : 0u;
        const uint32_t tiny_total = wave_sum_u32(w0);
        tiny_end = tiny_total;
        cold_total = tiny_total + wave_sum_u32(w1);
        const uint32_t lim = (uint32_t)min((int64_t)cold_total, stage_cap);
        bool overflow = false;
        {
            // one pass over the wave's slots: a slot belongs to exactly one tier, so each lane
            // takes its own tier's prefix out of three independent scans (their DPP chains
            // interleave), and the chunk is read once instead of once per tier (round 4: the
            // bucketing kernel 2.67 -> 2.62-2.63 ms on configs[3]; one tier per pass was chosen
            // earlier when three scans live at once spilled the kernel, which they no longer do)
            uint32_t carry0 = wave_sum_u32(lane < wave ? w0 : 0u);
            uint32_t carry1 = tiny_total + wave_sum_u32(lane < wave ? w1 : 0u);
            uint32_t carry2 = cold_total + wave_sum_u32(lane < wave ? w2 : 0u);
            for (int64_t c = c_lo; c < c_hi; c += 64) {
                const int64_t s = c + lane;
                uint32_t keep = 0, total = 0;
                int k = 3;  // none
                if (s < c_hi) {
                    total = cnt[s];
                    keep = keep_of(total);
                    k = tier_of(total);
                }
                const uint32_t padded = (keep + 3u) & ~3u;
                const uint32_t i0 = wave_incl_scan_u32(k == 0 ? padded : 0u);
                const uint32_t i1 = wave_incl_scan_u32(k == 1 ? padded : 0u);
                const uint32_t i2 = wave_incl_scan_u32(k == 2 ? padded : 0u);
                if (k < 3) {
                    const uint32_t st = (k == 0 ? carry0 + i0 : k == 1 ? carry1 + i1 : carry2 + i2) - padded;
                    const bool ovf = keep != total;
                    overflow |= ovf;
                    const uint32_t flag = ovf || force_stable ? RB_OVF : 0u;
                    start[s] = st | flag;
                    cur[s] = flag ? RB_OVF : st;  // pass 2's write cursor (absolute in the stream)
                    const int64_t g = t * seg_stride + slot_lo + s;
                    // a bucket this kernel reduces itself (after pass 2): a negative length
                    const bool reduced = tiny.num && k == 0 && keep >= 1 && st + padded <= lim;
                    if (NVRX_RB_ABLATE != 7) {  // 7: the scans without their global stores
                        // a reduced bucket's offset is never read (records_stats: not written)
                        if (!reduced || NVRX_RB_TINY_COPY) seg_off[g] = ns_off + base + st;
                        seg_len[g] = reduced ? -(int32_t)keep : (int32_t)keep;
                        if (counts) counts[g] = (int32_t)total;  // optional in records_stats
                    }
                }
                carry0 += __builtin_amdgcn_readlane(i0, 63);
                carry1 += __builtin_amdgcn_readlane(i1, 63);
                carry2 += __builtin_amdgcn_readlane(i2, 63);
            }
        }
        if (__ballot(overflow) != 0 && lane == 0) any_ovf = 1u;
    }
    __syncthreads();
    if (NVRX_RB_ABLATE == 1 || NVRX_RB_ABLATE == 7) return;
    if (NVRX_RB_ABLATE == 4) {
        if (sink == 0x12345u) counts[0] = (int32_t)sink;  // keeps the loads alive
        return;
    }
    // positions below stage_lim go to LDS (cold buckets only: an overflowed slot's walk
    // writes to memory directly)
    const uint32_t stage_lim = (uint32_t)min((int64_t)cold_total, stage_cap);
    uint32_t* out = out_ns + ns_off + base;

    // records of slots that kept everything: any order.  The cursor starts at the bucket's
    // start, so a record costs one returning LDS atomic (a lookup of start[] before the atomic
    // doubled the dependent LDS round trips: 4.5 -> 3.x ms on configs[3]); overflowed slots
    // hold RB_OVF, which the increments keep set, and are skipped here.
    const auto place = [&](const nvrx_record& r) {
        const uint32_t ls = r.slot - slot_lo;
        if (ls < (uint32_t)nslots) {
            const uint32_t pos = atomicAdd(&cur[ls], 1u);
            if (pos < stage_lim)
                stage[pos] = r.ns;
            else if (!(pos & RB_OVF))
                out[pos] = r.ns;
        }
    };
    // The stashed head of the chunk (LDS) is placed while each batch of the rest's loads is
    // in flight: `per_it` stashed pairs per lane between issuing a batch and consuming it.
    int64_t sp = lane;  // this lane's stash cursor
    const auto place_stash = [&](int m) {
        for (int j = 0; j < m && sp < snp; ++j, sp += 64) {
            const u32x4 w = wstash[sp];
            place(nvrx_record{w.x, w.y});
            place(nvrx_record{w.z, w.w});
        }
    };
    if (NVRX_RB_HOTPASS > 0 && stage_cap >= 8192) {
        for (int lvl = 0; lvl < NVRX_RB_HOTPASS; ++lvl) {
            const uint32_t sh = 24u - 8u * (uint32_t)lvl;
            const auto hp = [&](uint32_t slot, uint32_t ns) {
                const uint32_t ls = slot - slot_lo;
                if (ls < 32u) atomicAdd(&stage[ls * 256u + ((ns >> sh) & 255u)], 1u);
            };
#pragma unroll
            for (int u = 0; u < RB_REGS; ++u) {
                hp(reg[u].x, reg[u].y);
                hp(reg[u].z, reg[u].w);
            }
            for (int64_t k = lane; k < snp; k += 64) {
                const u32x4 w = wstash[k];
                hp(w.x, w.y);
                hp(w.z, w.w);
            }
            __syncthreads();
        }
    }
    if (RB_REGS > 0) {  // no memory dependency: their atomics and stores go out first
#pragma unroll
        for (int u = 0; u < RB_REGS; ++u) {
            place(nvrx_record{reg[u].x, reg[u].y});
            place(nvrx_record{reg[u].z, reg[u].w});
        }
    }
    {
        const int64_t iters = (np - held) / (64 * RB_UNROLL);
        const int per_it = iters > 0 ? (int)((snp / 64 + iters - 1) / iters) : 0;
        int64_t i = held + lane;
        for (; i + 64 * (RB_UNROLL - 1) < np; i += 64 * RB_UNROLL) {
            u32x4 w[RB_UNROLL];
#pragma unroll
            for (int u = 0; u < RB_UNROLL; ++u) w[u] = __builtin_nontemporal_load(wq + i + 64 * u);
            place_stash(per_it);
#pragma unroll
            for (int u = 0; u < RB_UNROLL; ++u) {
                place(nvrx_record{w[u].x, w[u].y});
                place(nvrx_record{w[u].z, w[u].w});
            }
        }
        for (; i < np; i += 64) {
            const u32x4 w = wq[i];
            place(nvrx_record{w.x, w.y});
            place(nvrx_record{w.z, w.w});
        }
        place_stash(1 << 30);
        // a chunk that is not pair-aligned (np = 0): its records one by one
        if (!wpairs) for_records(rs, lo, hi, lane, false, place);
    }
    if (NVRX_RB_ABLATE == 2) return;
    if (stage_lim > 0) {  // the assembled head of the bucket array, in 16-byte stores
        __syncthreads();
        const u32x4* sv = (const u32x4*)stage;
        u32x4* ov = (u32x4*)out;  // out = stream base: 16-byte aligned
        // records_stats with the whole tiny tier staged: every tiny bucket is reduced below from
        // LDS and flagged (negative seg_len), so its records are never read from out_ns -- the
        // copy-out starts past them (NVRX_RB_TINY_COPY=1 writes them anyway)
        const uint32_t skip = (tiny.num && !NVRX_RB_TINY_COPY && tiny_end <= stage_lim) ? tiny_end / 4 : 0u;
        for (uint32_t i = skip + threadIdx.x; i < stage_lim / 4; i += blockDim.x) ov[i] = sv[i];
        // records_stats: the statistics of the staged buckets of <= RB_TINY records, one lane
        // per bucket straight from LDS (lane_stats: computeStats bit for bit, as the ragged
        // lane<8> class does), instead of a later kernel re-reading them through a class list
        if (tiny.num && NVRX_RB_ABLATE != 3) {
            for (int64_t s = threadIdx.x; s < nslots; s += blockDim.x) {
                const uint32_t total = cnt[s];
                const uint32_t keep = keep_of(total);
                const uint32_t st = start[s];
                if (tier_of(total) == 0 && keep >= 1 && st + ((keep + 3u) & ~3u) <= stage_lim) {
                    const u32x4 a = sv[st / 4];
                    const u32x4 b = keep > 4 ? sv[st / 4 + 1] : u32x4{~0u, ~0u, ~0u, ~0u};
                    unsigned v[RB_TINY] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
                    lane_stats<RB_TINY>(v, (int)keep, t * seg_stride + slot_lo + s, tiny, ColRef{});
                }
            }
        }
    }
    if (!any_ovf) return;
    __syncthreads();  // every wave's pass-2 increments of the RB_OVF cursors are done
    if (wave != 0) return;
    // the ordered walk counts occurrences of the overflowed slots from zero
    for (int64_t s = lane; s < nslots; s += 64)
        if (start[s] & RB_OVF) cur[s] = 0u;
    __builtin_amdgcn_wave_barrier();
    // overflowed slots: wave 0 walks the whole stream in push order
    for (int64_t b = 0; b < n; b += 64) {
        const int64_t i = b + lane;
        nvrx_record rec = {0xFFFFFFFFu, 0u};
        if (i < n) rec = rs[i];
        rec.slot -= slot_lo;  // this pass's local slot
        const bool ok = rec.slot < (uint32_t)nslots && (start[rec.slot] & RB_OVF);
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
            const uint32_t total = cnt[rec.slot];
            const uint32_t keep = (cap > 0 && total > (uint32_t)cap) ? (uint32_t)cap : total;
            const uint32_t drop = total - keep;
            if (occ >= drop) out[(start[rec.slot] & ~RB_OVF) + (occ - drop)] = rec.ns;
        }
    }
}

int64_t records_bucket_capacity(int64_t n, int64_t nstreams, int64_t nslots) {
    int64_t c = 0;
    for (int64_t lo = 0; lo < nslots; lo += RB_PASS_SLOTS) {
        const int64_t m = std::min<int64_t>(RB_PASS_SLOTS, nslots - lo);
        c += ((n + 3) & ~(int64_t)3) + nstreams * stream_slack(m);
    }
    return c;
}

// dynamic LDS of a bucketing launch: a single workgroup may take the whole 160 KiB of a CU
// (MI355X_MICROARCH.md), less the kernel's few static bytes.  NVRX_RB_LDS_KB (a build-time
// tuning constant) caps it lower (round 4's variants that left class-kernel blocks room beside a
// bucketing block: slower, profiles/r04/zipf_ab/).
#ifndef NVRX_RB_LDS_KB
#define NVRX_RB_LDS_KB 160
#endif
constexpr size_t RB_LAUNCH_LDS = (size_t)NVRX_RB_LDS_KB * 1024 - 256;
// register-held record pairs per block, whatever the wave count: 16,384 pairs = 256 KiB =
// 64 KiB per SIMD (half its register file) -- 4 waves x 64 pairs per lane (256 VGPRs),
// 8 x 32 or 16 x 16 (64 VGPRs)
#ifndef NVRX_RB_REGS_PER_BLOCK
#define NVRX_RB_REGS_PER_BLOCK 16384
#endif
constexpr int RB_REGS_PER_BLOCK = NVRX_RB_REGS_PER_BLOCK;
#ifndef NVRX_RB_STAGE_KB
#define NVRX_RB_STAGE_KB 96
#endif
constexpr int RB_STAGE_KB = NVRX_RB_STAGE_KB;  // LDS staging of the cold buckets
#ifndef NVRX_RB_COLD  // build-time tuning constant
#define NVRX_RB_COLD 512
#endif
constexpr int RB_COLD = NVRX_RB_COLD;  // largest cold bucket (records)

// The shipped configuration: 16 waves x 16 register pairs per lane (4 waves / SIMD, 128
// VGPRs), LDS stash interleaved with pass 2, 96 KiB of cold-bucket staging, cold = keep <= 512.
// The alternatives measured on configs[3] (4 / 8 waves, no register pairs, 2-3 blocks per CU,
// other stage sizes and cold limits, no stash) are in DESIGN.md section 3.4.
#ifndef NVRX_RB_WAVES
#define NVRX_RB_WAVES 16
#endif
constexpr int RB_WAVES = NVRX_RB_WAVES;
constexpr int RB_REGS = RB_REGS_PER_BLOCK / (64 * RB_WAVES);

static hipError_t records_bucket_pass(const nvrx_record* recs, const int64_t* rec_off, int64_t t0,
                                      int64_t nlaunch, int64_t nstreams, int64_t nslots, int64_t cap,
                                      int force_stable, int64_t* seg_off, int32_t* seg_len, uint32_t* out_ns,
                                      int32_t* counts, hipStream_t st, const nvrx_stats_soa* tiny,
                                      uint32_t slot_lo, int64_t seg_stride, int pass) {
    if (nlaunch <= 0 || nslots <= 0) return hipSuccess;
    const size_t lds = (size_t)nslots * 3 * sizeof(uint32_t);
    if (lds > NVRX_RECORDS_MAX_LDS) return hipErrorInvalidValue;
    const nvrx_stats_soa tiny_soa = tiny ? *tiny : nvrx_stats_soa{};
    // Streams resident at once = blocks per CU x CUs.  One block per CU (the whole LDS) keeps
    // the resident streams and their bucket outputs (scattered 4-B writes) inside the 256 MB
    // Infinity Cache, where partial lines merge (configs[3]: 5.6 ms with 6 blocks/CU -> 4.4 ms
    // with one, round 1).  That block holds a whole configs[3] stream between the passes:
    // its LDS stash plus RB_REGS_PER_BLOCK register pairs, so pass 2 reads little back.
    // Pass 2 is LDS-atomic latency bound: 16 waves x 16 register pairs (4 waves per SIMD)
    // beat 8 x 32 and 4 x 64 (configs[3] statistics 5.25 / 5.31 / 5.51 ms).
    const size_t lds_launch = std::max(lds, RB_LAUNCH_LDS);
    // The LDS that the counters leave over: the staged cold buckets, then the head of every
    // wave's chunk from pass 1 to pass 2 (a whole number of 64-pair wave loads per wave).
    const size_t counters = (size_t)((3 * nslots + 3) & ~(int64_t)3) * sizeof(uint32_t);
    int64_t stage_cap = 0;
    if (lds_launch > counters)
        stage_cap = std::min<int64_t>((int64_t)RB_STAGE_KB * 256, (int64_t)(lds_launch - counters) / 4) & ~(int64_t)3;
    const size_t fixed = counters + (size_t)stage_cap * 4;
    int64_t stash_pairs = 0;
    if (lds_launch > fixed) stash_pairs = (int64_t)((lds_launch - fixed) / (16 * (size_t)RB_WAVES)) & ~(int64_t)63;
    if (fixed + (size_t)RB_WAVES * 16 * (size_t)stash_pairs > lds_launch) return hipErrorInvalidValue;
    static size_t attr_lds = 0;
    if (attr_lds < lds_launch) {
        const void* k = (const void*)records_bucket_kernel<RB_WAVES, RB_REGS>;
        hipFuncAttributes fa;
        hipError_t e = hipFuncGetAttributes(&fa, k);
        if (e != hipSuccess) return e;
        if (fa.sharedSizeBytes + lds_launch > 160 * 1024) return hipErrorInvalidConfiguration;  // static LDS grew
        e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_launch);
        if (e != hipSuccess) return e;
        attr_lds = lds_launch;
    }
    hipLaunchKernelGGL((records_bucket_kernel<RB_WAVES, RB_REGS>), dim3((unsigned)nlaunch), dim3(64 * RB_WAVES),
                       lds_launch, st, recs, rec_off, nslots, cap, force_stable, seg_off, seg_len, out_ns,
                       counts, stash_pairs, stage_cap, (uint32_t)RB_COLD, tiny_soa, slot_lo, seg_stride, pass,
                       t0, nstreams);
    return hipGetLastError();
}

// streams [t0, t0 + nlaunch) of nstreams
static hipError_t records_bucket_range(const nvrx_record* recs, const int64_t* rec_off, int64_t t0,
                                       int64_t nlaunch, int64_t nstreams, int64_t nslots, int64_t cap,
                                       int force_stable, int64_t* seg_off, int32_t* seg_len,
                                       uint32_t* out_ns, int32_t* counts, hipStream_t st,
                                       const nvrx_stats_soa* tiny) {
    // seg_off / seg_len / counts stay [nstreams][nslots]; pass p writes its slot range's columns
    // and its buckets into out_ns after the regions of the passes before it
    int pass = 0;
    for (int64_t lo = 0; lo < nslots; lo += RB_PASS_SLOTS, ++pass) {
        const int64_t m = std::min<int64_t>(RB_PASS_SLOTS, nslots - lo);
        hipError_t e = records_bucket_pass(recs, rec_off, t0, nlaunch, nstreams, m, cap, force_stable,
                                           seg_off, seg_len, out_ns, counts, st, tiny, (uint32_t)lo,
                                           nslots, pass);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t records_bucket(const nvrx_record* recs, const int64_t* rec_off, int64_t nstreams,
                          int64_t nslots, int64_t cap, int force_stable, int64_t* seg_off,
                          int32_t* seg_len, uint32_t* out_ns, int32_t* counts, hipStream_t st,
                          const nvrx_stats_soa* tiny) {
    return records_bucket_range(recs, rec_off, 0, nstreams, nstreams, nslots, cap, force_stable, seg_off,
                                seg_len, out_ns, counts, st, tiny);
}

// Whole record-stream report statistics: bucketing (which reduces the staged buckets of <=
// RB_TINY records itself), then length-classed statistics of every other bucket; col_ref by a
// column reduction (cheaper than per-segment atomics once there are many streams).
hipError_t records_stats(const nvrx_record* recs, const int64_t* rec_off, int64_t nstreams,
                         int64_t nslots, int64_t cap, int mode, int64_t max_len, int64_t* seg_off,
                         int32_t* seg_len, uint32_t* out_ns, int32_t* counts,
                         const nvrx_stats_soa& out, uint32_t* col_ref, hipStream_t st) {
    // (round 4 measured bucketing stream chunks while the previous chunk's class kernels ran on
    // a second stream, with and without a smaller bucketing block to make room for them: 4.57-5.43
    // against 4.15-4.17 ms, profiles/r04/zipf_ab/)
    hipError_t e = records_bucket(recs, rec_off, nstreams, nslots, cap, 0, seg_off, seg_len, out_ns,
                                  counts, st, &out);
    if (e != hipSuccess) return e;
    const int64_t keep = std::max<int64_t>(1, (cap > 0 && max_len > cap) ? cap : max_len);
    e = segment_stats_ragged(out_ns, seg_off, seg_len, nstreams * nslots, keep, 0, mode, true, out,
                             nullptr, 0, st);
    if (e != hipSuccess || !col_ref) return e;
    return kernel_ref(out.num, out.med, nstreams, nslots, nullptr, col_ref, st);
}

// Turn retained buckets back into a record stream (slot-major, push order kept inside a
// slot): used to compact a long-lived device record log without changing which records
// a later retention step keeps.  dst_off[s] = first output index of slot s.
__global__ void records_unbucket_kernel(const int64_t* seg_off, const int32_t* seg_len,
                                        const int64_t* dst_off, const uint32_t* ns, int64_t nslots,
                                        nvrx_record* out) {
    const int64_t s = blockIdx.x;
    if (s >= nslots) return;
    const int64_t b = seg_off[s], d = dst_off[s];
    const int32_t len = seg_len[s];
    for (int32_t i = threadIdx.x; i < len; i += blockDim.x) {
        nvrx_record r;
        r.slot = (uint32_t)s;
        r.ns = ns[b + i];
        out[d + i] = r;
    }
}

hipError_t records_unbucket(const int64_t* seg_off, const int32_t* seg_len, const int64_t* dst_off,
                            const uint32_t* ns, int64_t nslots, nvrx_record* out, hipStream_t st) {
    if (nslots <= 0) return hipSuccess;
    hipLaunchKernelGGL(records_unbucket_kernel, dim3((unsigned)nslots), dim3(256), 0, st, seg_off,
                       seg_len, dst_off, ns, nslots, out);
    return hipGetLastError();
}

// nvrx_profiler_ingest's copy into the device log: slots not registered when the records were
// handed over are invalidated, so a slot registered later never counts them
__global__ void records_ingest_kernel(nvrx_record* dst, const nvrx_record* src, int64_t n, uint32_t nslots) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        nvrx_record r = src[i];
        if (r.slot >= nslots) r.slot = 0xFFFFFFFFu;
        dst[i] = r;
    }
}

hipError_t records_ingest(nvrx_record* dst, const nvrx_record* src, int64_t n, uint32_t nslots,
                          hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(records_ingest_kernel, dim3((unsigned)blocks), dim3(256), 0, st, dst, src, n, nslots);
    return hipGetLastError();
}

}  // namespace nvrx
