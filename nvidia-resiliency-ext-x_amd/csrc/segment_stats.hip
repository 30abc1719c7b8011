// segment_stats.hip -- per-kernel duration statistics on gfx950 (MI355X).
//
// Replaces the reference's CPU computeStats (straggler/cupti_src/CuptiProfiler.cpp:44-74,
// reached from CuptiProfiler::getStats :136-146) for a whole batch of segments at once.
// A segment is one (rank, kernel) ring: the last `cap` integer-ns durations
// (CircularBuffer.h:53-69 keeps the last statsMaxLenPerKernel pushes).
//
// FAST mode (the batch/bench path), one 64-lane wave per segment:
//   * the segment (<= 64*PL samples) is streamed HBM -> VGPRs with 16-B loads, once;
//   * MIN/MAX: wave min/max of the u32 keys;
//   * AVG/STD: exact u64 sum of (x - min) and an f64 sum of squares (no sort needed);
//   * MED: radix select on (x - min) with a wave-private LDS histogram (NB bins);
//     the target bucket is then resolved by candidate extraction (<= 64 values,
//     ballot/mbcnt compaction + rank-by-compare) or another histogram level.
//   MIN/MAX/MED are selected on the integer keys and converted exactly as
//   CuptiProfiler.cpp:187 converts one duration; ns -> us is monotone, so the
//   k-th smallest key converts to the k-th smallest float: NUM/MIN/MAX/MED are
//   bit-exact with the reference.  AVG/STD are the exact mean/population std of
//   the retained samples rounded once to f32 (within ~1e-6 of the reference's
//   sequential-f32 values; see DESIGN.md, "AVG/STD modes").
//
// EXACT mode (live path, small batches): one 256-thread workgroup per segment,
//   samples converted to f32 us, bitonic-sorted in LDS, then AVG = sequential f32
//   sum over the sorted samples and STD = sqrtf(sequential sum of squares / n),
//   exactly as CuptiProfiler.cpp:63-69 -- every field bit-exact.

#include "segment_kernels.h"

namespace nvrx {

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
// Shape checks happen here, on the host, before any launch: a fast-mode wave
// holds at most 64*128 samples (+ up to 3 slots of 16-B misalignment); longer
// or misaligned-and-full segments go to the EXACT kernel (bit-exact, slower).
hipError_t segment_stats_strided(const uint32_t* ns, int64_t nseg, int64_t seg_stride,
                                 int64_t seg_begin, int64_t seg_len, int64_t cap, int mode,
                                 const nvrx_stats_soa& out, uint32_t* col_ref, int64_t ncols,
                                 hipStream_t st) {
    const bool ready = (mode & NVRX_STATS_COLREF_READY) != 0;
    mode &= ~NVRX_STATS_COLREF_READY;
    ColRef cr;
    if (hipError_t e = make_colref(col_ref, ncols, st, cr, ready); e != hipSuccess) return e;
    if (nseg <= 0) return hipSuccess;
    StridedSegs segs{ns, seg_stride, seg_begin, seg_len, cap};
    const int64_t keep = (cap > 0 && seg_len > cap) ? cap : seg_len;
    if (keep > NVRX_MAX_SEGMENT) return hipErrorInvalidValue;
    const bool aligned = ((seg_stride % 4) == 0) &&
                         ((((uintptr_t)(ns + seg_begin + (seg_len - keep))) & 15) == 0);
    const int64_t need = aligned ? keep : keep + 3;
    if (mode == NVRX_STATS_EXACT || need > 64 * 128) return launch_exact(segs, nseg, keep, out, cr, st);
    // every strided segment has the same length and (aligned) phase
    return launch_fast(segs, nseg, need, aligned ? keep : -1, out, cr, st);
}

// raw u32 ns (durations below 2^32 ns, never encoded) -> duration keys, in place: values from
// NVRX_KEY_WIDE (3.76 s) up become 0xE0000000 + bits(f32(ns)) - bits(f32(0xE0000000)), as
// nvrx_duration_key encodes the same u64 (v_cvt_f32_u32 rounds to nearest even, like the u64
// conversion of CuptiProfiler.cpp:187).  One coalesced read-modify-write pass.
__global__ __launch_bounds__(256) void encode_ns_u32_kernel(uint32_t* ns, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint32_t v = ns[i];
        if (v >= NVRX_KEY_WIDE) ns[i] = NVRX_KEY_WIDE + (__float_as_uint((float)v) - NVRX_KEY_WIDE_F32BITS);
    }
}

hipError_t encode_ns_u32(uint32_t* ns, int64_t n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(encode_ns_u32_kernel, dim3((unsigned)blocks), dim3(256), 0, st, ns, n);
    return hipGetLastError();
}

}  // namespace nvrx
