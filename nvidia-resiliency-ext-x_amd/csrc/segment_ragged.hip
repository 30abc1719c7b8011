// segment_ragged.hip -- statistics of ragged segments (gfx950): length classes.
//
// Ragged inputs (the per-(rank, kernel) buckets of record streams, the profiler's
// per-kernel rings) mix a few long segments with very many short ones: under a Zipf
// kernel-frequency law most kernels fire a handful of times per report interval
// (SURVEY.md 8(d), C4).  One wave per segment sized for the longest one would spend
// 64*PL lanes-slots on a 3-sample segment, so segments are first sorted into length
// classes and each class runs the kernel shaped for it:
//
//   n == 0            classifier writes the empty KernelStats (num 0, NaN) itself
//   n <= 8/32/64/128  one LANE per segment: the samples in registers, a bitonic
//                     sorting network, then CuptiProfiler.cpp:53-71 statement by
//                     statement (sequential f32 sums) -- every field bit-exact
//   n <= 64*PL        one WAVE per segment (fast_body, segment_kernels.h), PL 4..128
//   longer / EXACT    one WORKGROUP per segment (exact_body)
//
// Classification is three small launches over the segment lengths (count per block,
// scan, scatter) into one id list ordered by class; every class kernel is persistent
// (grid = CUs x occupancy) and reads its [start, count) from device memory, so the
// host never waits for the class sizes.
#include "segment_ragged_kernels.h"

namespace nvrx {

using namespace ragged;

hipError_t segment_stats_ragged(const uint32_t* ns, const int64_t* seg_off, const int32_t* seg_len,
                                int64_t nseg, int64_t max_len, int64_t cap, int mode,
                                bool aligned16, const nvrx_stats_soa& out, uint32_t* col_ref,
                                int64_t ncols, hipStream_t st) {
    ColRef cr;
    if (hipError_t e = make_colref(col_ref, ncols, st, cr); e != hipSuccess) return e;
    if (nseg <= 0) return hipSuccess;
    RaggedSegs segs{ns, seg_off, seg_len, cap};
    const int64_t keep = (cap > 0 && max_len > cap) ? cap : max_len;
    if (keep > NVRX_MAX_SEGMENT) return hipErrorInvalidValue;
    const int64_t need = aligned16 ? keep : keep + 3;
    const bool exact = mode == NVRX_STATS_EXACT;
    if (nseg >= ((int64_t)1 << 32) - ((int64_t)1 << 26)) return hipErrorInvalidValue;  // 32-bit lists

    const int64_t nblocks = std::min<int64_t>(CLS_MAX_BLOCKS, (nseg + CLS_THREADS - 1) / CLS_THREADS);
    const int64_t chunk = (nseg + nblocks - 1) / nblocks;
    // scratch: list [nseg] | bcnt [nblocks][NCLASS] | cls [NCLASS][2]
    const size_t bytes = (size_t)(nseg + nblocks * NCLASS + 2 * NCLASS) * sizeof(uint32_t);
    void* ws = nullptr;
    if (hipError_t e = scratch_alloc(&ws, bytes, st); e != hipSuccess) return e;
    uint32_t* list = (uint32_t*)ws;
    uint32_t* bcnt = list + nseg;
    uint32_t* cls = bcnt + nblocks * NCLASS;

    hipLaunchKernelGGL(classify_count_kernel, dim3((unsigned)nblocks), dim3(CLS_THREADS), 0, st, segs,
                       nseg, chunk, aligned16 ? 1 : 0, exact ? 1 : 0, bcnt, out, cr);
    hipLaunchKernelGGL(classify_scan_kernel, dim3(1), dim3(CLS_MAX_BLOCKS), 0, st, bcnt, (int)nblocks,
                       cls);
    hipLaunchKernelGGL(classify_scatter_kernel, dim3((unsigned)nblocks), dim3(CLS_THREADS), 0, st,
                       segs, nseg, chunk, aligned16 ? 1 : 0, exact ? 1 : 0, bcnt, list);
    // class kernels; classes that max_len rules out are not launched
    const uint32_t* c = cls;
    ragged_launch_lane(8, segs, list, c + 2 * C_T8, aligned16, out, cr, st);
    if (keep > 8) ragged_launch_lane(32, segs, list, c + 2 * C_T32, aligned16, out, cr, st);
    if (keep > 32) ragged_launch_lane(64, segs, list, c + 2 * C_T64, aligned16, out, cr, st);
    if (keep > 64) ragged_launch_lane(128, segs, list, c + 2 * C_T128, aligned16, out, cr, st);
    if (!exact) {
        if (keep > 128) ragged_launch_list(4, segs, list, c + 2 * C_W4, out, cr, st);
        if (need > 64 * 4) ragged_launch_list(8, segs, list, c + 2 * C_W8, out, cr, st);
        if (need > 64 * 8) ragged_launch_list(16, segs, list, c + 2 * C_W16, out, cr, st);
        if (need > 64 * 16) ragged_launch_list(32, segs, list, c + 2 * C_W32, out, cr, st);
        if (need > 64 * 32) ragged_launch_list(64, segs, list, c + 2 * C_W64, out, cr, st);
        if (need > 64 * 64) ragged_launch_list(128, segs, list, c + 2 * C_W128, out, cr, st);
    }
    if (exact ? keep > 128 : need > 64 * 128) {
        if (hipError_t e = ragged_launch_exact(segs, list, c + 2 * C_X, keep, out, cr, st); e != hipSuccess)
            return e;
    }
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    return hipFreeAsync(ws, st);
}

}  // namespace nvrx
