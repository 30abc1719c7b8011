// nvrx_internal.h -- internal (C++) interfaces between the HIP kernel files and the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nvrx_straggler.h"

namespace nvrx {

// longest retained segment the one-workgroup EXACT kernel sorts in LDS (128 KiB of f32); longer
// rings (up to NVRX_MAX_SEGMENT) sort in device scratch (exact_global_body, segment_kernels.h)
#define NVRX_LDS_SEGMENT 32768

hipError_t segment_stats_strided(const uint32_t* ns, int64_t nseg, int64_t seg_stride,
                                 int64_t seg_begin, int64_t seg_len, int64_t cap, int mode,
                                 const nvrx_stats_soa& out, uint32_t* col_ref, int64_t ncols,
                                 hipStream_t st);
hipError_t segment_stats_ragged(const uint32_t* ns, const int64_t* seg_off, const int32_t* seg_len,
                                int64_t nseg, int64_t max_len, int64_t cap, int mode,
                                bool aligned16, const nvrx_stats_soa& out, uint32_t* col_ref,
                                int64_t ncols, hipStream_t st);

hipError_t encode_ns_u32(uint32_t* ns, int64_t n, hipStream_t st);

hipError_t kernel_ref(const int32_t* num, const float* med, int64_t R, int64_t K, float* ref,
                      uint32_t* scratch, hipStream_t st);
hipError_t pack_min_times(const double* med, const int32_t* ids, int64_t n, float* times,
                          int64_t total, hipStream_t st);
hipError_t scores(const nvrx_score_args& a, hipStream_t st);
hipError_t finalize_scores(const double* partials, int64_t R, int64_t nshards, int round_f32,
                           double thr_rel, double thr_ind, double* gpu_rel, double* gpu_ind,
                           uint8_t* strag_rel, uint8_t* strag_ind, int32_t* err, hipStream_t st);
hipError_t section_scores(const double* med, const uint8_t* present, int64_t R, int64_t S,
                          const float* ref_in, const int32_t* ref_index, float* ref_work,
                          double* hist, int round_f32, double* out_rel, double* out_ind,
                          int32_t* err, hipStream_t st);
hipError_t section_stats(const double* vals, const int64_t* off, int64_t nsec, int64_t max_len,
                         int32_t* num, double* mn, double* mx, double* med, double* avg,
                         double* sd, hipStream_t st);
hipError_t stragglers(const double* score, int64_t n, double thr, uint8_t* mask, hipStream_t st);

#define NVRX_RECORDS_MAX_LDS (144 * 1024)
// Stream-ordered device scratch from a private memory pool per device (segment_ragged.hip): it keeps
// up to NVRX_SCRATCH_KEEP_BYTES of freed blocks across synchronisations, so steady-state reports
// do not return to the driver, while a long-ring report's larger scratch goes back to the job.
#define NVRX_SCRATCH_KEEP_BYTES ((uint64_t)256 << 20)
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t st);
int64_t records_bucket_capacity(int64_t n, int64_t nstreams, int64_t nslots);
hipError_t records_bucket(const nvrx_record* recs, const int64_t* rec_off, int64_t nstreams,
                          int64_t nslots, int64_t cap, int force_stable, int64_t* seg_off,
                          int32_t* seg_len, uint32_t* out_ns, int32_t* counts, hipStream_t st,
                          const nvrx_stats_soa* tiny = nullptr);
hipError_t records_stats(const nvrx_record* recs, const int64_t* rec_off, int64_t nstreams,
                         int64_t nslots, int64_t cap, int mode, int64_t max_len, int64_t* seg_off,
                         int32_t* seg_len, uint32_t* out_ns, int32_t* counts,
                         const nvrx_stats_soa& out, uint32_t* col_ref, hipStream_t st);
// dst[i] = src[i] with every slot >= nslots replaced by UINT32_MAX (never counted)
hipError_t records_ingest(nvrx_record* dst, const nvrx_record* src, int64_t n, uint32_t nslots,
                          hipStream_t st);
hipError_t records_unbucket(const int64_t* seg_off, const int32_t* seg_len, const int64_t* dst_off,
                            const uint32_t* ns, int64_t nslots, nvrx_record* out, hipStream_t st);

// abi.cpp <-> capture.cpp
#include <string>
void set_error(const std::string& msg);
// one completed dispatch: what the reference's composite key is built from
// (CuptiProfiler.cpp:182-185: kernel name, block dims, grid dims in blocks)
struct DispatchKey {
    uint64_t kernel_id;
    uint32_t bx, by, bz, gx, gy, gz;
    bool operator==(const DispatchKey& o) const {
        return kernel_id == o.kernel_id && bx == o.bx && by == o.by && bz == o.bz && gx == o.gx &&
               gy == o.gy && gz == o.gz;
    }
};
struct DispatchKeyHash {
    size_t operator()(const DispatchKey& k) const {
        uint64_t h = k.kernel_id * 0x9E3779B97F4A7C15ull;
        for (uint32_t v : {k.bx, k.by, k.bz, k.gx, k.gy, k.gz}) h = (h ^ v) * 0x100000001B3ull;
        return (size_t)(h ^ (h >> 29));
    }
};
struct DispatchRec {
    DispatchKey key;
    uint64_t ns;  // end - start
};
// push one delivered batch; composite_name builds "%s_blk_%d_%d_%d_grid_%d_%d_%d" for a key
// the profiler has not seen since its last reset
void profiler_push_dispatches(nvrx_profiler* p, const DispatchRec* r, size_t n,
                              std::string (*composite_name)(const DispatchKey&));
bool capture_ready();
int capture_start(nvrx_profiler* p);
int capture_stop(nvrx_profiler* p);
int capture_flush();
// callback delivery: move the completed dispatches queued so far into p (the caller's thread)
void capture_drain(nvrx_profiler* p);
void capture_detach(nvrx_profiler* p);
// mark the calling thread's kernel dispatches as the library's own (not captured) until
// capture_self_end; false when the capture is off or rocprofiler-sdk cannot mark them
bool capture_self_begin();
void capture_self_end();

}  // namespace nvrx
