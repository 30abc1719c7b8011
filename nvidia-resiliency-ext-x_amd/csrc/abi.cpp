// abi.cpp -- the extern "C" boundary of libnvrx_hip.so (declared in include/nvrx_straggler.h).
//
// Thin host glue: argument/shape checks on the host before any launch, HIP error ->
// status code + thread-local message, and the profiler handle that replaces the
// reference's nvrx_cupti_module.CuptiProfiler (straggler/cupti_src/CuptiProfiler.cpp,
// cupti_module_py.cpp).  All arithmetic runs in the HIP kernels of segment_stats.hip,
// scores.hip and records.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "nvrx_internal.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
int hip_status(hipError_t e, const char* where) {
    if (e == hipSuccess) return NVRX_OK;
    return fail(e == hipErrorInvalidValue ? NVRX_ERR_INVALID : NVRX_ERR_HIP,
                std::string(where) + ": " + hipGetErrorString(e));
}
#define NVRX_CHECK_ARG(cond, msg) \
    do {                          \
        if (!(cond)) return fail(NVRX_ERR_INVALID, msg); \
    } while (0)

hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace

namespace nvrx {
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace nvrx

extern "C" {

const char* nvrx_last_error(void) { return g_last_error.c_str(); }

uint32_t nvrx_duration_key(uint64_t ns) {
    if (ns < NVRX_KEY_WIDE) return (uint32_t)ns;
    const float f = (float)ns;  // u64 -> f32, round to nearest: CuptiProfiler.cpp:187's conversion
    uint32_t b;
    std::memcpy(&b, &f, sizeof b);
    return NVRX_KEY_WIDE + (b - NVRX_KEY_WIDE_F32BITS);
}
int nvrx_abi_version(void) { return NVRX_ABI_VERSION; }

int nvrx_encode_ns_u32(uint32_t* ns, int64_t n, void* stream) {
    NVRX_CHECK_ARG(n >= 0 && (n == 0 || ns), "nvrx_encode_ns_u32: bad args");
    return hip_status(nvrx::encode_ns_u32(ns, n, S(stream)), "nvrx_encode_ns_u32");
}

int nvrx_device_count(int* count) {
    NVRX_CHECK_ARG(count, "nvrx_device_count: null count");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e == hipErrorNoDevice) c = 0, e = hipSuccess;
    *count = c;
    return hip_status(e, "hipGetDeviceCount");
}

int nvrx_sync(void* stream) { return hip_status(hipStreamSynchronize(S(stream)), "nvrx_sync"); }

// ------------------------------------------------------------------ statistics
int nvrx_segment_stats_strided(const uint32_t* ns, int64_t nseg, int64_t seg_stride,
                               int64_t seg_begin, int64_t seg_len, int64_t cap, int32_t mode,
                               const nvrx_stats_soa* out, uint32_t* col_ref, int64_t ncols,
                               void* stream) {
    NVRX_CHECK_ARG(out && out->num && out->min && out->max && out->med && out->avg && out->std,
                   "nvrx_segment_stats_strided: null output array");
    NVRX_CHECK_ARG(nseg >= 0 && seg_len >= 0 && seg_begin >= 0 && seg_stride >= 0,
                   "nvrx_segment_stats_strided: negative size");
    NVRX_CHECK_ARG(nseg == 0 || seg_len == 0 || ns, "nvrx_segment_stats_strided: null ns");
    NVRX_CHECK_ARG((mode & ~NVRX_STATS_COLREF_READY) == NVRX_STATS_FAST ||
                       (mode & ~NVRX_STATS_COLREF_READY) == NVRX_STATS_EXACT,
                   "nvrx_segment_stats_strided: unknown mode");
    NVRX_CHECK_ARG(nseg <= 1 || seg_stride >= seg_begin + seg_len,
                   "nvrx_segment_stats_strided: segments overlap (stride < begin + len)");
    const int64_t keep = (cap > 0 && seg_len > cap) ? cap : seg_len;
    NVRX_CHECK_ARG(keep <= NVRX_MAX_SEGMENT,
                   "nvrx_segment_stats_strided: retained segment longer than NVRX_MAX_SEGMENT (2^30)");
    NVRX_CHECK_ARG(nseg < (int64_t)1 << 33, "nvrx_segment_stats_strided: too many segments");
    NVRX_CHECK_ARG(!col_ref || (ncols > 0 && nseg % ncols == 0),
                   "nvrx_segment_stats_strided: col_ref needs ncols > 0 dividing nseg");
    return hip_status(nvrx::segment_stats_strided(ns, nseg, seg_stride, seg_begin, seg_len, cap,
                                                  mode, *out, col_ref, ncols, S(stream)),
                      "nvrx_segment_stats_strided");
}

int nvrx_segment_stats_ragged(const uint32_t* ns, const int64_t* seg_off, const int32_t* seg_len,
                              int64_t nseg, int64_t max_len, int64_t cap, int32_t mode,
                              int32_t aligned16, const nvrx_stats_soa* out, uint32_t* col_ref,
                              int64_t ncols, void* stream) {
    NVRX_CHECK_ARG(out && out->num && out->min && out->max && out->med && out->avg && out->std,
                   "nvrx_segment_stats_ragged: null output array");
    NVRX_CHECK_ARG(nseg >= 0 && max_len >= 0, "nvrx_segment_stats_ragged: negative size");
    NVRX_CHECK_ARG(nseg == 0 || (seg_off && ns), "nvrx_segment_stats_ragged: null input");
    NVRX_CHECK_ARG(mode == NVRX_STATS_FAST || mode == NVRX_STATS_EXACT,
                   "nvrx_segment_stats_ragged: unknown mode");
    const int64_t keep = (cap > 0 && max_len > cap) ? cap : max_len;
    NVRX_CHECK_ARG(keep <= NVRX_MAX_SEGMENT,
                   "nvrx_segment_stats_ragged: retained segment longer than NVRX_MAX_SEGMENT (2^30)");
    NVRX_CHECK_ARG(nseg < (int64_t)1 << 31, "nvrx_segment_stats_ragged: too many segments");
    NVRX_CHECK_ARG(!col_ref || (ncols > 0 && nseg % ncols == 0),
                   "nvrx_segment_stats_ragged: col_ref needs ncols > 0 dividing nseg");
    return hip_status(nvrx::segment_stats_ragged(ns, seg_off, seg_len, nseg, max_len, cap, mode,
                                                 aligned16 != 0, *out, col_ref, ncols, S(stream)),
                      "nvrx_segment_stats_ragged");
}

// ------------------------------------------------------------------ scoring
int nvrx_kernel_ref(const int32_t* num, const float* med, int64_t R, int64_t K, float* ref,
                    uint32_t* scratch, void* stream) {
    NVRX_CHECK_ARG(R >= 0 && K >= 0, "nvrx_kernel_ref: negative size");
    NVRX_CHECK_ARG(K == 0 || (ref && scratch), "nvrx_kernel_ref: null ref/scratch");
    NVRX_CHECK_ARG(R == 0 || K == 0 || (num && med), "nvrx_kernel_ref: null num/med");
    NVRX_CHECK_ARG((R + 63) / 64 < 65536, "nvrx_kernel_ref: too many rows");
    return hip_status(nvrx::kernel_ref(num, med, R, K, ref, scratch, S(stream)), "nvrx_kernel_ref");
}

int nvrx_pack_min_times(const double* med, const int32_t* ids, int64_t n, float* times,
                        int64_t total, void* stream) {
    NVRX_CHECK_ARG(n >= 0 && total >= 0, "nvrx_pack_min_times: negative size");
    NVRX_CHECK_ARG(total == 0 || times, "nvrx_pack_min_times: null times");
    NVRX_CHECK_ARG(n == 0 || (med && ids), "nvrx_pack_min_times: null inputs");
    NVRX_CHECK_ARG(n <= total, "nvrx_pack_min_times: more entries than the tensor holds");
    return hip_status(nvrx::pack_min_times(med, ids, n, times, total, S(stream)),
                      "nvrx_pack_min_times");
}

int nvrx_scores(const nvrx_score_args* a, void* stream) {
    NVRX_CHECK_ARG(a, "nvrx_scores: null args");
    NVRX_CHECK_ARG(a->R >= 0 && a->K >= 0, "nvrx_scores: negative size");
    NVRX_CHECK_ARG(a->R == 0 || a->partials || a->gpu_rel || a->gpu_ind || a->strag_rel ||
                       a->strag_ind,
                   "nvrx_scores: no output (partials or finalized scores)");
    NVRX_CHECK_ARG(a->R == 0 || a->K == 0 || (a->num && a->med && a->avg),
                   "nvrx_scores: null num/med/avg");
    NVRX_CHECK_ARG(!a->hist_index || a->hist_stride > 0,
                   "nvrx_scores: hist_index requires hist_stride");
    NVRX_CHECK_ARG(a->value_f64 == 0 || a->value_f64 == 1, "nvrx_scores: bad value_f64");
    NVRX_CHECK_ARG(a->reset_ncols >= 0 && (a->reset_ncols == 0 || (a->reset_col_ref && a->done)),
                   "nvrx_scores: reset_col_ref needs done and reset_ncols >= 0");
    return hip_status(nvrx::scores(*a, S(stream)), "nvrx_scores");
}

int nvrx_finalize_scores(const double* partials, int64_t R, int64_t nshards, int32_t round_f32,
                         double thr_rel, double thr_ind, double* gpu_rel, double* gpu_ind,
                         uint8_t* strag_rel, uint8_t* strag_ind, int32_t* err, void* stream) {
    NVRX_CHECK_ARG(R >= 0 && nshards >= 1, "nvrx_finalize_scores: bad size");
    NVRX_CHECK_ARG(R == 0 || partials, "nvrx_finalize_scores: null partials");
    return hip_status(nvrx::finalize_scores(partials, R, nshards, round_f32, thr_rel, thr_ind,
                                            gpu_rel, gpu_ind, strag_rel, strag_ind, err, S(stream)),
                      "nvrx_finalize_scores");
}

int nvrx_section_scores(const double* med, const uint8_t* present, int64_t R, int64_t S_,
                        const float* ref_in, const int32_t* ref_index, float* ref_work,
                        double* hist, int32_t round_f32, double* out_rel, double* out_ind,
                        int32_t* err, void* stream) {
    NVRX_CHECK_ARG(R >= 0 && S_ >= 0, "nvrx_section_scores: negative size");
    NVRX_CHECK_ARG(R == 0 || S_ == 0 || (med && present), "nvrx_section_scores: null med/present");
    NVRX_CHECK_ARG(!out_ind || hist, "nvrx_section_scores: individual scores need hist");
    NVRX_CHECK_ARG(!out_rel || ref_in || ref_work, "nvrx_section_scores: need ref_in or ref_work");
    return hip_status(nvrx::section_scores(med, present, R, S_, ref_in, ref_index, ref_work, hist,
                                           round_f32, out_rel, out_ind, err, S(stream)),
                      "nvrx_section_scores");
}

int nvrx_section_stats(const double* vals, const int64_t* off, int64_t nsec, int64_t max_len,
                       int32_t* num, double* mn, double* mx, double* med, double* avg,
                       double* sd, void* stream) {
    NVRX_CHECK_ARG(nsec >= 0 && max_len >= 0, "nvrx_section_stats: negative size");
    NVRX_CHECK_ARG(nsec == 0 || (vals && off && num && mn && mx && med && avg && sd),
                   "nvrx_section_stats: null array");
    return hip_status(nvrx::section_stats(vals, off, nsec, max_len, num, mn, mx, med, avg, sd,
                                          S(stream)),
                      "nvrx_section_stats");
}

int nvrx_stragglers(const double* score, int64_t n, double thr, uint8_t* mask, void* stream) {
    NVRX_CHECK_ARG(n >= 0 && (n == 0 || (score && mask)), "nvrx_stragglers: bad args");
    return hip_status(nvrx::stragglers(score, n, thr, mask, S(stream)), "nvrx_stragglers");
}

// ------------------------------------------------------------------ record streams
int64_t nvrx_records_bucket_capacity(int64_t n, int64_t nstreams, int64_t nslots) {
    return nvrx::records_bucket_capacity(n, nstreams, nslots);
}
int nvrx_records_stats(const nvrx_record* recs, const int64_t* rec_off, int64_t nstreams,
                       int64_t nslots, int64_t cap, int32_t mode, int64_t max_len, int64_t* seg_off,
                       int32_t* seg_len, uint32_t* out_ns, int32_t* counts,
                       const nvrx_stats_soa* out, uint32_t* col_ref, void* stream) {
    NVRX_CHECK_ARG(nstreams >= 0 && nslots >= 0 && max_len >= 0, "nvrx_records_stats: negative size");
    NVRX_CHECK_ARG(out && out->num && out->min && out->max && out->med && out->avg && out->std,
                   "nvrx_records_stats: null output array");
    NVRX_CHECK_ARG(nstreams == 0 || nslots == 0 || (recs && rec_off && seg_off && seg_len && out_ns),
                   "nvrx_records_stats: null array");  // counts may be NULL (not written)
    NVRX_CHECK_ARG(mode == NVRX_STATS_FAST || mode == NVRX_STATS_EXACT,
                   "nvrx_records_stats: unknown mode");
    NVRX_CHECK_ARG(nstreams * nslots < (int64_t)1 << 31, "nvrx_records_stats: too many segments");
    NVRX_CHECK_ARG(((uintptr_t)out_ns & 15) == 0, "nvrx_records_stats: out_ns not 16-byte aligned");
    const int64_t keep = (cap > 0 && max_len > cap) ? cap : max_len;
    NVRX_CHECK_ARG(keep <= NVRX_MAX_SEGMENT, "nvrx_records_stats: retained run longer than NVRX_MAX_SEGMENT (2^30)");
    return hip_status(nvrx::records_stats(recs, rec_off, nstreams, nslots, cap, mode, max_len,
                                          seg_off, seg_len, out_ns, counts, *out, col_ref, S(stream)),
                      "nvrx_records_stats");
}

int64_t nvrx_records_max_slots(void) { return NVRX_RECORDS_MAX_LDS / (3 * sizeof(uint32_t)); }  // W = 1

int nvrx_records_bucket(const nvrx_record* recs, const int64_t* rec_off, int64_t nstreams,
                        int64_t nslots, int64_t cap, int64_t* seg_off, int32_t* seg_len,
                        uint32_t* out_ns, int32_t* counts, void* stream) {
    NVRX_CHECK_ARG(nstreams >= 0 && nslots >= 0, "nvrx_records_bucket: negative size");
    NVRX_CHECK_ARG(nstreams == 0 || nslots == 0 ||
                       (rec_off && seg_off && seg_len && out_ns && counts),
                   "nvrx_records_bucket: null array");
    NVRX_CHECK_ARG(nstreams < (int64_t)1 << 31, "nvrx_records_bucket: too many streams");
    NVRX_CHECK_ARG(((uintptr_t)out_ns & 15) == 0, "nvrx_records_bucket: out_ns not 16-byte aligned");
    return hip_status(nvrx::records_bucket(recs, rec_off, nstreams, nslots, cap, 0, seg_off,
                                           seg_len, out_ns, counts, S(stream)),
                      "nvrx_records_bucket");
}

}  // extern "C"

// ====================================================================== profiler handle
struct nvrx_profiler {
    nvrx_profiler_config cfg{};
    std::mutex mu;
    std::mutex ctx_mu;  // start / stop against a report's capture pause (CaptureSelf fallback)
    bool initialized = false;
    bool started = false;
    // kernels seen since the last reset (the keys of CuptiProfiler's _kernelDurations map,
    // which reset() clears, CuptiProfiler.cpp:148-152): slots are renumbered from 0 after
    // every reset, so a long job with changing launch shapes never runs out of slots
    std::unordered_map<std::string, uint32_t> name_to_slot;
    std::vector<std::string> names;
    // live-capture fast path: (kernel id, block, grid) -> slot, no string work per record
    std::unordered_map<nvrx::DispatchKey, uint32_t, nvrx::DispatchKeyHash> key_to_slot;
    std::vector<nvrx_record> staged;  // host records not yet in the device log
    uint64_t saturated = 0;           // wide-key durations (>= 3.76 s) since the last reset
    uint64_t version = 0;             // bumped whenever the record set or the slot table changes
    uint64_t generation = 1;          // slot numbering epoch: bumped by every reset
    hipStream_t stream = nullptr;
    hipEvent_t ingest_ev = nullptr;   // last nvrx_profiler_ingest copy (on the caller's stream)
    bool ingest_pending = false;
    // device record log (push order since the last reset)
    nvrx_record* d_log = nullptr;
    int64_t log_n = 0, log_cap = 0;
    nvrx_record* h_pinned = nullptr;  // pinned staging of the host -> device drain
    int64_t pinned_cap = 0;
    // pinned staging of a report's small transfers: the bucketing's stream offsets up, the six
    // statistics columns down in one copy (pageable copies each cost a blocking round trip)
    char* h_small = nullptr;
    size_t small_bytes = 0;
    // work buffers (grown on demand)
    void* d_work = nullptr;
    size_t work_bytes = 0;
    // the last get_stats result (name-sorted), valid while version == cache_version
    uint64_t cache_version = ~(uint64_t)0;
    std::vector<uint32_t> c_slot;
    std::vector<int32_t> c_num;
    std::vector<float> c_mn, c_mx, c_med, c_avg, c_sd;
    // staged host records move to the device log once `drain_records` wait (at push, and
    // at stop for the live capture -- on the caller's thread, never on rocprofiler's), so
    // host memory stays bounded between reports
    int64_t drain_records = (int64_t)1 << 16;
};

namespace {

std::mutex g_instance_mu;
nvrx_profiler* g_instance = nullptr;

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int grow_log(nvrx_profiler* p, int64_t need) {
    if (need <= p->log_cap) return NVRX_OK;
    int64_t cap = std::max<int64_t>(need, std::max<int64_t>(1 << 16, p->log_cap * 2));
    nvrx_record* nl = nullptr;
    hipError_t e = hipMalloc(&nl, (size_t)cap * sizeof(nvrx_record));
    if (e != hipSuccess) return hip_status(e, "nvrx_profiler: hipMalloc(record log)");
    if (p->log_n > 0) {
        e = hipMemcpyAsync(nl, p->d_log, (size_t)p->log_n * sizeof(nvrx_record),
                           hipMemcpyDeviceToDevice, p->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
        if (e != hipSuccess) {
            (void)hipFree(nl);
            return hip_status(e, "nvrx_profiler: grow record log");
        }
    }
    if (p->d_log) (void)hipFree(p->d_log);
    p->d_log = nl;
    p->log_cap = cap;
    return NVRX_OK;
}

int ensure_work(nvrx_profiler* p, size_t bytes) {
    if (bytes <= p->work_bytes) return NVRX_OK;
    if (p->d_work) (void)hipFree(p->d_work);
    p->d_work = nullptr;
    p->work_bytes = 0;
    size_t b = std::max(bytes, p->work_bytes * 2);
    hipError_t e = hipMalloc(&p->d_work, b);
    if (e != hipSuccess) return hip_status(e, "nvrx_profiler: hipMalloc(work)");
    p->work_bytes = b;
    return NVRX_OK;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// p->h_small holding at least `bytes` (grown on demand)
int ensure_small(nvrx_profiler* p, size_t bytes) {
    if (bytes <= p->small_bytes) return NVRX_OK;
    if (p->h_small) (void)hipHostFree(p->h_small);
    p->h_small = nullptr;
    p->small_bytes = 0;
    const size_t b = std::max<size_t>(bytes, 4096);
    hipError_t e = hipHostMalloc((void**)&p->h_small, b, 0);
    if (e != hipSuccess) return hip_status(e, "nvrx_profiler: hipHostMalloc(small staging)");
    p->small_bytes = b;
    return NVRX_OK;
}

struct Work {  // carve of d_work for one bucket + stats pass over the record log
    int64_t* rec_off;
    int64_t* seg_off;
    int32_t* seg_len;
    int32_t* counts;
    uint32_t* ns;
    int32_t* num;
    float *mn, *mx, *med, *avg, *sd;
    int64_t* dst_off;
    size_t bytes;
};

Work carve(char* base, int64_t nslots, int64_t ns_cap) {
    Work w{};
    size_t o = 0;
    auto take = [&](size_t b) {
        char* p = base ? base + o : nullptr;
        o += align256(b);
        return p;
    };
    w.rec_off = (int64_t*)take(2 * sizeof(int64_t));
    w.seg_off = (int64_t*)take(nslots * sizeof(int64_t));
    w.seg_len = (int32_t*)take(nslots * sizeof(int32_t));
    w.counts = (int32_t*)take(nslots * sizeof(int32_t));
    w.ns = (uint32_t*)take(ns_cap * sizeof(uint32_t));
    w.num = (int32_t*)take(nslots * sizeof(int32_t));
    w.mn = (float*)take(nslots * sizeof(float));
    w.mx = (float*)take(nslots * sizeof(float));
    w.med = (float*)take(nslots * sizeof(float));
    w.avg = (float*)take(nslots * sizeof(float));
    w.sd = (float*)take(nslots * sizeof(float));
    w.dst_off = (int64_t*)take(nslots * sizeof(int64_t));
    w.bytes = o;
    return w;
}

// Bucket the whole device log (one stream).  Caller holds p->mu.
int bucket_log(nvrx_profiler* p, int64_t nslots, int force_stable, Work& w) {
    const int64_t ns_cap = nvrx::records_bucket_capacity(p->log_n, 1, nslots);
    Work probe = carve(nullptr, nslots, ns_cap);
    int rc = ensure_work(p, probe.bytes);
    if (rc) return rc;
    w = carve((char*)p->d_work, nslots, ns_cap);
    // sized here for get_stats' download too (h_small is never reallocated under a pending copy)
    rc = ensure_small(p, std::max<size_t>(2 * sizeof(int64_t), 6 * align256((size_t)nslots * 4)));
    if (rc) return rc;
    int64_t* off = (int64_t*)p->h_small;  // (the previous use of h_small has completed: synchronous calls)
    off[0] = 0;
    off[1] = p->log_n;
    hipError_t e = hipMemcpyAsync(w.rec_off, off, 2 * sizeof(int64_t), hipMemcpyHostToDevice, p->stream);
    if (e != hipSuccess) return hip_status(e, "nvrx_profiler: rec_off upload");
    e = nvrx::records_bucket(p->d_log, w.rec_off, 1, nslots, p->cfg.stats_max_len_per_kernel,
                             force_stable, w.seg_off, w.seg_len, w.ns, w.counts, p->stream);
    return hip_status(e, "nvrx_profiler: records_bucket");
}

// Move staged host records into the device log (through a pinned buffer: a DMA copy, no
// kernel launch that a started capture could record); compact the log when it is much larger
// than what the rings can retain.  Caller holds p->mu.
int flush_locked(nvrx_profiler* p) {
    DeviceGuard g(p->cfg.device);
    if (p->ingest_pending) {  // device-ingested records were copied on the caller's stream
        hipError_t e = hipStreamWaitEvent(p->stream, p->ingest_ev, 0);
        if (e != hipSuccess) return hip_status(e, "nvrx_profiler: wait for ingest");
        p->ingest_pending = false;
    }
    if (!p->staged.empty()) {
        const int64_t add = (int64_t)p->staged.size();
        int rc = grow_log(p, p->log_n + add);
        if (rc) return rc;
        if (add > p->pinned_cap) {
            if (p->h_pinned) (void)hipHostFree(p->h_pinned);
            p->h_pinned = nullptr;
            p->pinned_cap = 0;
            const int64_t c = std::max<int64_t>(add, p->drain_records);
            hipError_t e = hipHostMalloc((void**)&p->h_pinned, (size_t)c * sizeof(nvrx_record), 0);
            if (e != hipSuccess) return hip_status(e, "nvrx_profiler: hipHostMalloc(staging)");
            p->pinned_cap = c;
        }
        std::memcpy(p->h_pinned, p->staged.data(), (size_t)add * sizeof(nvrx_record));
        hipError_t e = hipMemcpyAsync(p->d_log + p->log_n, p->h_pinned,
                                      (size_t)add * sizeof(nvrx_record), hipMemcpyHostToDevice,
                                      p->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
        if (e != hipSuccess) return hip_status(e, "nvrx_profiler: flush");
        p->log_n += add;
        p->staged.clear();
        if (p->staged.capacity() > (size_t)4 * p->drain_records) p->staged.shrink_to_fit();
    }
    const int64_t nslots = (int64_t)p->names.size();
    const int64_t cap = p->cfg.stats_max_len_per_kernel;
    const int64_t retain_bound = nslots * (cap > 0 ? cap : p->log_n);
    if (cap > 0 && p->log_n > (int64_t)1 << 22 && p->log_n > 4 * retain_bound) {
        // compaction keeps exactly the records a later retention step could still keep
        Work w;
        int rc = bucket_log(p, nslots, /*force_stable=*/1, w);
        if (rc) return rc;
        std::vector<int32_t> len(nslots);
        hipError_t e = hipMemcpyAsync(len.data(), w.seg_len, nslots * sizeof(int32_t),
                                      hipMemcpyDeviceToHost, p->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
        if (e != hipSuccess) return hip_status(e, "nvrx_profiler: compaction lengths");
        std::vector<int64_t> dst(nslots);
        int64_t tot = 0;
        for (int64_t s = 0; s < nslots; ++s) dst[s] = tot, tot += len[s];
        nvrx_record* nl = nullptr;
        e = hipMalloc(&nl, (size_t)std::max<int64_t>(tot, 1) * sizeof(nvrx_record));
        if (e != hipSuccess) return hip_status(e, "nvrx_profiler: hipMalloc(compaction)");
        e = hipMemcpyAsync(w.dst_off, dst.data(), nslots * sizeof(int64_t), hipMemcpyHostToDevice,
                           p->stream);
        if (e == hipSuccess)
            e = nvrx::records_unbucket(w.seg_off, w.seg_len, w.dst_off, w.ns, nslots, nl, p->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
        if (e != hipSuccess) {
            (void)hipFree(nl);
            return hip_status(e, "nvrx_profiler: compaction");
        }
        (void)hipFree(p->d_log);
        p->d_log = nl;
        p->log_n = tot;
        p->log_cap = std::max<int64_t>(tot, 1);
    }
    return NVRX_OK;
}

// The report's own kernels (bucketing, statistics, copies) must not be captured as dispatches
// of the profiled job -- the reference's getStats runs on the host and adds nothing.  They are
// marked by thread (capture_self_begin: rocprofiler-sdk's external correlation id of every
// dispatch this thread makes until the guard ends), so kernels that OTHER threads launch during
// the report are still captured, as CUPTI keeps its activity enabled through getStats.  If the
// marking is unavailable, the dispatch context is paused instead (kernels other threads launch
// meanwhile are then lost); start / stop wait for a pause to end (ctx_mu), and the capture is
// restarted only if the profiler is still started.  Neither makes the flush cheaper
// (rocprofiler_flush_buffer).
struct CaptureSelf {
    nvrx_profiler* p;
    bool marked = false, paused = false;
    std::unique_lock<std::mutex> ctx;
    explicit CaptureSelf(nvrx_profiler* q) : p(q) {
        if (!nvrx::capture_ready()) return;
        marked = nvrx::capture_self_begin();
        if (marked) return;
        ctx = std::unique_lock<std::mutex>(p->ctx_mu);
        bool started;
        {
            std::lock_guard<std::mutex> lk(p->mu);
            started = p->started;
        }
        if (started) paused = nvrx::capture_stop(p) == 0;
    }
    ~CaptureSelf() {
        if (marked) nvrx::capture_self_end();
        if (!paused) return;
        bool started;
        {
            std::lock_guard<std::mutex> lk(p->mu);
            started = p->started;
        }
        if (started) (void)nvrx::capture_start(p);
    }
};

uint32_t slot_of_name(nvrx_profiler* p, const std::string& key) {
    auto it = p->name_to_slot.find(key);
    if (it != p->name_to_slot.end()) return it->second;
    const uint32_t slot = (uint32_t)p->names.size();
    p->name_to_slot.emplace(key, slot);
    p->names.push_back(key);
    return slot;
}

}  // namespace

namespace nvrx {
// the capture's delivery (capture_drain / q_harvest): one batch of completed dispatches.  A dispatch
// enqueued while the profiler was started may complete (and its record arrive) after stop;
// it is still counted, as CUPTI delivers the activity records of kernels launched while the
// activity kind was enabled (bufferCompleted, CuptiProfiler.cpp:168-203, pushes regardless
// of _isStarted).
void profiler_push_dispatches(nvrx_profiler* p, const DispatchRec* r, size_t n,
                              std::string (*composite_name)(const DispatchKey&)) {
    {
        std::lock_guard<std::mutex> lk(p->mu);
        if (!p->initialized) return;
        for (size_t i = 0; i < n; ++i) {
            uint32_t slot;
            auto it = p->key_to_slot.find(r[i].key);
            if (it != p->key_to_slot.end()) {
                slot = it->second;
            } else {
                slot = slot_of_name(p, composite_name(r[i].key));  // CuptiProfiler.cpp:182-185
                p->key_to_slot.emplace(r[i].key, slot);
            }
            // CuptiProfiler.cpp:187 keeps f32(end - start): the duration key carries exactly
            // that for any u64 (the integer ns below 3.76 s)
            const uint32_t key = nvrx_duration_key(r[i].ns);
            if (key >= NVRX_KEY_WIDE) ++p->saturated;
            p->staged.push_back(nvrx_record{slot, key});
        }
        ++p->version;
    }
}
}  // namespace nvrx

extern "C" {

int nvrx_profiler_create(const nvrx_profiler_config* cfg, nvrx_profiler** out) {
    NVRX_CHECK_ARG(cfg && out, "nvrx_profiler_create: null argument");
    NVRX_CHECK_ARG(cfg->stats_max_len_per_kernel > 0 &&
                       cfg->stats_max_len_per_kernel <= NVRX_MAX_SEGMENT,
                   "nvrx_profiler_create: statsMaxLenPerKernel must be in [1, 2^30]");
    NVRX_CHECK_ARG(cfg->mode == NVRX_STATS_FAST || cfg->mode == NVRX_STATS_EXACT,
                   "nvrx_profiler_create: unknown mode");
    if (cfg->stats_max_len_per_kernel > ((int64_t)1 << 24))
        std::fprintf(stderr, "nvrx_profiler_create: statsMaxLenPerKernel=%lld: rings above 2^24 samples "
                             "are reduced in device scratch of up to 4 B per retained sample (4 GiB at "
                             "2^30) by one workgroup per kernel -- slow\n",
                     (long long)cfg->stats_max_len_per_kernel);
    std::lock_guard<std::mutex> lk(g_instance_mu);
    if (g_instance)  // CuptiProfiler.cpp:86-87
        return fail(NVRX_ERR_SINGLETON, "Only one CuptiProfiler instance is allowed.");
    auto* p = new nvrx_profiler();
    p->cfg = *cfg;
    // the drain watermark follows the host buffer size (CUPTI bufferSize, cupti.py:25)
    if (cfg->buffer_size >= (int64_t)sizeof(nvrx_record) * 1024)
        p->drain_records = cfg->buffer_size / (int64_t)sizeof(nvrx_record);
    {
        DeviceGuard g(cfg->device);
        hipError_t e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&p->ingest_ev, hipEventDisableTiming);
        if (e != hipSuccess) {
            if (p->stream) (void)hipStreamDestroy(p->stream);
            delete p;
            return hip_status(e, "nvrx_profiler_create: stream/event");
        }
    }
    g_instance = p;
    *out = p;
    return NVRX_OK;
}

int nvrx_profiler_destroy(nvrx_profiler* p) {
    NVRX_CHECK_ARG(p, "nvrx_profiler_destroy: null handle");
    // no capture callback may touch the handle after this: capture_detach delivers what is
    // pending, unhooks the handle and waits for any callback still running
    nvrx::capture_detach(p);
    {
        std::lock_guard<std::mutex> lk(g_instance_mu);
        if (g_instance == p) g_instance = nullptr;
    }
    {
        DeviceGuard g(p->cfg.device);
        if (p->stream) (void)hipStreamSynchronize(p->stream);
        if (p->d_log) (void)hipFree(p->d_log);
        if (p->d_work) (void)hipFree(p->d_work);
        if (p->h_pinned) (void)hipHostFree(p->h_pinned);
        if (p->h_small) (void)hipHostFree(p->h_small);
        if (p->ingest_ev) (void)hipEventDestroy(p->ingest_ev);
        if (p->stream) (void)hipStreamDestroy(p->stream);
    }
    delete p;
    return NVRX_OK;
}

int nvrx_profiler_initialize(nvrx_profiler* p) {
    NVRX_CHECK_ARG(p, "nvrx_profiler_initialize: null handle");
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->initialized)
        std::fprintf(stderr, "CuptiProfiler::initializeProfiling subsequent call.\n");
    p->initialized = true;
    return NVRX_OK;
}

int nvrx_profiler_shutdown(nvrx_profiler* p) {
    NVRX_CHECK_ARG(p, "nvrx_profiler_shutdown: null handle");
    std::lock_guard<std::mutex> lk(p->mu);
    if (!p->initialized)
        std::fprintf(stderr, "CuptiProfiler::shutdownProfiling called while not initialized.\n");
    p->initialized = false;
    p->started = false;
    return NVRX_OK;
}

int nvrx_profiler_start(nvrx_profiler* p) {
    NVRX_CHECK_ARG(p, "nvrx_profiler_start: null handle");
    std::lock_guard<std::mutex> ctx(p->ctx_mu);  // not inside a report's pause
    {
        std::lock_guard<std::mutex> lk(p->mu);
        if (p->started) std::fprintf(stderr, "CuptiProfiler::startProfiling subsequent call.\n");
        p->started = true;
    }
    // live capture (CuptiProfiler.cpp:115-118 enables the activity kind)
    if (nvrx::capture_start(p) != 0)
        return fail(NVRX_ERR_STATE, "nvrx_profiler_start: rocprofiler_start_context failed");
    return NVRX_OK;
}

int nvrx_profiler_stop(nvrx_profiler* p) {
    NVRX_CHECK_ARG(p, "nvrx_profiler_stop: null handle");
    std::lock_guard<std::mutex> ctx(p->ctx_mu);  // not inside a report's pause
    const int rc = nvrx::capture_stop(p);
    nvrx::capture_drain(p);  // callback delivery: completed dispatches queued so far (before p->mu)
    std::lock_guard<std::mutex> lk(p->mu);
    if (!p->started) std::fprintf(stderr, "CuptiProfiler::stopProfiling called while not profiling.\n");
    p->started = false;
    if (rc != 0) return fail(NVRX_ERR_STATE, "nvrx_profiler_stop: rocprofiler_stop_context failed");
    // bounded host memory: what the capture delivered so far moves to the device log here,
    // on the caller's thread, once a buffer's worth waits
    if ((int64_t)p->staged.size() >= p->drain_records) return flush_locked(p);
    return NVRX_OK;
}

int nvrx_profiler_reset(nvrx_profiler* p) {
    NVRX_CHECK_ARG(p, "nvrx_profiler_reset: null handle");
    CaptureSelf self(p);
    (void)nvrx::capture_flush();  // CuptiProfiler.cpp:149: flush, then clear (outside the lock)
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceGuard g(p->cfg.device);
    if (p->ingest_pending) {  // an ingest copy may still target the log
        (void)hipEventSynchronize(p->ingest_ev);
        p->ingest_pending = false;
    }
    // CuptiProfiler.cpp:148-152: clear every kernel's ring -- and forget the kernels, so
    // the slots are renumbered from 0 in the next interval
    p->staged.clear();
    p->log_n = 0;
    p->names.clear();
    p->name_to_slot.clear();
    p->key_to_slot.clear();
    p->saturated = 0;
    ++p->version;
    ++p->generation;  // slots handed out before this reset are void
    return NVRX_OK;
}

int nvrx_profiler_generation(nvrx_profiler* p, uint64_t* generation) {
    NVRX_CHECK_ARG(p && generation, "nvrx_profiler_generation: null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    *generation = p->generation;
    return NVRX_OK;
}

int nvrx_profiler_register_kernel(nvrx_profiler* p, const char* name, uint32_t* slot) {
    NVRX_CHECK_ARG(p && name && slot, "nvrx_profiler_register_kernel: null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    const size_t before = p->names.size();
    *slot = slot_of_name(p, name);
    if (p->names.size() != before) ++p->version;  // a cached get_stats result is stale
    return NVRX_OK;
}

int nvrx_profiler_push(nvrx_profiler* p, const nvrx_record* recs, int64_t n) {
    NVRX_CHECK_ARG(p && (n == 0 || recs) && n >= 0, "nvrx_profiler_push: bad arguments");
    std::lock_guard<std::mutex> lk(p->mu);
    if (!p->started) return NVRX_OK;  // activity disabled: records are not captured
    const uint32_t nslots = (uint32_t)p->names.size();
    for (int64_t i = 0; i < n; ++i)
        if (recs[i].slot >= nslots) return fail(NVRX_ERR_INVALID, "nvrx_profiler_push: unknown slot");
    for (int64_t i = 0; i < n; ++i) p->saturated += recs[i].ns >= NVRX_KEY_WIDE;
    p->staged.insert(p->staged.end(), recs, recs + n);
    ++p->version;
    if ((int64_t)p->staged.size() >= p->drain_records) return flush_locked(p);
    return NVRX_OK;
}

int nvrx_profiler_ingest(nvrx_profiler* p, const nvrx_record* dev_recs, int64_t n,
                         uint64_t generation, void* stream) {
    NVRX_CHECK_ARG(p && n >= 0 && (n == 0 || dev_recs), "nvrx_profiler_ingest: bad arguments");
    CaptureSelf self(p);  // the ingest copy is the library's own kernel, not the job's
    std::lock_guard<std::mutex> lk(p->mu);
    if (generation != p->generation)
        return fail(NVRX_ERR_STATE, "nvrx_profiler_ingest: slots of another generation (a reset "
                                    "renumbered them; register the kernels again)");
    if (!p->started || n == 0) return NVRX_OK;  // activity disabled: records are not captured
    DeviceGuard g(p->cfg.device);
    int rc = flush_locked(p);  // host records staged earlier come first (push order)
    if (rc) return rc;
    rc = grow_log(p, p->log_n + n);
    if (rc) return rc;
    // a copy that drops (slot := UINT32_MAX) records of slots not registered at this call
    hipError_t e = nvrx::records_ingest(p->d_log + p->log_n, dev_recs, n, (uint32_t)p->names.size(),
                                        S(stream));
    if (e == hipSuccess) e = hipEventRecord(p->ingest_ev, S(stream));
    if (e != hipSuccess) return hip_status(e, "nvrx_profiler_ingest");
    p->ingest_pending = true;
    p->log_n += n;
    ++p->version;
    return NVRX_OK;
}

int nvrx_profiler_saturated(nvrx_profiler* p, int64_t* count) {
    NVRX_CHECK_ARG(p && count, "nvrx_profiler_saturated: null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    *count = (int64_t)p->saturated;
    return NVRX_OK;
}

int nvrx_profiler_get_stats(nvrx_profiler* p, int64_t cap_out, int64_t* count, uint32_t* slots,
                            int32_t* num, float* mn, float* mx, float* med, float* avg, float* sd) {
    NVRX_CHECK_ARG(p && count && cap_out >= 0, "nvrx_profiler_get_stats: bad arguments");
    CaptureSelf self(p);  // the report's own kernels are not captured
    (void)nvrx::capture_flush();  // CuptiProfiler.cpp:138 cuptiActivityFlushAll (before the lock)
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceGuard g(p->cfg.device);
    int rc = flush_locked(p);
    if (rc) return rc;
    if (p->cache_version != p->version) {
        // recompute (a size query followed by the copy call reuses this result)
        for (auto* v : {&p->c_mn, &p->c_mx, &p->c_med, &p->c_avg, &p->c_sd}) v->clear();
        p->c_slot.clear();
        p->c_num.clear();
        const int64_t nslots = (int64_t)p->names.size();
        if (p->log_n > 0 && nslots > 0) {
            Work w;
            rc = bucket_log(p, nslots, 0, w);
            if (rc) return rc;
            nvrx_stats_soa soa{w.num, w.mn, w.mx, w.med, w.avg, w.sd};
            const int64_t cap = p->cfg.stats_max_len_per_kernel;
            hipError_t e = nvrx::segment_stats_ragged(w.ns, w.seg_off, w.seg_len, nslots,
                                                      std::min<int64_t>(cap, p->log_n), cap,
                                                      p->cfg.mode, true, soa, nullptr, 0, p->stream);
            if (e != hipSuccess) return hip_status(e, "nvrx_profiler_get_stats: segment_stats");
            // the six columns are consecutive in the carve (num, mn, mx, med, avg, sd, each
            // 256-B aligned): one copy into pinned staging, one synchronisation
            const size_t span = (size_t)((char*)(w.sd + nslots) - (char*)w.num);
            rc = ensure_small(p, span);
            if (rc) return rc;
            e = hipMemcpyAsync(p->h_small, w.num, span, hipMemcpyDeviceToHost, p->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
            if (e != hipSuccess) return hip_status(e, "nvrx_profiler_get_stats: download");
            const auto col = [&](const void* d) { return p->h_small + ((const char*)d - (const char*)w.num); };
            const int32_t* hnum = (const int32_t*)col(w.num);
            const float *hmn = (const float*)col(w.mn), *hmx = (const float*)col(w.mx),
                        *hmed = (const float*)col(w.med), *havg = (const float*)col(w.avg),
                        *hsd = (const float*)col(w.sd);
            // std::map order of getStats (CuptiProfiler.cpp:137-145): sorted by composite name
            for (int64_t s = 0; s < nslots; ++s)
                if (hnum[s] > 0) p->c_slot.push_back((uint32_t)s);
            std::sort(p->c_slot.begin(), p->c_slot.end(),
                      [&](uint32_t a, uint32_t b) { return p->names[a] < p->names[b]; });
            for (uint32_t s : p->c_slot) {
                p->c_num.push_back(hnum[s]);
                p->c_mn.push_back(hmn[s]);
                p->c_mx.push_back(hmx[s]);
                p->c_med.push_back(hmed[s]);
                p->c_avg.push_back(havg[s]);
                p->c_sd.push_back(hsd[s]);
            }
        }
        p->cache_version = p->version;
    }
    *count = (int64_t)p->c_slot.size();
    const int64_t m = std::min<int64_t>(cap_out, *count);
    for (int64_t i = 0; i < m; ++i) {
        if (slots) slots[i] = p->c_slot[i];
        if (num) num[i] = p->c_num[i];
        if (mn) mn[i] = p->c_mn[i];
        if (mx) mx[i] = p->c_mx[i];
        if (med) med[i] = p->c_med[i];
        if (avg) avg[i] = p->c_avg[i];
        if (sd) sd[i] = p->c_sd[i];
    }
    return NVRX_OK;
}

int nvrx_profiler_get_records(nvrx_profiler* p, int64_t cap_out, int64_t* count,
                              nvrx_record* out) {
    NVRX_CHECK_ARG(p && count && cap_out >= 0 && (cap_out == 0 || out),
                   "nvrx_profiler_get_records: bad arguments");
    CaptureSelf self(p);
    (void)nvrx::capture_flush();
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceGuard g(p->cfg.device);
    int rc = flush_locked(p);
    if (rc) return rc;
    *count = p->log_n;
    const int64_t m = std::min<int64_t>(cap_out, p->log_n);
    if (m == 0) return NVRX_OK;
    hipError_t e = hipMemcpyAsync(out, p->d_log, (size_t)m * sizeof(nvrx_record),
                                  hipMemcpyDeviceToHost, p->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    return hip_status(e, "nvrx_profiler_get_records: download");
}

int nvrx_profiler_kernel_name(nvrx_profiler* p, uint32_t slot, char* buf, int64_t buflen) {
    NVRX_CHECK_ARG(p && buf && buflen > 0, "nvrx_profiler_kernel_name: bad arguments");
    std::lock_guard<std::mutex> lk(p->mu);
    NVRX_CHECK_ARG(slot < p->names.size(), "nvrx_profiler_kernel_name: unknown slot");
    const std::string& s = p->names[slot];
    if ((int64_t)s.size() + 1 > buflen)
        return fail(NVRX_ERR_INVALID, "nvrx_profiler_kernel_name: buffer too small");
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return NVRX_OK;
}

}  // extern "C"
