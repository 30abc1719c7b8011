/*
 * nvrx_straggler.h -- C ABI of the MI355X-native straggler-detection scoring path.
 *
 * Implemented by libnvrx_hip.so (hand-written HIP kernels for gfx950).  Every entry
 * point takes plain pointers and sizes; no torch types cross this boundary.  Device
 * pointers are caller-owned (e.g. torch tensors' data_ptr()); `stream` is a
 * hipStream_t (NULL = default stream).  Calls are stream-ordered and asynchronous,
 * except nvrx_sync, the nvrx_profiler_* lifecycle calls and functions documented as
 * "synchronous".  Nothing is retained after return except state owned by a
 * nvrx_profiler handle.
 *
 * Errors: every function returns NVRX_OK (0) or a negative NVRX_ERR_*; the message
 * of the last error on the calling thread is nvrx_last_error().  The Python layer
 * raises RuntimeError with that message, as the reference's CUPTI_CALL -> std::
 * runtime_error -> RuntimeError path does (cupti_src/CuptiProfiler.cpp:30-38).
 *
 * Reference interfaces replaced (paths relative to
 * /root/reference/src/nvidia_resiliency_ext/straggler):
 *   nvrx_segment_stats_*   computeStats + CuptiProfiler::getStats   cupti_src/CuptiProfiler.cpp:44-74, 136-146
 *   nvrx_kernel_ref        ReportGenerator._all_reduce_times (MIN over ranks, -1 => NaN)   reporting.py:255-296
 *   nvrx_pack_min_times    the [K+Nsec] float32 pack of _all_reduce_times                 reporting.py:269-279
 *   nvrx_scores            _update_local_min_times + _compute_gpu_perf_score              reporting.py:298-314, 219-253
 *   nvrx_finalize_scores   score = sum(s*w)/sum(w), NaN if no common kernel; optional
 *                          float32 rounding of _get_tensor_from_scores                    reporting.py:251-253, 338-361
 *   nvrx_section_scores    _compute_sections_perf_scores (+ section MIN reduce, history)  reporting.py:196-217, 255-314
 *   nvrx_stragglers        Report.identify_stragglers (score < threshold, strict)         reporting.py:84-151
 *   nvrx_section_stats     Detector._get_section_summaries (torch f64 stats)             straggler.py:171-197
 *   nvrx_profiler_*        nvrx_cupti_module.CuptiProfiler (ctor, initialize, shutdown,
 *                          start, stop, get_stats, reset)                                 cupti_src/cupti_module_py.cpp:33-54
 *   nvrx_records_*         CuptiProfiler::bufferCompleted record loop + CircularBuffer     cupti_src/CuptiProfiler.cpp:168-203, CircularBuffer.h:53-69
 */
#ifndef NVRX_STRAGGLER_H
#define NVRX_STRAGGLER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NVRX_ABI_VERSION 6

#define NVRX_OK 0
#define NVRX_ERR_INVALID -1   /* bad argument / shape */
#define NVRX_ERR_HIP -2       /* HIP runtime error */
#define NVRX_ERR_STATE -3     /* call not valid in the current state */
#define NVRX_ERR_SINGLETON -4 /* a second profiler instance (CuptiProfiler.cpp:86-87) */
#define NVRX_ERR_NOMEM -5
#define NVRX_ERR_RUNTIME -6 /* rocprofiler-sdk / runtime configuration refused */

/* statistics modes */
#define NVRX_STATS_FAST 0  /* NUM/MIN/MAX/MED bit-exact; AVG/STD exact mean/std rounded once to f32 */
#define NVRX_STATS_EXACT 1 /* every field bit-exact with computeStats (sequential f32 over sorted) */
/* flag OR-ed into the mode of nvrx_segment_stats_strided: col_ref already holds the initial
 * column reference (+inf bits | 0), e.g. re-initialised by the previous report's nvrx_scores
 * (nvrx_score_args.reset_col_ref), so the initialising launch is skipped */
#define NVRX_STATS_COLREF_READY 0x10

/* largest retained segment (statsMaxLenPerKernel) the kernels accept.  The reference's ring takes
 * any capacity (CuptiProfiler.h:49-51); rings of up to 32,768 samples are sorted on chip, longer
 * ones in device scratch (slower, same bits): 4 B per retained sample of every segment in flight,
 * up to 256 MiB per launch and, near 2^30, 4 GiB for one segment's workgroup.  Freed scratch above
 * 256 MiB returns to the driver at the next synchronisation.  Practical rings are <= 2^24 samples
 * (nvrx_profiler_create warns above that). */
#define NVRX_MAX_SEGMENT (1 << 30)

/* SoA output of the statistics kernels: one entry per segment (device pointers).
 * Units are microseconds as float32, like KernelStats (CuptiProfiler.h:39-45). */
typedef struct nvrx_stats_soa {
    int32_t* num;
    float* min;
    float* max;
    float* med;
    float* avg;
    float* std;
} nvrx_stats_soa;

/* Arguments of nvrx_scores: R score rows (ranks) x K kernel columns, row-major.
 * value_f64 selects the element type of med / avg / hist: 0 = float32 (statistics from
 * the segment kernels, exact in f64), 1 = float64 (summaries handed in through the
 * ReportGenerator API, whose MED/AVG are Python floats). */
typedef struct nvrx_score_args {
    int64_t R, K;
    int32_t value_f64;
    const int32_t* num;        /* [R][K] NUM; <= 0 means the kernel is absent on that rank */
    const void* med;           /* [R][K] MED (us), float or double */
    const void* avg;           /* [R][K] AVG (us), float or double */
    const uint8_t* col_valid;  /* [K] 0 = column filtered out ("ncclDev"), NULL = all valid */
    /* relative score reference (NULL = relative scores not computed) */
    const float* ref;          /* ref[ref_index ? ref_index[k] : k]; a value !(>= 0) (NaN, -1) = missing */
    const int32_t* ref_index;  /* [K] or NULL */
    const uint32_t* ref_missing; /* [K] or NULL: nonzero => reference missing (NaN) */
    /* individual score history (NULL = individual scores not computed); updated in place
     * to min(hist, MED) for every present kernel BEFORE scoring (reporting.py:469-474) */
    void* hist;                /* hist[r*hist_stride + (hist_index ? hist_index[k] : k)], float or double */
    const int32_t* hist_index; /* [K] or NULL */
    int64_t hist_stride;       /* per-row stride of hist; 0 => K */
    /* output: partial sums per row, 6 doubles (NULL allowed when finalizing in place):
     * {sum s*w (rel), sum w (rel), n (rel), sum s*w (ind), sum w (ind), n (ind)} */
    double* partials;          /* [R][6] */
    int32_t* err;              /* [1] device flags |= 1 when some MED == 0, |= 2 when a score's
                                  total weight is 0 (ZeroDivisionError) */
    /* optional in-kernel finalize (single shard), as nvrx_finalize_scores: any may be NULL */
    int32_t round_f32;
    double thr_rel, thr_ind;
    double* gpu_rel;
    double* gpu_ind;
    uint8_t* strag_rel;
    uint8_t* strag_ind;
    /* optional self-resetting epilogue, for reports replayed back to back (HIP graphs): with
     * `done` (2 u32 of device memory, zero before the first call) the error bits collect in
     * done[1] and the LAST workgroup to finish stores them to *err (no zeroing of *err needed
     * before the call), re-initialises reset_col_ref[0 : 2*reset_ncols] to the initial column
     * reference for the next report's statistics (NVRX_STATS_COLREF_READY) and zeroes done. */
    uint32_t* done;
    uint32_t* reset_col_ref;
    int64_t reset_ncols;
} nvrx_score_args;

/* ---------------------------------------------------------------- library */
const char* nvrx_last_error(void);
int nvrx_abi_version(void);
int nvrx_device_count(int* count);             /* synchronous */
int nvrx_sync(void* stream);                   /* synchronous: waits for `stream` */

/* ---------------------------------------------------------------- durations */
/* Every duration the library reads is a u32 DURATION KEY.  The reference keeps
 * (end - start) / 1000.0f (CuptiProfiler.cpp:187): the u64 ns difference rounded to f32, then
 * divided.  A key is the integer ns below NVRX_KEY_WIDE (3.76 s) and the f32 bits of f32(ns)
 * above it (0xE0000000 + bits(f32(ns)) - bits(f32(0xE0000000)), at most 0xF0200000), so it
 * keeps exactly what the reference keeps for any u64 duration, and keys order like the
 * durations.  nvrx_duration_key encodes one (host); a tracer feeding nvrx_profiler_ingest or a
 * matrix of durations of 3.76 s and more must encode them.  Below 3.76 s keys are plain ns.
 * Every u32 is read as a key: a RAW u32 ns of 3.76 s or more (never encoded) would be read as
 * the f32 bits of a far larger duration, so nvrx_encode_ns_u32 turns a device array of raw u32
 * ns into keys in place first.  u32 values above NVRX_KEY_MAX come from no u64 duration (they
 * decode beyond 2^64 ns, keeping the order). */
#define NVRX_KEY_WIDE 0xE0000000u
#define NVRX_KEY_WIDE_F32BITS 0x4F600000u /* bits of f32(0xE0000000) */
#define NVRX_KEY_MAX 0xF0200000u          /* key of f32(2^64 - 1) */
uint32_t nvrx_duration_key(uint64_t ns);
int nvrx_encode_ns_u32(uint32_t* ns, int64_t n, void* stream);

/* ---------------------------------------------------------------- statistics */
/* Segment s = ns[s*seg_stride + seg_begin : + seg_len] (uint32 duration keys); the
 * last min(seg_len, cap) samples are retained (cap <= 0: all).  out->* are [nseg].
 * col_ref (optional, [2*ncols] uint32): segments form a [nseg/ncols][ncols] rank x kernel
 * matrix; the call also produces the per-kernel relative reference of _all_reduce_times
 * (reporting.py:255-296): col_ref[c] = float bits of min over rows of MED, col_ref[ncols+c]
 * != 0 when some row has no sample of c (=> NaN).  Feed (float*)col_ref as nvrx_score_args
 * .ref and col_ref + ncols as .ref_missing. */
int nvrx_segment_stats_strided(const uint32_t* ns, int64_t nseg, int64_t seg_stride,
                               int64_t seg_begin, int64_t seg_len, int64_t cap, int32_t mode,
                               const nvrx_stats_soa* out, uint32_t* col_ref, int64_t ncols,
                               void* stream);
/* Segment s = ns[seg_off[s] : seg_off[s] + seg_len[s]] (device arrays; seg_len NULL:
 * seg_off has nseg+1 entries and segment s ends at seg_off[s+1]); max_len bounds every
 * segment length (host-known); aligned16 != 0 promises every retained run starts on a
 * 16-byte boundary; seg_len[s] < 0 skips segment s (outputs untouched).  col_ref / ncols:
 * as for the strided call (segment s is row s / ncols, column s % ncols).  Segments of <= 128 retained samples are bit-exact in every field in
 * both modes (one lane per segment, the reference's sequential f32 sums). */
int nvrx_segment_stats_ragged(const uint32_t* ns, const int64_t* seg_off, const int32_t* seg_len,
                              int64_t nseg, int64_t max_len, int64_t cap, int32_t mode,
                              int32_t aligned16, const nvrx_stats_soa* out, uint32_t* col_ref,
                              int64_t ncols, void* stream);

/* ---------------------------------------------------------------- scoring */
/* ref[k] = min over r of med[r][k] if num[r][k] > 0 for every r, else NaN.
 * scratch: >= 2*K uint32 of device memory. */
int nvrx_kernel_ref(const int32_t* num, const float* med, int64_t R, int64_t K, float* ref,
                    uint32_t* scratch, void* stream);
/* times[0:total] = -1; times[ids[i]] = float32(med[i]) for i < n: the float32 pack of
 * _all_reduce_times (kernel ids first, section ids offset by the kernel count). */
int nvrx_pack_min_times(const double* med, const int32_t* ids, int64_t n, float* times,
                        int64_t total, void* stream);
int nvrx_scores(const nvrx_score_args* args, void* stream);
/* partials: [nshards][R][6], combined in shard order 0..nshards-1.
 * score = n > 0 ? sum(s*w)/sum(w) : NaN; round_f32 != 0 rounds to float32 (the
 * gather_on_rank0 tensor); err |= 2 when n > 0 and sum(w) == 0.
 * Any output pointer may be NULL. strag_* = score < thr (strict; NaN never). */
int nvrx_finalize_scores(const double* partials, int64_t R, int64_t nshards, int32_t round_f32,
                         double thr_rel, double thr_ind, double* gpu_rel, double* gpu_ind,
                         uint8_t* strag_rel, uint8_t* strag_ind, int32_t* err, void* stream);
/* Sections, R rows x S sections: med [R][S] f64, present [R][S] u8.
 * rel: ref_s = min over rows of float32(med) when ref_in == NULL (every row must be
 *      present, else NaN; computed into ref_work [S]), or ref_in[ref_index ? ref_index[s] : s]
 *      (float32, !(>= 0) = missing => NaN score);
 * ind: hist[R][S] f64 updated to min(hist, med) first.
 * out_rel / out_ind [R][S] f64 (NaN where absent); round_f32 as above.  Either may be NULL;
 * err |= 1 when a present med == 0 (ZeroDivisionError). */
int nvrx_section_scores(const double* med, const uint8_t* present, int64_t R, int64_t S,
                        const float* ref_in, const int32_t* ref_index, float* ref_work,
                        double* hist, int32_t round_f32, double* out_rel, double* out_ind,
                        int32_t* err, void* stream);
int nvrx_stragglers(const double* score, int64_t n, double thr, uint8_t* mask, void* stream);
/* Statistics of section CPU timings (ms, float64): section s = vals[off[s] : off[s+1]]
 * (off: [nsec+1], device).  MIN, MAX, MED = lower median s[(n-1)/2] (torch.median),
 * AVG, STD = unbiased (NaN for n == 1), NUM -- Detector._get_section_summaries
 * (straggler.py:171-197).  max_len bounds every section's length (any length: sections
 * longer than 16384 timings are sorted in a device scratch buffer instead of LDS). */
int nvrx_section_stats(const double* vals, const int64_t* off, int64_t nsec, int64_t max_len,
                       int32_t* num, double* mn, double* mx, double* med, double* avg,
                       double* sd, void* stream);

/* ---------------------------------------------------------------- record streams */
/* A record is one kernel execution: the slot of its composite kernel name and its duration
 * key (end - start, CuptiProfiler.cpp:187; nvrx_duration_key above 3.76 s). */
typedef struct nvrx_record {
    uint32_t slot;
    uint32_t ns;
} nvrx_record;

/* Bucket nstreams push-ordered record streams (stream t = recs[rec_off[t] : rec_off[t+1]],
 * one per rank) by slot, keeping for every (stream, slot) only its LAST `cap` records
 * (CircularBuffer semantics; order inside a bucket is push order).  Outputs (device):
 *   seg_off [nstreams*nslots] int64, seg_len [nstreams*nslots] int32:
 *       bucket (t, s) = out_ns[seg_off[t*nslots+s] : + seg_len[t*nslots+s]]; every bucket
 *       starts 16-byte aligned, so it feeds nvrx_segment_stats_ragged(aligned16=1); where a
 *       stream's buckets lie inside its region is unspecified (slots with few records are
 *       laid out first and assembled in LDS)
 *   out_ns  [>= nvrx_records_bucket_capacity(n, nstreams, nslots)] uint32, 16-byte aligned
 *   counts  [nstreams*nslots] int32: total pushes per (stream, slot) on return */
int64_t nvrx_records_bucket_capacity(int64_t n, int64_t nstreams, int64_t nslots);
int nvrx_records_bucket(const nvrx_record* recs, const int64_t* rec_off, int64_t nstreams,
                        int64_t nslots, int64_t cap, int64_t* seg_off, int32_t* seg_len,
                        uint32_t* out_ns, int32_t* counts, void* stream);
/* The whole per-(stream, slot) statistics of record streams (ring retention +
 * CuptiProfiler::getStats for every stream): nvrx_records_bucket, then
 * nvrx_segment_stats_ragged(aligned16) over the buckets (runs of <= 128 samples bit-exact in
 * every field).  out->* are [nstreams*nslots]; max_len bounds every stream's length
 * (host-known); col_ref (optional, [2*nslots]) as for nvrx_segment_stats_strided (rows =
 * streams), produced by a column reduction; counts may be NULL here (the pushes per bucket are
 * then not written: 4 B per (stream, slot) less).  On return seg_len[g] < 0 marks a bucket of
 * -seg_len[g] records whose statistics the bucketing kernel computed itself; neither its
 * seg_off[g] nor its records in out_ns are written. */
int nvrx_records_stats(const nvrx_record* recs, const int64_t* rec_off, int64_t nstreams,
                       int64_t nslots, int64_t cap, int32_t mode, int64_t max_len, int64_t* seg_off,
                       int32_t* seg_len, uint32_t* out_ns, int32_t* counts,
                       const nvrx_stats_soa* out, uint32_t* col_ref, void* stream);
/* Slots one bucketing pass counts (its per-slot counters live in LDS).  Any nslots is accepted:
 * a larger slot table is bucketed in passes over ranges of this many slots, each re-reading the
 * streams (the reference's per-kernel map is unbounded, CuptiProfiler.cpp:189-198);
 * nvrx_records_bucket_capacity accounts for the passes' regions of out_ns. */
int64_t nvrx_records_max_slots(void);

/* ---------------------------------------------------------------- profiler handle */
/* Replacement of nvrx_cupti_module.CuptiProfiler: owns device-resident per-kernel
 * duration records; only one instance may exist (CuptiProfiler.cpp:83-90). */
typedef struct nvrx_profiler nvrx_profiler;

typedef struct nvrx_profiler_config {
    int64_t buffer_size;              /* bytes of host record buffer per flush (CUPTI bufferSize) */
    int64_t num_buffers;              /* CUPTI numBuffers (kept for API parity) */
    int64_t stats_max_len_per_kernel; /* ring capacity per kernel (statsMaxLenPerKernel) */
    int32_t device;                   /* HIP device ordinal */
    int32_t mode;                     /* NVRX_STATS_EXACT (default) or NVRX_STATS_FAST */
} nvrx_profiler_config;

int nvrx_profiler_create(const nvrx_profiler_config* cfg, nvrx_profiler** out);
int nvrx_profiler_destroy(nvrx_profiler* p);
int nvrx_profiler_initialize(nvrx_profiler* p);
int nvrx_profiler_shutdown(nvrx_profiler* p);
int nvrx_profiler_start(nvrx_profiler* p);
int nvrx_profiler_stop(nvrx_profiler* p);
int nvrx_profiler_reset(nvrx_profiler* p);
/* Register a composite kernel name ("%s_blk_%d_%d_%d_grid_%d_%d_%d") -> slot. */
int nvrx_profiler_register_kernel(nvrx_profiler* p, const char* name, uint32_t* slot);
/* Slots are valid until the next nvrx_profiler_reset, which forgets every kernel (the
 * reference clears its per-kernel map, CuptiProfiler.cpp:148-152): names are registered again
 * (from slot 0) in the next report interval. */
/* Append host records (push order).  Ignored while stopped (records are dropped).  Staged
 * host records move to the device log once buffer_size bytes of them wait (and at every
 * get_stats / get_records / reset). */
int nvrx_profiler_push(nvrx_profiler* p, const nvrx_record* recs, int64_t n);
/* Slot-numbering generation: bumped by every nvrx_profiler_reset (slots are renumbered from 0
 * after it).  A caller that builds device records from registered slots reads it after
 * registering and passes it to nvrx_profiler_ingest. */
int nvrx_profiler_generation(nvrx_profiler* p, uint64_t* generation);
/* Append n DEVICE records (push order, after every record staged before) to the device log:
 * one copy kernel enqueued on `stream`, so dev_recs must stay valid until that stream reaches
 * it; later profiler calls order themselves after it.  Ignored while stopped.  `generation`
 * must be the current nvrx_profiler_generation (NVRX_ERR_STATE otherwise: the slots were
 * numbered before a reset).  Records whose slot is not registered at this call are dropped
 * (never counted, even if that slot number is handed out later).  The copy is the library's
 * own kernel: a live capture leaves it out.  No
 * reference counterpart: the device-side entry of an external tracer (SURVEY 8(b)
 * nvrx_ingest_records). */
int nvrx_profiler_ingest(nvrx_profiler* p, const nvrx_record* dev_recs, int64_t n,
                         uint64_t generation, void* stream);
/* *count = captured / pushed durations of 3.76 s or more (stored as wide keys, nothing lost)
 * since the last reset: a diagnostic of hung or very long kernels. */
int nvrx_profiler_saturated(nvrx_profiler* p, int64_t* count);
/* Flush, then compute stats of every slot with >= 1 record.  Synchronous.
 * Returns the number of kernels in *count; fills up to `cap_out` entries of slots
 * (sorted by kernel name, as std::map in getStats) and host SoA outputs.  The result is
 * cached: a size query (cap_out = 0) followed by the copying call computes once, unless
 * records arrived in between. */
int nvrx_profiler_get_stats(nvrx_profiler* p, int64_t cap_out, int64_t* count, uint32_t* slots,
                            int32_t* num, float* mn, float* mx, float* med, float* avg,
                            float* sd);
int nvrx_profiler_kernel_name(nvrx_profiler* p, uint32_t slot, char* buf, int64_t buflen);
/* Flush, then copy the record log since the last reset ({slot, ns}, push order per slot;
 * after a compaction only the records the rings can still retain) into host `out`
 * (up to cap_out records; *count = log length).  Synchronous.  No reference counterpart:
 * it lets a caller (the live-capture parity check) recompute the statistics elsewhere. */
int nvrx_profiler_get_records(nvrx_profiler* p, int64_t cap_out, int64_t* count,
                              nvrx_record* out);
/* Live kernel-dispatch capture (CuptiProfiler.cpp:96-203).  nvrx_capture_configure registers
 * the library as a rocprofiler-sdk tool; it must run before the process's first HIP call
 * (NVRX_ERR_STATE otherwise).  Once the runtime has initialised, nvrx_profiler_capture_available()
 * returns 1 and every kernel enqueued while a profiler handle is started is pushed into it, once it
 * has completed, under the reference's composite key "%s_blk_%d_%d_%d_grid_%d_%d_%d" (mangled name,
 * block dims, grid dims in blocks, a partial last block counted) with its integer-ns duration;
 * nvrx_profiler_stop / _get_stats flush the capture first.  By default the runtime's HSA queues are
 * intercepted and each dispatch gets a completion record in device memory (NVRX_CAPTURE_DELIVERY=
 * queue); callback / buffer / callback_counted use rocprofiler-sdk's kernel-dispatch tracing.  As CUPTI_ACTIVITY_KIND_CONCURRENT_KERNEL does (CuptiProfiler.cpp:118,
 * 179), copies and fills are not kernels: the ROCm runtime's blit kernels ("__amd_rocclr_*",
 * which carry out hipMemcpy* / hipMemset*) are left out unless NVRX_CAPTURE_RUNTIME_KERNELS=1. */
int nvrx_capture_configure(void);
int nvrx_profiler_capture_available(void);
/* Deliver the dispatch records completed so far to the started / stopped profiler
 * (cuptiActivityFlushAll(0), CuptiProfiler.cpp:138).  Synchronous; no-op without capture. */
int nvrx_capture_flush(void);
/* Cost accounting of the live capture since configuration (process-wide, monotone): delivery
 * callbacks (queue delivery: harvests), records in them, dispatch records handed to a profiler,
 * wall time spent inside this library's delivery callbacks, and the number and wall time of
 * report-time flushes.  No reference counterpart (CUPTI's
 * cost is not exposed either); tools/capture_cost.cpp reads it.  runtime_kernels counts the runtime
 * blit dispatches left out (above), own_kernels the library's own report kernels left out: while
 * get_stats / get_records / reset / ingest run, the dispatches of the calling thread are marked
 * (a rocprofiler-sdk external correlation id) and not captured, while other threads' kernels
 * still are, as CUPTI keeps its activity enabled through getStats.  All zero without capture. */
typedef struct nvrx_capture_counters {
    int64_t callbacks, headers, dispatches, callback_ns, flushes, flush_ns, runtime_kernels,
        own_kernels;
    /* where the flushes' time goes: summed over flushes, the time from a flush's start to the
     * first buffer callback it delivered, the callbacks delivered during flushes, and the time
     * from a flush's last callback to its return */
    int64_t flush_first_cb_ns, flush_callbacks, flush_tail_ns;
    /* flush completeness (capture.cpp, top): job dispatches counted at enqueue (the external
     * correlation id request), flushes that waited for every counted dispatch enqueued before
     * them, flushes without that count (marking off: NVRX_CAPTURE_MARKING=0 or the service
     * refused; a 200 us quiet period / the ENQUEUE count / the buffer flush alone), counted
     * flushes that timed out (NVRX_CAPTURE_FLUSH_TIMEOUT_MS, default 1000: a kernel still running)
     * and the dispatches they gave up on (delivered to a later report).  delivery: 0 buffer,
     * 1 callback (default), 2 callback_counted, -1 capture not configured; marking: 1 when the
     * request service is on. */
    int64_t enqueues_counted, counted_flushes, quiet_flushes, flush_timeouts, owed_abandoned;
    int32_t delivery, marking;
    /* queue delivery (3): HSA queues intercepted, dispatches given a completion record of the
     * device ring, dispatches given a pooled HSA signal instead (ring full or absent), packets
     * whose own completion signal was chained behind them, and ring records found past their
     * expected value (0 unless the packet processor does not decrement by one) */
    int64_t queues, ring_records, pool_signals, chained_signals, ring_anomalies;
    /* (ABI 6) queue delivery: dispatches not captured because NVRX_CAPTURE_MAX_PENDING (default
     * 2^20) dispatches already waited for a harvest, or no completion signal was left -- a profiler
     * started for a very long time with no stop, get_stats or flush in between.  The reference's
     * CUPTI buffer pool drops records the same way when every buffer is in use (BufferPool.cpp:44-52);
     * at every start the library harvests once half the completion ring waits, so a started /
     * stopped profiler (a detection section per step) never reaches the bound. */
    int64_t dropped;
} nvrx_capture_counters;
int nvrx_capture_stats(nvrx_capture_counters* out);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* NVRX_STRAGGLER_H */
