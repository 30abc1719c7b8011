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
//   n <= 8..128       one LANE per segment: the samples in registers, a sorting
//                     sorting network, then CuptiProfiler.cpp:53-71 statement by
//                     statement (sequential f32 sums) -- every field bit-exact
//   n <= 64*PL        one WAVE per segment (lean_core, segment_kernels.h), PL 4..128
//   longer / EXACT    one WORKGROUP per segment (exact_body)
//
// Classification is three small launches over the segment lengths (count per block,
// scan, scatter) into one id list ordered by class; every class kernel is persistent
// (grid = CUs x occupancy) and reads its [start, count) from device memory, so the
// host never waits for the class sizes.
#include <mutex>

#include "segment_ragged_kernels.h"

namespace nvrx {

// (nvrx_internal.h) scratch comes from a memory pool of the library's own per device,
// whose release threshold is capped: freed scratch up to NVRX_SCRATCH_KEEP_BYTES stays reserved for
// the next report; above it (the long-ring paths: up to 4 B per retained sample of the segments in
// flight) it is released at the next synchronisation instead of staying taken from the training job.
// The device's default pool -- PyTorch's hipMallocAsync allocator backend sets its threshold to keep
// everything -- is left as the job configured it.  Inside a stream capture the allocation is the
// graph's own node (hipMallocAsync: the graph memory pool).
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipError_t e = hipStreamIsCapturing(st, &cs); e != hipSuccess) return e;
    if (cs != hipStreamCaptureStatusNone) return hipMallocAsync(p, bytes, st);
    static std::once_flag once[64];
    static hipMemPool_t pools[64] = {};
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipMallocAsync(p, bytes, st);
    std::call_once(once[dev], [dev] {
        hipMemPoolProps props{};
        props.allocType = hipMemAllocationTypePinned;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        hipMemPool_t pool = nullptr;
        if (hipMemPoolCreate(&pool, &props) != hipSuccess) return;  // the default pool then
        uint64_t thr = NVRX_SCRATCH_KEEP_BYTES;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
        pools[dev] = pool;
    });
    return pools[dev] ? hipMallocFromPoolAsync(p, bytes, pools[dev], st) : hipMallocAsync(p, bytes, st);
}

using namespace ragged;

// The class kernels are dealt over the caller's stream and one side stream per device
// (configs[3]: 4.28 -> 4.15 ms; 3 / 4 streams were no faster).
#ifndef NVRX_RAGGED_STREAMS  // build-time tuning constant
#define NVRX_RAGGED_STREAMS 2
#endif
constexpr int RAGGED_STREAMS = NVRX_RAGGED_STREAMS;
struct Fork {
    hipStream_t s[RAGGED_STREAMS];  // s[0] unused: slot 0 is the caller's stream
    hipEvent_t fork, join[RAGGED_STREAMS];
};
// One caller at a time per process from fork to join (the caller holds `fork_mutex()`): the
// fork / join events and side streams are shared, and another thread's event record between
// this caller's record and wait would hand it the wrong dependency.
static std::mutex& fork_mutex() {
    static std::mutex mu;
    return mu;
}
// out = nullptr (every class on `st`) unless the side stream of st's device can take work:
// st must belong to the current device (the side stream is created there) and the side
// stream must not be inside a graph capture -- once forked into a capture it stays part of
// it until that capture ends, and another caller's eager work on it would be recorded into
// that graph.  A capturing `st` forks as usual (the capture follows the events), also into
// a side stream already joined to that same capture.
static hipError_t ragged_fork(hipStream_t st, Fork*& out) {
    out = nullptr;
    static Fork* forks[64] = {nullptr};
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipSuccess;
    if (st != nullptr) {
        hipDevice_t sdev = 0;
        if (hipError_t e = hipStreamGetDevice(st, &sdev); e != hipSuccess) return e;
        if ((int)sdev != dev) return hipSuccess;
    }
    if (!forks[dev]) {
        Fork* f = new Fork{};
        hipError_t e = hipEventCreateWithFlags(&f->fork, hipEventDisableTiming);
        for (int i = 1; i < RAGGED_STREAMS && e == hipSuccess; ++i) {
            e = hipStreamCreateWithFlags(&f->s[i], hipStreamNonBlocking);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&f->join[i], hipEventDisableTiming);
        }
        if (e != hipSuccess) return e;  // leaked on failure: a one-time setup
        forks[dev] = f;
    }
    Fork* f = forks[dev];
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    unsigned long long id_st = 0;
    if (hipError_t e = hipStreamGetCaptureInfo(st, &cst, &id_st); e != hipSuccess) return e;
    for (int i = 1; i < RAGGED_STREAMS; ++i) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        unsigned long long id = 0;
        if (hipError_t e = hipStreamGetCaptureInfo(f->s[i], &cs, &id); e != hipSuccess) return e;
        // busy in a capture other than st's own
        if (cs != hipStreamCaptureStatusNone && !(cst == hipStreamCaptureStatusActive && id == id_st))
            return hipSuccess;
    }
    if (hipError_t e = hipEventRecord(f->fork, st); e != hipSuccess) return e;
    for (int i = 1; i < RAGGED_STREAMS; ++i)
        if (hipError_t e = hipStreamWaitEvent(f->s[i], f->fork, 0); e != hipSuccess) return e;
    out = f;
    return hipSuccess;
}
static hipError_t ragged_join(hipStream_t st, Fork* f) {
    for (int i = 1; i < RAGGED_STREAMS; ++i) {
        if (hipError_t e = hipEventRecord(f->join[i], f->s[i]); e != hipSuccess) return e;
        if (hipError_t e = hipStreamWaitEvent(st, f->join[i], 0); e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t ragged_launch_classes(const RaggedSegs& segs, const uint32_t* cls_list, const uint32_t* cls,
                                 int64_t keep, bool aligned16, bool exact, const nvrx_stats_soa& out,
                                 hipStream_t st) {
    const uint32_t* list = cls_list;
    const int64_t need = aligned16 ? keep : keep + 3;
    // class kernels; classes that max_len rules out are not launched.  With side streams the
    // classes are dealt round robin over them in launch order (fork / join by events, which HIP
    // graph capture follows), so one class's tail and latency-bound waves overlap the next class.
    std::lock_guard<std::mutex> lock(fork_mutex());
    Fork* fk = nullptr;
    if (hipError_t e = ragged_fork(st, fk); e != hipSuccess) return e;
    int k = 0;
    const auto S = [&]() {
        const int i = fk ? k++ % RAGGED_STREAMS : 0;
        return i ? fk->s[i] : st;
    };
    const uint32_t* c = cls;
    // the launches: (kind, size); kind 0 lane<size>, 1 list<size>, 2 FULL<size / 64>, 3 workgroup
    struct L {
        int kind, n;
    };
    L lane[5], wave[6], big[2];
    int nl = 0, nw = 0, nb = 0;
    for (int n = 8; n <= 128; n *= 2)
        if (n == 8 || keep > n / 2) lane[nl++] = {0, n};
    if (!exact) {
        if (keep > 128) wave[nw++] = {1, 4};
        for (int pl = 8; pl <= 128; pl *= 2)
            if (need > 64 * (pl / 2)) wave[nw++] = {1, pl};
        if (const int fn = full_len(keep, aligned16, exact)) big[nb++] = {2, fn};  // the FULL class
    }
    if (exact ? keep > 128 : need > 64 * 128) big[nb++] = {3, 0};
    // order: the long-segment classes first, then the wave classes, then the lane classes (a FULL
    // kernel last ran alone behind the others; DESIGN 3.2, profiles/r05/class_order_ab.log)
#ifndef NVRX_CLASS_ORDER  // build-time tuning constant (timing A/B of the launch order)
#define NVRX_CLASS_ORDER 2
#endif
    L order[13];
    int no = 0;
    const auto put = [&](const L* a, int n, bool rev) {
        for (int i = 0; i < n; ++i) order[no++] = a[rev ? n - 1 - i : i];
    };
    switch (NVRX_CLASS_ORDER) {
        case 0: put(lane, nl, false); put(wave, nw, false); put(big, nb, false); break;
        case 1: put(big, nb, false); put(lane, nl, false); put(wave, nw, false); break;
        case 2: put(big, nb, false); put(wave, nw, false); put(lane, nl, false); break;
        case 3: put(big, nb, false); put(wave, nw, true); put(lane, nl, true); break;
        case 4: put(big, nb, false); put(lane, nl, true); put(wave, nw, true); break;
        case 6: put(big, nb, false); put(wave, nw, false); put(lane, nl, true); break;
        default: {  // 5: big first, then wave and lane classes interleaved, longest first
            put(big, nb, false);
            for (int i = 0; i < std::max(nl, nw); ++i) {
                if (i < nw) order[no++] = wave[nw - 1 - i];
                if (i < nl) order[no++] = lane[nl - 1 - i];
            }
        }
    }
    hipError_t e = hipSuccess;
    for (int i = 0; i < no && e == hipSuccess; ++i) {
        const L& o = order[i];
        switch (o.kind) {
            case 0: {
                const int cl = o.n == 8 ? C_T8 : o.n == 16 ? C_T16 : o.n == 32 ? C_T32 : o.n == 64 ? C_T64 : C_T128;
                ragged_launch_lane(o.n, segs, list, c + 2 * cl, aligned16, out, S());
                break;
            }
            case 1: {
                const int cl = o.n == 4 ? C_W4 : o.n == 8 ? C_W8 : o.n == 16 ? C_W16 : o.n == 32 ? C_W32
                             : o.n == 64 ? C_W64 : C_W128;
                ragged_launch_list(o.n, segs, list, c + 2 * cl, out, S());
                break;
            }
            case 2: ragged_launch_full(o.n / 64, segs, list, c + 2 * C_F, out, S()); break;
            default: e = ragged_launch_exact(segs, list, c + 2 * C_X, keep, out, S());
        }
    }
    if (e == hipSuccess) e = hipGetLastError();
    // joined on every path: a side stream left forked would leave a graph capture unjoined
    if (fk) {
        const hipError_t j = ragged_join(st, fk);
        if (e == hipSuccess) e = j;
    }
    return e;
}

hipError_t segment_stats_ragged(const uint32_t* ns, const int64_t* seg_off, const int32_t* seg_len,
                                int64_t nseg, int64_t max_len, int64_t cap, int mode,
                                bool aligned16, const nvrx_stats_soa& out, uint32_t* col_ref,
                                int64_t ncols, hipStream_t st) {
    // the column reference (MIN over rows of MED, missing flags) is a column reduction over the
    // finished statistics (kernel_ref), not per-segment atomics in the class kernels: the class
    // kernels then carry no column-reference state (fewer SGPRs, fewer spills)
    const auto colref = [&]() -> hipError_t {
        if (!col_ref || ncols <= 0) return hipSuccess;
        return kernel_ref(out.num, out.med, nseg > 0 ? nseg / ncols : 0, ncols, nullptr, col_ref, st);
    };
    if (nseg <= 0) return colref();
    RaggedSegs segs{ns, seg_off, seg_len, cap};
    const int64_t keep = (cap > 0 && max_len > cap) ? cap : max_len;
    if (keep > NVRX_MAX_SEGMENT) return hipErrorInvalidValue;
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

    // (a one-pass variant -- per-block totals reserving each class's range with global atomics,
    // lists of nseg entries per class -- measured 4.17 / 4.37 ms with 1024 / 256-thread blocks
    // against 4.13 for these three launches on configs[3]: the reservations contend on one
    // address per class)
    hipLaunchKernelGGL(classify_count_kernel, dim3((unsigned)nblocks), dim3(CLS_THREADS), 0, st, segs,
                       nseg, chunk, aligned16 ? 1 : 0, exact ? 1 : 0, full_len(keep, aligned16, exact), bcnt, out);
    hipLaunchKernelGGL(classify_scan_kernel, dim3(1), dim3(CLS_MAX_BLOCKS), 0, st, bcnt, (int)nblocks,
                       cls);
    hipLaunchKernelGGL(classify_scatter_kernel, dim3((unsigned)nblocks), dim3(CLS_THREADS), 0, st,
                       segs, nseg, chunk, aligned16 ? 1 : 0, exact ? 1 : 0, full_len(keep, aligned16, exact), bcnt, list);
    const hipError_t e = ragged_launch_classes(segs, list, cls, keep, aligned16, exact, out, st);
    const hipError_t f = hipFreeAsync(ws, st);  // on the error path too
    if (e != hipSuccess) return e;
    if (f != hipSuccess) return f;
    return colref();
}

}  // namespace nvrx
