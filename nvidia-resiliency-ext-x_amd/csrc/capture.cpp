// capture.cpp -- live kernel-dispatch capture (replaces the CUPTI activity path of
// nvrx_cupti_module: CuptiProfiler.cpp:96-203): the rocprofiler-sdk tool, its kernel-dispatch
// tracing modes and the C ABI; queue delivery lives in capture_queue.cpp, the shared state in
// capture_internal.h.
//
// The reference enables CUPTI_ACTIVITY_KIND_CONCURRENT_KERNEL, receives activity buffers on
// CUPTI's thread and, per record, builds the key "%s_blk_%d_%d_%d_grid_%d_%d_%d" (mangled
// kernel name, block dims, grid dims in blocks) and pushes (end - start) / 1000.0f into that
// key's ring.  Here a rocprofiler-sdk tool owns a "symbols" context (code-object callback tracing,
// kernel_id / kernel_object -> name, started at configuration) and one of two capture mechanisms:
//   * queue delivery (the default, "Queue delivery" below): through rocprofiler-sdk's
//     intercept-table service the library takes hsa_queue_create, so every HSA queue the HIP runtime
//     creates is an intercept queue; while the profiler is started each kernel dispatch packet gets
//     a completion record in device memory, whose start / end timestamps the packet processor
//     writes, and flushes harvest the records that completed -- nothing runs per dispatch but a
//     packet copy, nothing per completion at all (GPT-2 small, profiling_interval 1: +0.7 % per
//     training step, profiles/r05/capture_queue.json);
//   * the rocprofiler-sdk KERNEL_DISPATCH modes (NVRX_CAPTURE_DELIVERY=callback | buffer |
//     callback_counted): a "dispatch" context with callback (or buffer) tracing, plus the
//     external-correlation-id request service that marks the library's own report kernels and
//     counts every job dispatch at enqueue ("Flush completeness" below) -- ~5 us of
//     rocprofiler-sdk work per dispatch, +10 % per GPT-2 step.
// Each completed dispatch becomes the reference's key (workgroup size = block dims; grid_size is
// in work-items, so blocks = ceil(grid_size / workgroup_size)) and an integer-ns duration record
// for the profiler handle; the per-key rings and statistics are then the HIP kernels of the report
// path.
//
// Flush completeness (rocprofiler-sdk modes).  The reference's getStats calls
// cuptiActivityFlushAll(0) after the Detector's torch.cuda.synchronize() (CuptiProfiler.cpp:138,
// straggler.py:234-235): every kernel that completed is in the report.  rocprofiler-sdk hands a
// completion over on the runtime's signal-handler thread, some time after the device finished --
// long after it when the host is loaded.  So every job dispatch is counted at enqueue, in the
// external-correlation-id request rocprofiler-sdk makes on the launching thread (a callback that is
// on anyway for the marking, so the count is one atomic add), under the current flush EPOCH, which
// the request hands back as the dispatch's external correlation id.  Its completion subtracts it
// from that epoch once the record is queued.  A flush opens a new epoch and waits until no earlier
// epoch is owed anything: every dispatch enqueued before the flush has then been handed over,
// however late the runtime's thread ran.  A dispatch that is still running (enqueued by another
// thread after the caller's synchronize) is waited for up to NVRX_CAPTURE_FLUSH_TIMEOUT_MS (default
// 1000); then its epoch is given up, counted (flush_timeouts, owed_abandoned), and the record joins
// a later report.  (Queue delivery needs none of this: a flush reads the completion records
// themselves, which the device writes before the kernel counts as complete.)
//
// rocprofiler-sdk tools configure when the ROCm runtime initialises: nvrx_capture_configure
// must run before the process's first HIP call (the Python side does it at
// KernelProfiler(capture=True) construction and reports whether it took effect).
#include "capture_internal.h"

namespace nvrx {
namespace capture_detail {

thread_local SelfMark t_mark;

void code_object_cb(rocprofiler_callback_tracing_record_t record, rocprofiler_user_data_t*,
                    void*) {
    if (record.kind != ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT ||
        record.operation != ROCPROFILER_CODE_OBJECT_DEVICE_KERNEL_SYMBOL_REGISTER ||
        record.phase != ROCPROFILER_CALLBACK_PHASE_LOAD)
        return;
    auto* d = static_cast<rocprofiler_callback_tracing_code_object_kernel_symbol_register_data_t*>(
        record.payload);
    std::string n = d->kernel_name ? d->kernel_name : "";
    if (n.size() > 3 && n.compare(n.size() - 3, 3, ".kd") == 0) n.resize(n.size() - 3);
    std::lock_guard<std::mutex> lk(cap().mu);
    cap().names[d->kernel_object] = n;  // queue delivery keys dispatches by the packet's kernel_object
    cap().names[d->kernel_id] = std::move(n);
}

// External correlation ids of the dispatch context.  The reference's getStats runs on the host and
// adds no activity of its own; this library's report runs HIP kernels.  They are told apart from
// the job's by thread: while a report is in progress on thread T (T in `marks`), the request for a
// dispatch made on T gets SELF_MARK and the delivery drops that record.  Kernels other threads
// launch meanwhile keep being captured, as CUPTI keeps its activity enabled through getStats (a
// pause of the whole dispatch context would lose them).  Every other dispatch gets JOB_TAG | the
// current flush epoch, and is counted as owed in that epoch.
constexpr uint64_t SELF_MARK = 0x4E56525853454C46ull;  // "NVRXSELF"
constexpr uint64_t JOB_TAG = 0x4A4F42ull << 40;          // "JOB" | 40-bit epoch
constexpr uint64_t EPOCH_MASK = (1ull << 40) - 1;

bool marked_thread(uint64_t tid) {
    Capture& c = cap();
    if (c.n_marked.load(std::memory_order_acquire) == 0) return false;
    for (auto& m : c.marks)
        if (m.load(std::memory_order_relaxed) == tid) return true;
    return false;
}

int external_corr_request(rocprofiler_thread_id_t tid, rocprofiler_context_id_t,
                          rocprofiler_external_correlation_id_request_kind_t, rocprofiler_tracing_operation_t,
                          uint64_t, rocprofiler_user_data_t* value, void*) {
    Capture& c = cap();
    if (tid != 0 && marked_thread(tid)) {
        value->value = SELF_MARK;
        return 0;
    }
    const uint64_t e = c.epoch.load(std::memory_order_acquire);
    c.owed[e % kEpochs].fetch_add(1, std::memory_order_relaxed);
    c.n_requested.fetch_add(1, std::memory_order_relaxed);
    value->value = JOB_TAG | e;
    return 0;
}

// a delivered dispatch (job, runtime blit or, untagged, anything else) is no longer owed: called
// after its record is queued / pushed, so a flush that sees its epoch settled also drains it
void settle(uint64_t external) {
    if ((external & ~EPOCH_MASK) != JOB_TAG) return;
    Capture& c = cap();
    const uint64_t e = external & EPOCH_MASK;
    // an epoch given up long ago: its slot may already count a newer epoch
    if (c.epoch.load(std::memory_order_relaxed) - e >= kEpochs / 2) return;
    c.owed[e % kEpochs].fetch_sub(1, std::memory_order_release);
}

// The reference enables only CUPTI_ACTIVITY_KIND_CONCURRENT_KERNEL (CuptiProfiler.cpp:118) and
// keeps only those records (:179): memcpy and memset are other activity kinds and never reach the
// kernel summaries.  On ROCm, hipMemcpy*/hipMemset* (and torch's same-device copy_, which takes
// hipMemcpyAsync) are carried out by the runtime's own blit kernels, which rocprofiler-sdk reports
// as KERNEL_DISPATCH records like any other; their symbols carry the "__amd_rocclr_" prefix.
bool runtime_blit_name(const std::string& n) { return n.compare(0, 13, "__amd_rocclr_") == 0; }

// is kernel_id one of those blits?  The name is registered at code-object load, before any
// dispatch of it; each delivery thread caches the answer so the lock is taken once per kernel.
bool runtime_blit(uint64_t kernel_id) {
    thread_local std::unordered_map<uint64_t, bool> known;
    auto it = known.find(kernel_id);
    if (it != known.end()) return it->second;
    std::lock_guard<std::mutex> lk(cap().mu);
    auto nt = cap().names.find(kernel_id);
    if (nt == cap().names.end()) return false;  // not registered (yet): keep, do not cache
    return known[kernel_id] = runtime_blit_name(nt->second);
}

// CuptiProfiler.cpp:182-185: "%s_blk_%d_%d_%d_grid_%d_%d_%d" (only for a key the profiler
// has not seen since its last reset; known keys map to their slot without string work)
std::string composite_name(const nvrx::DispatchKey& k) {
    std::string name;
    {
        std::lock_guard<std::mutex> lk(cap().mu);
        auto it = cap().names.find(k.kernel_id);
        name = it != cap().names.end() ? it->second : std::string("unknown_kernel");
    }
    std::vector<char> buf(name.size() + 96);
    std::snprintf(buf.data(), buf.size(), "%s_blk_%d_%d_%d_grid_%d_%d_%d", name.c_str(), (int)k.bx,
                  (int)k.by, (int)k.bz, (int)k.gx, (int)k.gy, (int)k.gz);
    return std::string(buf.data());
}

// One completed dispatch -> the reference's record, or not the job's kernel (a report kernel of
// ours, or a runtime blit).
Kind to_dispatch(const rocprofiler_kernel_dispatch_info_t& di, uint64_t start, uint64_t end,
                 uint64_t external, nvrx::DispatchRec& d) {
    if (external == SELF_MARK) return Kind::own;  // a report kernel of ours
    if (!cap().keep_runtime && runtime_blit(di.kernel_id)) return Kind::runtime;
    // block dims = workgroup size; grid_size is in work-items, CUPTI's gridX..Z count blocks,
    // including a partial last block (a module / ext launch whose global size is not a multiple
    // of the workgroup): ceil
    const uint32_t bx = di.workgroup_size.x, by = di.workgroup_size.y, bz = di.workgroup_size.z;
    auto blocks = [](uint32_t g, uint32_t b) -> uint32_t {
        return b ? (uint32_t)(((uint64_t)g + b - 1) / b) : 0;
    };
    d.key = {di.kernel_id, bx, by, bz, blocks(di.grid_size.x, bx), blocks(di.grid_size.y, by),
             blocks(di.grid_size.z, bz)};
    d.ns = end > start ? end - start : 0;
    return Kind::job;
}

// a delivery callback's bookkeeping: in-flight count first, then the target (capture_detach
// clears the target and then waits for the count to drain, so a callback never touches a
// destroyed handle), and the flush accounting
struct CallbackScope {
    Capture& c;
    std::chrono::steady_clock::time_point t0;
    CallbackScope() : c(cap()) {
        c.inflight.fetch_add(1);
        t0 = std::chrono::steady_clock::now();
        if (const int64_t f0 = c.flush_t0.load()) {  // delivered by a flush in progress
            if (c.flush_cbs.fetch_add(1) == 0 || c.last_cb_end.load() < f0)  // its first callback
                c.flush_first_cb_ns.fetch_add((uint64_t)(t0.time_since_epoch().count() - f0));
        }
    }
    ~CallbackScope() {
        const auto t1 = std::chrono::steady_clock::now();
        c.cb_ns.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count());
        c.last_cb_end.store(t1.time_since_epoch().count());
        c.inflight.fetch_sub(1);
    }
};

// buffer delivery (NVRX_CAPTURE_DELIVERY=buffer): batches of records from rocprofiler-sdk's
// buffer, at its watermark or at a flush
void dispatch_buffer_cb(rocprofiler_context_id_t, rocprofiler_buffer_id_t,
                        rocprofiler_record_header_t** headers, size_t num_headers, void*,
                        uint64_t) {
    CallbackScope scope;
    Capture& c = scope.c;
    nvrx_profiler* p = c.target.load();
    thread_local std::vector<nvrx::DispatchRec> batch;
    thread_local std::vector<uint64_t> tags;
    batch.clear();
    tags.clear();
    uint64_t runtime = 0, own = 0;
    for (size_t i = 0; i < num_headers; ++i) {
        const rocprofiler_record_header_t* h = headers[i];
        if (h->category != ROCPROFILER_BUFFER_CATEGORY_TRACING ||
            h->kind != ROCPROFILER_BUFFER_TRACING_KERNEL_DISPATCH)
            continue;
        auto* r = static_cast<const rocprofiler_buffer_tracing_kernel_dispatch_record_t*>(h->payload);
        tags.push_back(r->correlation_id.external.value);
        if (!p) continue;
        nvrx::DispatchRec d;
        switch (to_dispatch(r->dispatch_info, r->start_timestamp, r->end_timestamp,
                            r->correlation_id.external.value, d)) {
            case Kind::own: ++own; break;
            case Kind::runtime: ++runtime; break;
            case Kind::job: batch.push_back(d); break;
        }
    }
    c.n_cb.fetch_add(1);
    c.n_rec.fetch_add(num_headers);
    c.n_pushed.fetch_add(batch.size());
    c.n_runtime.fetch_add(runtime);
    c.n_own.fetch_add(own);
    if (!batch.empty()) nvrx::profiler_push_dispatches(p, batch.data(), batch.size(), composite_name);
    for (uint64_t t : tags) settle(t);  // after the push: a settled epoch's records are in p
}

// callback delivery (NVRX_CAPTURE_DELIVERY=callback, the default): rocprofiler-sdk's
// KERNEL_DISPATCH callback tracing hands over each dispatch once the runtime has processed its
// completion signal -- no buffer to flush, only completions still being processed to wait for.
void dispatch_callback_cb(rocprofiler_callback_tracing_record_t record, rocprofiler_user_data_t*, void*) {
    Capture& c = cap();
    if (record.kind != ROCPROFILER_CALLBACK_TRACING_KERNEL_DISPATCH) return;
    if (record.operation == ROCPROFILER_KERNEL_DISPATCH_ENQUEUE) {
        if (record.phase == ROCPROFILER_CALLBACK_PHASE_EXIT) c.n_enqueued.fetch_add(1);
        return;
    }
    if (record.operation != ROCPROFILER_KERNEL_DISPATCH_COMPLETE) return;
    {
        CallbackScope scope;
        if (scope.c.target.load()) {  // queued for the attached profiler (capture_drain)
            auto* r = static_cast<const rocprofiler_callback_tracing_kernel_dispatch_data_t*>(record.payload);
            nvrx::DispatchRec d;
            switch (to_dispatch(r->dispatch_info, r->start_timestamp, r->end_timestamp,
                                record.correlation_id.external.value, d)) {
                case Kind::own: c.n_own.fetch_add(1); break;
                case Kind::runtime: c.n_runtime.fetch_add(1); break;
                case Kind::job: {
                    std::lock_guard<std::mutex> lk(c.qmu);
                    c.queue.push_back(d);
                    break;
                }
            }
            c.n_cb.fetch_add(1);
            c.n_rec.fetch_add(1);
        }
    }
    settle(record.correlation_id.external.value);                // after the record is queued
    c.n_completed.fetch_add(1, std::memory_order_release);  // (the unmarked fallback's count)
}

int64_t env_int(const char* name, int64_t dflt) {
    const char* v = std::getenv(name);
    if (!v || !*v) return dflt;
    char* end = nullptr;
    const long long x = std::strtoll(v, &end, 10);
    if (*end) {
        std::fprintf(stderr, "nvrx capture: %s=%s is not an integer, using %lld\n", name, v, (long long)dflt);
        return dflt;
    }
    return x;
}

int tool_init(rocprofiler_client_finalize_t, void*) {
    Capture& c = cap();
    if (rocprofiler_create_context(&c.sym_ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
    // NVRX_CAPTURE_SYMBOLS=0 (cost attribution only, tools/capture_cost.cpp): no code-object
    // tracing -- every key is then "unknown_kernel_..." and runtime blits are not recognised
    if (env_int("NVRX_CAPTURE_SYMBOLS", 1) != 0 &&
        rocprofiler_configure_callback_tracing_service(c.sym_ctx,
                                                       ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT,
                                                       nullptr, 0, code_object_cb,
                                                       nullptr) != ROCPROFILER_STATUS_SUCCESS)
        return -1;
    if (rocprofiler_create_context(&c.disp_ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
    c.keep_runtime = env_int("NVRX_CAPTURE_RUNTIME_KERNELS", 0) != 0;
    c.flush_timeout_ms = std::max<int64_t>(1, env_int("NVRX_CAPTURE_FLUSH_TIMEOUT_MS", 1000));
    if (c.delivery == 3) {  // queue delivery: no dispatch tracing service (hsa_table_cb does the work)
        if (rocprofiler_start_context(c.sym_ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
        c.ready = true;
        return 0;
    }
    if (env_int("NVRX_CAPTURE_MARKING", 1) != 0) {
        const rocprofiler_external_correlation_id_request_kind_t kinds[] = {
            ROCPROFILER_EXTERNAL_CORRELATION_REQUEST_KERNEL_DISPATCH};
        c.marking = rocprofiler_configure_external_correlation_id_request_service(
                        c.disp_ctx, kinds, 1, external_corr_request, nullptr) == ROCPROFILER_STATUS_SUCCESS;
    }
    if (c.delivery != 0) {
        const rocprofiler_tracing_operation_t complete_only[] = {ROCPROFILER_KERNEL_DISPATCH_COMPLETE};
        const rocprofiler_tracing_operation_t both[] = {ROCPROFILER_KERNEL_DISPATCH_ENQUEUE,
                                                        ROCPROFILER_KERNEL_DISPATCH_COMPLETE};
        if (rocprofiler_configure_callback_tracing_service(
                c.disp_ctx, ROCPROFILER_CALLBACK_TRACING_KERNEL_DISPATCH,
                c.delivery == 1 ? complete_only : both, c.delivery == 1 ? 1 : 2, dispatch_callback_cb,
                nullptr) != ROCPROFILER_STATUS_SUCCESS)
            return -1;
    } else {
        size_t watermark = 1u << 20;  // ~ the Detector's CUPTI bufferSize (1 MB, cupti.py:25)
        // NVRX_CAPTURE_WATERMARK overrides it, not below 64 KiB: with watermarks of a few KB
        // rocprofiler-sdk (ROCm 7.2) was measured to lose dispatch records (tools/diag_capture.py)
        watermark = (size_t)std::max<int64_t>(env_int("NVRX_CAPTURE_WATERMARK", (int64_t)watermark),
                                              (int64_t)64 << 10);
        if (rocprofiler_create_buffer(c.disp_ctx, 8u << 20, watermark, ROCPROFILER_BUFFER_POLICY_LOSSLESS,
                                      dispatch_buffer_cb, nullptr, &c.buffer) != ROCPROFILER_STATUS_SUCCESS)
            return -1;
        // a delivery thread of our own instead of rocprofiler-sdk's shared default: the report-time
        // flush drops from 5.0-5.5 to 3.5-4.4 ms (profiles/r03/capture_cost.json, capture_cbthread_ab.log)
        rocprofiler_callback_thread_t th{};
        if (rocprofiler_create_callback_thread(&th) == ROCPROFILER_STATUS_SUCCESS)
            (void)rocprofiler_assign_callback_thread(c.buffer, th);
        if (rocprofiler_configure_buffer_tracing_service(c.disp_ctx,
                                                         ROCPROFILER_BUFFER_TRACING_KERNEL_DISPATCH,
                                                         nullptr, 0, c.buffer) != ROCPROFILER_STATUS_SUCCESS)
            return -1;
    }
    if (rocprofiler_start_context(c.sym_ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
    c.ready = true;
    return 0;
}

void tool_fini(void*) {
    Capture& c = cap();
    if (!c.ready) return;
    if (c.delivery == 0) (void)rocprofiler_flush_buffer(c.buffer);
    c.ready = false;
}

// NVRX_CAPTURE_DELIVERY: queue (the default) | callback | callback_counted | buffer (anything else:
// a warning and the default)
int parse_delivery() {
    const char* m = std::getenv("NVRX_CAPTURE_DELIVERY");
    if (!m || !*m) return 3;
    const std::string v(m);
    if (v == "buffer") return 0;
    if (v == "callback") return 1;
    if (v == "callback_counted") return 2;
    if (v == "queue") return 3;
    std::fprintf(stderr, "nvrx capture: NVRX_CAPTURE_DELIVERY=%s is not queue | callback | "
                         "callback_counted | buffer; using queue\n", m);
    return 3;
}

rocprofiler_tool_configure_result_t* nvrx_tool_configure(uint32_t, const char*, uint32_t,
                                                         rocprofiler_client_id_t* id) {
    id->name = "nvrx-straggler";
    cap().client = id;
    cap().delivery = parse_delivery();
    // queue delivery tells the library's own report kernels apart by the thread the intercept
    // handler runs on, which is the launching thread only under the HIP runtime's direct dispatch
    // (ADVICE r05): without it, rocprofiler-sdk's dispatch tracing (callback delivery) is used
    if (cap().delivery == 3) {
        const char* dd = std::getenv("AMD_DIRECT_DISPATCH");
        if (dd && std::string(dd) == "0") {
            std::fprintf(stderr, "nvrx capture: AMD_DIRECT_DISPATCH=0 (packets submitted off the launching "
                                 "thread); using callback delivery\n");
            cap().delivery = 1;
        }
    }
    if (cap().delivery == 3 &&
        rocprofiler_at_intercept_table_registration(hsa_table_cb, ROCPROFILER_HSA_TABLE, nullptr) !=
            ROCPROFILER_STATUS_SUCCESS) {
        std::fprintf(stderr, "nvrx capture: the HSA intercept table is not available; using callback delivery\n");
        cap().delivery = 1;
    }
    static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t),
                                                   &tool_init, &tool_fini, nullptr};
    return &cfg;
}

// a wait that spins (yielding) for the first 200 us -- the usual case after a synchronize -- and
// then sleeps in short steps, so a long wait does not take a core from the runtime's thread
struct Backoff {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void pause() const {
        if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200))
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    bool expired(int64_t ms) const {
        return std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(ms);
    }
};

// The counted flush: open a new epoch, then wait until no earlier one is owed anything (buffer
// delivery: flushing the buffer on every round, since its callback is what settles).  False on
// timeout, after giving the owed epochs up.
bool wait_owed(Capture& c) {
    std::lock_guard<std::mutex> lk(c.flush_mu);
    const uint64_t last = c.epoch.load(std::memory_order_relaxed);
    c.owed[(last + 1) % kEpochs].store(0, std::memory_order_relaxed);  // reused slot: kEpochs ago
    c.epoch.store(last + 1, std::memory_order_release);  // new enqueues count in the next epoch
    if (c.delivery == 0) (void)rocprofiler_flush_buffer(c.buffer);
    const Backoff b;
    for (uint64_t e = c.settled; e <= last; ++e) {
        while (c.owed[e % kEpochs].load(std::memory_order_acquire) > 0) {
            if (b.expired(c.flush_timeout_ms)) {
                int64_t lost = 0;
                for (uint64_t f = e; f <= last; ++f)
                    lost += std::max<int64_t>(0, c.owed[f % kEpochs].load());
                c.n_abandoned.fetch_add((uint64_t)lost);
                c.n_timeouts.fetch_add(1);
                c.settled = last + 1;
                return false;
            }
            b.pause();
            if (c.delivery == 0) (void)rocprofiler_flush_buffer(c.buffer);
        }
    }
    c.settled = last + 1;
    c.n_counted_flush.fetch_add(1);
    return true;
}

// Without the marking service nothing is counted at enqueue: callback_counted waits for the
// ENQUEUE callbacks' count, callback for a 200 us quiet period after the last completion
// (bounded; counted as quiet_flushes), buffer for rocprofiler_flush_buffer alone.
bool wait_uncounted(Capture& c) {
    c.n_quiet_flush.fetch_add(1);
    if (c.delivery == 0) return rocprofiler_flush_buffer(c.buffer) == ROCPROFILER_STATUS_SUCCESS;
    const Backoff b;
    if (c.delivery == 2) {
        const uint64_t want = c.n_enqueued.load();
        while (c.n_completed.load(std::memory_order_acquire) < want) {
            if (b.expired(c.flush_timeout_ms)) return false;
            b.pause();
        }
        return true;
    }
    using clk = std::chrono::steady_clock;
    uint64_t seen = c.n_completed.load(std::memory_order_acquire);
    auto quiet = clk::now();
    while (clk::now() - quiet < std::chrono::microseconds(200)) {
        if (b.expired(20)) break;
        const uint64_t now = c.n_completed.load(std::memory_order_acquire);
        if (now != seen) seen = now, quiet = clk::now();
        std::this_thread::yield();
    }
    return true;
}

}  // namespace capture_detail
}  // namespace nvrx

using namespace nvrx::capture_detail;

namespace nvrx {

bool capture_ready() { return cap().ready.load(); }

int capture_start(nvrx_profiler* p) {
    Capture& c = cap();
    if (!c.ready) return 0;
    c.target.store(p);
    if (c.delivery == 3) {
        ring_setup();  // once, on the first start (this thread may make HIP calls)
        // a profiler started again and again with no flush in between (a detection section per
        // step, reports rare) harvests here once half the ring waits, so the ring's records keep
        // being reused instead of the dispatches falling back to host-memory signals
        size_t waiting = 0;
        {
            std::lock_guard<std::mutex> lk(c.pmu);
            waiting = c.pending.size();
        }
        if (c.ring_n > 0 && waiting > (size_t)c.ring_n / 2) q_harvest(p);
        c.qactive.store(true, std::memory_order_release);
        return 0;
    }
    return rocprofiler_start_context(c.disp_ctx) == ROCPROFILER_STATUS_SUCCESS ? 0 : -1;
}

int capture_stop(nvrx_profiler* p) {
    Capture& c = cap();
    if (!c.ready) return 0;
    // no flush here: records of kernels enqueued while started are delivered later and still
    // counted, as CUPTI's are (their completions still arrive with the context stopped)
    (void)p;
    if (c.delivery == 3) {
        c.qactive.store(false, std::memory_order_release);
        return 0;
    }
    return rocprofiler_stop_context(c.disp_ctx) == ROCPROFILER_STATUS_SUCCESS ? 0 : -1;
}

void capture_drain(nvrx_profiler* p) {
    Capture& c = cap();
    if (c.delivery == 3) {  // what has completed, on this thread
        q_harvest(p);
        return;
    }
    if (c.delivery == 0 || !p) return;
    thread_local std::vector<nvrx::DispatchRec> batch;
    batch.clear();
    {
        std::lock_guard<std::mutex> lk(c.qmu);
        batch.swap(c.queue);
    }
    if (batch.empty()) return;
    c.n_pushed.fetch_add(batch.size());
    nvrx::profiler_push_dispatches(p, batch.data(), batch.size(), composite_name);
}

int capture_flush() {
    Capture& c = cap();
    if (!c.ready) return 0;
    struct Drain {  // whatever completed is moved into the attached profiler, on this thread
        ~Drain() { capture_drain(cap().target.load()); }
    } drain;
    const auto t0 = std::chrono::steady_clock::now();
    c.flush_t0.store(t0.time_since_epoch().count());
    // queue delivery: nothing to wait for -- the harvest (Drain) takes every dispatch whose
    // completion signal the device has written, and only those
    const bool ok = c.delivery == 3 ? (c.n_counted_flush.fetch_add(1), true)
                                    : c.marking ? wait_owed(c) : wait_uncounted(c);
    const auto t1 = std::chrono::steady_clock::now();
    const int64_t last = c.last_cb_end.load();
    if (last >= c.flush_t0.load()) c.flush_tail_ns.fetch_add((uint64_t)(t1.time_since_epoch().count() - last));
    c.flush_t0.store(0);
    c.n_flush.fetch_add(1);
    c.flush_ns.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count());
    return ok ? 0 : -1;
}

// Mark the calling thread's dispatches as the library's own until capture_self_end.  Each
// thread has a slot of its own, so reports on two threads (get_stats on one, an external tracer's
// ingest on another) never unmark each other.  False when marking is off or every slot is taken
// (the caller then pauses the dispatch context instead).
bool capture_self_begin() {
    Capture& c = cap();
    if (c.ready && c.delivery == 3) {  // the intercept handler reads the depth on the launching thread
        ++t_mark.depth;
        return true;
    }
    if (!c.ready || !c.marking) return false;
    if (t_mark.depth > 0) {
        ++t_mark.depth;
        return true;
    }
    rocprofiler_thread_id_t tid = 0;
    if (rocprofiler_get_thread_id(&tid) != ROCPROFILER_STATUS_SUCCESS || tid == 0) return false;
    for (int i = 0; i < kMarks; ++i) {
        uint64_t free = 0;
        if (c.marks[i].compare_exchange_strong(free, tid, std::memory_order_acq_rel)) {
            c.n_marked.fetch_add(1, std::memory_order_release);
            t_mark = {1, i};
            return true;
        }
    }
    return false;
}

void capture_self_end() {
    if (t_mark.depth == 0 || --t_mark.depth > 0 || t_mark.slot < 0) return;
    Capture& c = cap();
    c.marks[t_mark.slot].store(0, std::memory_order_release);
    c.n_marked.fetch_sub(1, std::memory_order_release);
    t_mark.slot = -1;
}

void capture_detach(nvrx_profiler* p) {
    Capture& c = cap();
    if (c.target.load() != p) return;
    if (c.ready) (void)capture_flush();  // deliver what is pending, to p
    nvrx_profiler* cur = p;
    if (c.target.compare_exchange_strong(cur, nullptr) && c.ready) {
        if (c.delivery == 3)
            c.qactive.store(false, std::memory_order_release);
        else
            (void)rocprofiler_stop_context(c.disp_ctx);
    }
    while (c.inflight.load() != 0) std::this_thread::yield();  // callbacks that loaded p
    capture_drain(p);  // what those callbacks queued is p's, not the next profiler's
}

}  // namespace nvrx

extern "C" {

int nvrx_capture_configure(void) {
    Capture& c = cap();
    if (c.requested || c.ready) return NVRX_OK;
    const rocprofiler_status_t st = rocprofiler_force_configure(&nvrx_tool_configure);
    if (st != ROCPROFILER_STATUS_SUCCESS) {
        nvrx::set_error(std::string("nvrx_capture_configure: rocprofiler_force_configure: ") +
                        rocprofiler_get_status_string(st) +
                        " (capture must be configured before the first HIP call)");
        return NVRX_ERR_RUNTIME;
    }
    c.requested = true;
    return NVRX_OK;
}

int nvrx_profiler_capture_available(void) {
    const Capture& c = cap();
    return c.ready.load() && (c.delivery != 3 || c.q_installed.load()) ? 1 : 0;
}

int nvrx_capture_stats(nvrx_capture_counters* out) {
    if (!out) {
        nvrx::set_error("nvrx_capture_stats: NULL output");
        return NVRX_ERR_INVALID;
    }
    Capture& c = cap();
    out->callbacks = (int64_t)c.n_cb.load();
    out->headers = (int64_t)c.n_rec.load();
    out->dispatches = (int64_t)c.n_pushed.load();
    out->callback_ns = (int64_t)c.cb_ns.load();
    out->flushes = (int64_t)c.n_flush.load();
    out->flush_ns = (int64_t)c.flush_ns.load();
    out->runtime_kernels = (int64_t)c.n_runtime.load();
    out->own_kernels = (int64_t)c.n_own.load();
    out->flush_first_cb_ns = (int64_t)c.flush_first_cb_ns.load();
    out->flush_callbacks = (int64_t)c.flush_cbs.load();
    out->flush_tail_ns = (int64_t)c.flush_tail_ns.load();
    out->enqueues_counted = (int64_t)c.n_requested.load();
    out->counted_flushes = (int64_t)c.n_counted_flush.load();
    out->quiet_flushes = (int64_t)c.n_quiet_flush.load();
    out->flush_timeouts = (int64_t)c.n_timeouts.load();
    out->owed_abandoned = (int64_t)c.n_abandoned.load();
    out->delivery = c.ready ? c.delivery : -1;
    out->marking = c.marking ? 1 : 0;
    out->queues = (int64_t)c.n_queues.load();
    out->ring_records = (int64_t)c.n_ring.load();
    out->pool_signals = (int64_t)(c.n_signals.load() - c.n_ring.load());
    out->chained_signals = (int64_t)c.n_chained.load();
    out->ring_anomalies = (int64_t)c.n_ring_bad.load();
    out->dropped = (int64_t)c.n_dropped.load();
    return NVRX_OK;
}

int nvrx_capture_flush(void) {
    if (nvrx::capture_flush() != 0) {
        nvrx::set_error("nvrx_capture_flush: timed out waiting for owed dispatch records "
                        "(NVRX_CAPTURE_FLUSH_TIMEOUT_MS); they join a later report");
        return NVRX_ERR_RUNTIME;
    }
    return NVRX_OK;
}

}  // extern "C"
