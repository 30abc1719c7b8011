// capture_queue.cpp -- queue delivery of the live capture (the default; see capture.cpp): the HSA
// queues of the runtime intercepted through rocprofiler-sdk's intercept-table service, a device
// completion record per kernel dispatch, and the harvest of the completed ones.
#include "capture_internal.h"

namespace nvrx {
namespace capture_detail {

// ------------------------------------------------------------------------------- queue delivery
// NVRX_CAPTURE_DELIVERY=queue (the default): no rocprofiler-sdk dispatch tracing at all.  Through
// rocprofiler-sdk's intercept-table service the library takes hsa_queue_create: every queue the
// HIP runtime creates is an HSA intercept queue with profiling enabled, and while the profiler is
// started each kernel dispatch packet (on a thread that is not running a report of ours) gets a
// completion record -- a record of the device ring ("Completion records" below), or a pooled HSA
// signal when the ring is full or the queue belongs to another device -- into which the packet
// processor writes the kernel's start / end timestamps and then decrements it.  Nothing runs per
// completion: a flush (and stop) harvests, in enqueue order, every pending dispatch whose record
// shows it completed -- exactly the kernels that completed, as cuptiActivityFlushAll(0) delivers
// them (CuptiProfiler.cpp:138) -- and frees the record.  A packet that carried a completion signal
// of its own keeps it through a barrier-AND packet right behind it (barrier bit set: it completes
// once the kernel has, and signals the original).
struct QueueFns {
    decltype(hsa_queue_create)* queue_create = nullptr;
    decltype(hsa_amd_queue_intercept_create)* icreate = nullptr;
    decltype(hsa_amd_queue_intercept_register)* iregister = nullptr;
    decltype(hsa_amd_profiling_set_profiler_enabled)* prof_enable = nullptr;
    decltype(hsa_amd_profiling_get_dispatch_time)* dispatch_time = nullptr;
    decltype(hsa_amd_signal_create)* signal_create = nullptr;
    decltype(hsa_signal_destroy)* signal_destroy = nullptr;
    decltype(hsa_signal_load_scacquire)* load = nullptr;
    decltype(hsa_signal_store_relaxed)* store = nullptr;
    decltype(hsa_system_get_info)* sys_info = nullptr;
    decltype(hsa_agent_get_info)* agent_info = nullptr;
};
QueueFns qf;

struct QueueInfo {
    hsa_agent_t agent;
    double ns_per_tick;  // the agent's timestamp counter (HSA_AMD_AGENT_INFO_TIMESTAMP_FREQUENCY)
    int64_t pci;         // (PCI domain, bus, device) of the agent; -1 unknown
};

constexpr uint16_t packet_type(uint16_t header) {
    return (uint16_t)((header >> HSA_PACKET_HEADER_TYPE) & ((1u << HSA_PACKET_HEADER_WIDTH_TYPE) - 1));
}

// runs on the thread that rings the queue's doorbell (the launching thread under HIP's direct
// dispatch), for every batch of packets written to an intercepted queue
void q_intercept(const void* pkts, uint64_t n, uint64_t, void* data,
                 hsa_amd_queue_intercept_packet_writer writer) {
    Capture& c = cap();
    if (!c.qactive.load(std::memory_order_acquire)) {
        writer(pkts, n);
        return;
    }
    const auto* in = static_cast<const hsa_kernel_dispatch_packet_t*>(pkts);
    uint64_t nk = 0;
    for (uint64_t i = 0; i < n; ++i) nk += packet_type(in[i].header) == HSA_PACKET_TYPE_KERNEL_DISPATCH;
    // t_mark: a report of ours runs on this thread -- not captured.  This needs the handler on the
    // launching thread: HIP's direct dispatch (AMD_DIRECT_DISPATCH=0 selects callback delivery at
    // configuration, capture.cpp) and a queue with room for the packets -- ROCr defers the handler
    // of a batch that does not fit the wrapped queue.  The Detector synchronizes before it reports
    // (straggler.py:234-235 in the reference), so its report kernels meet drained queues.
    if (nk == 0 || t_mark.depth > 0) {
        if (t_mark.depth > 0) c.n_own.fetch_add(nk, std::memory_order_relaxed);
        writer(pkts, n);
        return;
    }
    if (c.qdiag == 1) {  // diagnostic: the interception alone
        c.n_requested.fetch_add(nk, std::memory_order_relaxed);
        writer(pkts, n);
        return;
    }
    thread_local std::vector<hsa_signal_t> sigs;
    sigs.assign(nk, hsa_signal_t{0});
    {
        std::lock_guard<std::mutex> lk(c.pmu);
        uint64_t j = 0;
        for (uint64_t i = 0; i < n; ++i) {
            if (packet_type(in[i].header) != HSA_PACKET_TYPE_KERNEL_DISPATCH) continue;
            if (c.pending.size() >= c.max_pending) {
                // started for long without a stop or flush: dropped, not held (bounded memory, and
                // no harvest walk over an unbounded list under pmu); the packet goes out as it came
                c.n_dropped.fetch_add(1, std::memory_order_relaxed);
                ++j;
                continue;
            }
            const hsa_kernel_dispatch_packet_t& k = in[i];
            Capture::Pending e{hsa_signal_t{0}, data, k.kernel_object, k.workgroup_size_x, k.workgroup_size_y,
                               k.workgroup_size_z, k.grid_size_x, k.grid_size_y, k.grid_size_z, -1, 0, 0};
            // a free record of the ring (a busy one -- a kernel still unharvested -- is skipped), for
            // a queue of the ring's own device (another GPU's packet processor may not map it)
            if (c.ring && static_cast<const QueueInfo*>(data)->pci == c.ring_pci) {
                for (int tries = 0; tries < 8 && e.slot < 0; ++tries) {
                    const uint64_t seq = c.ring_next++;
                    const int64_t s = (int64_t)(seq % (uint64_t)c.ring_n);
                    if (c.ring_busy[s]) continue;
                    c.ring_busy[s] = 1;
                    e.slot = s;
                    e.seq = seq;
                    e.want = --c.ring_val[s];
                    e.sig.handle = (uint64_t)(uintptr_t)(c.ring + s);
                }
                if (e.slot < 0) c.n_ring_full.fetch_add(1, std::memory_order_relaxed);
                else c.n_ring.fetch_add(1, std::memory_order_relaxed);
            }
            if (e.slot < 0) {  // an HSA signal of the pool
                if (c.pool.empty() && c.pool_total < Capture::kPoolMax) {  // grow (the pool keeps what reports returned)
                    for (int g = 0; g < 256; ++g) {
                        hsa_signal_t s{0};
                        if (qf.signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &s) != HSA_STATUS_SUCCESS) break;
                        c.pool.push_back(s);
                        ++c.pool_total;
                    }
                }
                if (c.pool.empty()) {
                    c.n_dropped.fetch_add(1, std::memory_order_relaxed);
                    ++j;  // no signal: the packet goes out as it came
                    continue;
                }
                e.sig = c.pool.back();
                c.pool.pop_back();
            }
            sigs[j++] = e.sig;
            c.pending.push_back(e);
        }
    }
    thread_local std::vector<hsa_kernel_dispatch_packet_t> out;  // 64-byte AQL slots
    out.clear();
    uint64_t j = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (packet_type(in[i].header) != HSA_PACKET_TYPE_KERNEL_DISPATCH || sigs[j].handle == 0) {
            if (packet_type(in[i].header) == HSA_PACKET_TYPE_KERNEL_DISPATCH) {
                ++j;
                c.n_signal_fail.fetch_add(1, std::memory_order_relaxed);
            }
            out.push_back(in[i]);
            continue;
        }
        hsa_kernel_dispatch_packet_t k = in[i];
        const hsa_signal_t orig = k.completion_signal;
        k.completion_signal = sigs[j++];
        out.push_back(k);
        if (orig.handle != 0) {  // the packet's own signal, behind it
            hsa_barrier_and_packet_t b{};
            const uint16_t release = (uint16_t)((k.header >> HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE) &
                                                ((1u << HSA_PACKET_HEADER_WIDTH_SCRELEASE_FENCE_SCOPE) - 1));
            b.header = (uint16_t)((HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) |
                                  (1u << HSA_PACKET_HEADER_BARRIER) |
                                  (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                  (release << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
            b.completion_signal = orig;
            hsa_kernel_dispatch_packet_t slot;
            static_assert(sizeof(slot) == sizeof(b), "AQL packets are 64 bytes");
            std::memcpy(&slot, &b, sizeof(b));
            out.push_back(slot);
            c.n_chained.fetch_add(1, std::memory_order_relaxed);
        }
    }
    uint64_t attached = 0;
    for (const auto& s : sigs) attached += s.handle != 0;
    c.n_signals.fetch_add(attached, std::memory_order_relaxed);
    c.n_requested.fetch_add(nk, std::memory_order_relaxed);
    writer(out.data(), out.size());
}

hsa_status_t q_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                      void (*callback)(hsa_status_t, hsa_queue_t*, void*), void* data,
                      uint32_t private_segment_size, uint32_t group_segment_size, hsa_queue_t** queue) {
    const hsa_status_t st = qf.icreate(agent, size, type, callback, data, private_segment_size,
                                       group_segment_size, queue);
    if (st != HSA_STATUS_SUCCESS)  // not interceptable: a plain queue, not captured
        return qf.queue_create(agent, size, type, callback, data, private_segment_size, group_segment_size,
                               queue);
    uint64_t freq = 0;
    (void)qf.agent_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_TIMESTAMP_FREQUENCY, &freq);
    uint32_t bdf = 0, dom = 0;
    const bool pci_ok = qf.agent_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS &&
                        qf.agent_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) == HSA_STATUS_SUCCESS;
    auto* qi = new QueueInfo{agent, freq ? 1e9 / (double)freq : 0.0,  // queues live as long as the process
                             pci_ok ? ((int64_t)dom << 16) | (int64_t)(bdf >> 3) : -1};
    if (qf.iregister(*queue, q_intercept, qi) != HSA_STATUS_SUCCESS ||
        (cap().qdiag != 2 && qf.prof_enable(*queue, 1) != HSA_STATUS_SUCCESS))
        std::fprintf(stderr, "nvrx capture: could not intercept an HSA queue; its kernels are not captured\n");
    cap().n_queues.fetch_add(1);
    return st;
}

// rocprofiler-sdk hands over the HSA API table as the runtime initialises
void hsa_table_cb(rocprofiler_intercept_table_t type, uint64_t, uint64_t, void** tables, uint64_t num,
                  void*) {
    if (type != ROCPROFILER_HSA_TABLE || num == 0 || !tables[0]) return;
    auto* t = static_cast<HsaApiTable*>(tables[0]);
    qf.queue_create = t->core_->hsa_queue_create_fn;
    qf.icreate = t->amd_ext_->hsa_amd_queue_intercept_create_fn;
    qf.iregister = t->amd_ext_->hsa_amd_queue_intercept_register_fn;
    qf.prof_enable = t->amd_ext_->hsa_amd_profiling_set_profiler_enabled_fn;
    qf.dispatch_time = t->amd_ext_->hsa_amd_profiling_get_dispatch_time_fn;
    qf.signal_create = t->amd_ext_->hsa_amd_signal_create_fn;
    qf.signal_destroy = t->core_->hsa_signal_destroy_fn;
    qf.load = t->core_->hsa_signal_load_scacquire_fn;
    qf.store = t->core_->hsa_signal_store_relaxed_fn;
    qf.sys_info = t->core_->hsa_system_get_info_fn;
    qf.agent_info = t->core_->hsa_agent_get_info_fn;
    if (!qf.queue_create || !qf.icreate || !qf.iregister || !qf.prof_enable || !qf.dispatch_time ||
        !qf.signal_create || !qf.signal_destroy || !qf.load || !qf.store || !qf.sys_info || !qf.agent_info) {
        // too late to fall back to rocprofiler-sdk dispatch tracing (its services are configured in
        // tool_init, before the runtime hands over this table): capture stays unavailable
        // (nvrx_profiler_capture_available() == 0) and says so
        cap().q_table_incomplete = true;
        std::fprintf(stderr, "nvrx capture: the HSA API table lacks an entry queue delivery needs; kernel "
                             "dispatches are NOT captured (NVRX_CAPTURE_DELIVERY=callback uses "
                             "rocprofiler-sdk tracing instead)\n");
        return;
    }
    cap().max_pending = (size_t)std::max<int64_t>(1024, env_int("NVRX_CAPTURE_MAX_PENDING", (int64_t)1 << 20));
    cap().qdiag = (int)env_int("NVRX_CAPTURE_QUEUE_DIAG", 0);
    t->core_->hsa_queue_create_fn = q_create;
    cap().q_installed = true;
}

// Completion records.  A completion signal in host memory costs every kernel ~1.2 us on the device
// (the packet processor's atomic on the signal crosses to host memory before the next packet of the
// queue may start: empty kernels 2.6 -> 4.0 us each, GPT-2 small +4.5 % per step,
// profiles/r05/capture_queue.json).  So the packets' completion "signals" are amd_signal_t records
// of a ring in fine-grained device memory (the CP decrements and timestamps them like any signal;
// no runtime object, no event mailbox, so no interrupt), each record's value counting down from
// 2^40 over its hand-outs: a dispatch has completed when its record holds the value the host
// expects after it (Pending::want).  A harvest copies the range of records still pending to a pinned
// mirror on a stream of its own (never waiting for the job's kernels) and reads them there.
constexpr int64_t RING_INIT = (int64_t)1 << 40;

void ring_setup() {  // on a caller's thread (HIP calls allowed), before the first hand-out
    Capture& c = cap();
    if (c.ring_tried) return;
    c.ring_tried = true;
    const int64_t n = env_int("NVRX_CAPTURE_RING", (int64_t)1 << 19);
    if (n <= 0) return;
    std::vector<amd_signal_t> h((size_t)n);
    std::memset(h.data(), 0, h.size() * sizeof(amd_signal_t));
    for (auto& s : h) {
        s.kind = AMD_SIGNAL_KIND_USER;
        s.value = RING_INIT;
    }
    int dev = 0, bus = 0, slot = 0, dom = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
        hipDeviceGetAttribute(&slot, hipDeviceAttributePciDeviceId, dev) != hipSuccess ||
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainId, dev) != hipSuccess)
        return;
    void* d = nullptr;
    void* m = nullptr;
    hipStream_t st = nullptr;
    const size_t bytes = (size_t)n * sizeof(amd_signal_t);
    if (hipExtMallocWithFlags(&d, bytes, hipDeviceMallocFinegrained) != hipSuccess ||
        hipHostMalloc(&m, bytes, hipHostMallocDefault) != hipSuccess ||
        hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
        hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
        std::fprintf(stderr, "nvrx capture: no device completion ring (%s); using HSA signals\n",
                     hipGetErrorString(hipGetLastError()));
        if (d) (void)hipFree(d);
        if (m) (void)hipHostFree(m);
        if (st) (void)hipStreamDestroy(st);
        return;
    }
    std::lock_guard<std::mutex> lk(c.pmu);
    c.ring_val.assign((size_t)n, RING_INIT);
    c.ring_busy.assign((size_t)n, 0);
    c.ring_last_end.assign((size_t)n, 0);
    c.ring_host = static_cast<amd_signal_t*>(m);
    c.ring_stream = st;
    c.ring_n = n;
    c.ring_pci = ((int64_t)dom << 16) | (int64_t)((bus << 5) | (slot & 31));
    c.ring = static_cast<amd_signal_t*>(d);
}

// ring records [seq_lo, seq_hi) -> the pinned mirror (slot-indexed), synchronously on the ring's stream
bool ring_copy(uint64_t seq_lo, uint64_t seq_hi) {
    Capture& c = cap();
    const uint64_t n = (uint64_t)c.ring_n;
    uint64_t cnt = std::min<uint64_t>(seq_hi - seq_lo, n);
    uint64_t s = seq_lo % n;
    hipError_t e = hipSuccess;
    while (cnt > 0 && e == hipSuccess) {
        const uint64_t m = std::min<uint64_t>(cnt, n - s);
        e = hipMemcpyAsync(c.ring_host + s, c.ring + s, m * sizeof(amd_signal_t), hipMemcpyDeviceToHost,
                           c.ring_stream);
        cnt -= m;
        s = 0;
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c.ring_stream);
    return e == hipSuccess;
}

// the completed pending dispatches, in enqueue order, into p (or dropped without one); pool signals
// go back to the pool, ring records become free
void q_harvest(nvrx_profiler* p) {
    Capture& c = cap();
    if (!c.q_installed) return;
    thread_local std::vector<Capture::Pending> done;
    thread_local std::vector<nvrx::DispatchRec> batch;
    thread_local std::vector<uint64_t> ring_ns;  // durations of the harvested ring records (done order)
    done.clear();
    batch.clear();
    ring_ns.clear();
    std::lock_guard<std::mutex> copy_lk(c.ring_copy_mu);  // the mirror is shared
    // A record copied while the packet processor was writing it could show the new value with a
    // timestamp of its previous hand-out (the copy engine reads the line in its own order): a
    // record counts as completed only with start_ts after that hand-out's end and end_ts >= start_ts;
    // one that shows the value but not yet the timestamps is read again (at most twice more).
    for (int attempt = 0; attempt < 3; ++attempt) {
        // the hand-out range of the ring records pending now
        bool any_ring = false;
        uint64_t lo = ~0ull, hi = 0;
        {
            std::lock_guard<std::mutex> lk(c.pmu);
            for (const auto& e : c.pending)
                if (e.slot >= 0) {
                    any_ring = true;
                    lo = std::min(lo, e.seq);
                    hi = std::max(hi, e.seq + 1);
                }
        }
        const bool copied = any_ring && ring_copy(lo, hi);
        uint64_t torn = 0;
        {
            std::lock_guard<std::mutex> lk(c.pmu);
            size_t w = 0;
            for (size_t i = 0; i < c.pending.size(); ++i) {
                const Capture::Pending& e = c.pending[i];
                bool complete = false;
                if (e.slot < 0) {
                    complete = attempt == 0 && qf.load(e.sig) == 0;
                } else if (copied && e.seq >= lo && e.seq < hi) {
                    const amd_signal_t& r = c.ring_host[e.slot];
                    if (r.value <= e.want) {
                        if (r.start_ts > c.ring_last_end[e.slot] && r.end_ts >= r.start_ts) {
                            complete = true;
                            if (r.value != e.want) c.n_ring_bad.fetch_add(1, std::memory_order_relaxed);
                            const double npt = static_cast<const QueueInfo*>(e.queue)->ns_per_tick;
                            ring_ns.push_back(npt > 0.0 ? (uint64_t)((double)(r.end_ts - r.start_ts) * npt + 0.5) : 0);
                            c.ring_last_end[e.slot] = r.end_ts;
                            c.ring_busy[e.slot] = 0;
                        } else {
                            ++torn;
                        }
                    }
                }
                if (complete)
                    done.push_back(e);
                else
                    c.pending[w++] = e;
            }
            c.pending.resize(w);
        }
        if (torn == 0) break;
        c.n_ring_torn.fetch_add(torn, std::memory_order_relaxed);
    }
    // (copy_lk is held to the end: it also guards tick_ns and raw_ok)
    if (done.empty()) return;
    if (c.tick_ns == 0.0) {
        uint64_t f = 0;
        c.tick_ns = qf.sys_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &f) == HSA_STATUS_SUCCESS && f
                        ? 1e9 / (double)f : 1.0;
    }
    // pool signals: the duration from the CP's raw timestamps (amd_signal_t, GPU ticks) --
    // hsa_amd_profiling_get_dispatch_time translates them to the system clock domain, ~0.1 us per
    // call; the first harvest checks that both give the same duration (to 1 %, >= 1 us)
    const auto raw_ns = [](const Capture::Pending& e) -> uint64_t {
        const auto* as = reinterpret_cast<const amd_signal_t*>(e.sig.handle);
        const double npt = static_cast<const QueueInfo*>(e.queue)->ns_per_tick;
        return as->end_ts > as->start_ts && npt > 0.0 ? (uint64_t)((double)(as->end_ts - as->start_ts) * npt + 0.5) : 0;
    };
    const auto api_ns = [&](const Capture::Pending& e) -> uint64_t {
        hsa_amd_profiling_dispatch_time_t tm{0, 0};
        (void)qf.dispatch_time(static_cast<const QueueInfo*>(e.queue)->agent, e.sig, &tm);
        return tm.end > tm.start ? (c.tick_ns == 1.0 ? tm.end - tm.start
                                                     : (uint64_t)((double)(tm.end - tm.start) * c.tick_ns + 0.5))
                                 : 0;
    };
    if (c.raw_ok < 0) {
        int agree = 0, total = 0;
        for (const auto& e : done) {
            if (e.slot >= 0) continue;
            const uint64_t a = api_ns(e), r = raw_ns(e);
            if (a < 1000) continue;
            ++total;
            agree += (r > a ? r - a : a - r) * 100 <= a;
        }
        if (total > 0) {
            c.raw_ok = agree == total ? 1 : 0;
            if (!c.raw_ok)
                std::fprintf(stderr, "nvrx capture: raw dispatch timestamps disagree with the HSA runtime's "
                                     "(%d of %d); using hsa_amd_profiling_get_dispatch_time\n", total - agree, total);
        }
    }
    uint64_t runtime = 0;
    size_t ri = 0;
    for (const auto& e : done) {
        rocprofiler_kernel_dispatch_info_t di{};
        di.kernel_id = e.obj;
        di.workgroup_size = {e.bx, e.by, e.bz};
        di.grid_size = {e.gx, e.gy, e.gz};
        const uint64_t ns = e.slot >= 0 ? ring_ns[ri++] : c.raw_ok == 1 ? raw_ns(e) : api_ns(e);
        nvrx::DispatchRec d;
        switch (to_dispatch(di, 0, ns, 0, d)) {
            case Kind::runtime: ++runtime; break;
            case Kind::job: batch.push_back(d); break;
            case Kind::own: break;
        }
    }
    {
        std::lock_guard<std::mutex> lk(c.pmu);
        for (const auto& e : done) {
            if (e.slot >= 0) continue;
            qf.store(e.sig, 1);
            c.pool.push_back(e.sig);
        }
        while (c.pool.size() > Capture::kPoolKeep) {  // a burst's signals back to the runtime
            (void)qf.signal_destroy(c.pool.back());
            c.pool.pop_back();
            --c.pool_total;
        }
    }
    c.n_cb.fetch_add(1);
    c.n_rec.fetch_add(done.size());
    c.n_completed.fetch_add(done.size(), std::memory_order_release);
    c.n_runtime.fetch_add(runtime);
    if (!p || batch.empty()) return;
    c.n_pushed.fetch_add(batch.size());
    nvrx::profiler_push_dispatches(p, batch.data(), batch.size(), composite_name);
}

}  // namespace capture_detail
}  // namespace nvrx
