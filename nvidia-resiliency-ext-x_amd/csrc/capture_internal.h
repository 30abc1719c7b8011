// capture_internal.h -- state shared by the live-capture translation units: capture.cpp (the
// rocprofiler-sdk tool, its kernel-dispatch tracing modes and the C ABI) and capture_queue.cpp
// (queue delivery: intercepted HSA queues and device completion records).  See capture.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
// the installed hsa_api_trace.h names its sibling headers "inc/..." unless built as part of the runtime
#define AMD_INTERNAL_BUILD
#include <hsa/hsa_api_trace.h>
#undef AMD_INTERNAL_BUILD
#include <hsa/amd_hsa_signal.h>
#include <rocprofiler-sdk/external_correlation.h>
#include <rocprofiler-sdk/intercept_table.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "nvrx_internal.h"


namespace nvrx {
namespace capture_detail {

constexpr int kEpochs = 1024;  // epoch slots: a slot is reused kEpochs flushes later
constexpr int kMarks = 16;     // threads that may run a report of their own at once

struct Capture {
    std::mutex mu;
    std::unordered_map<uint64_t, std::string> names;  // kernel_id -> kernel name
    rocprofiler_context_id_t sym_ctx{0};
    rocprofiler_context_id_t disp_ctx{0};
    rocprofiler_buffer_id_t buffer{0};
    std::atomic<bool> ready{false};      // tool_init completed
    std::atomic<bool> requested{false};  // nvrx_capture_configure succeeded
    std::atomic<nvrx_profiler*> target{nullptr};
    std::atomic<int> inflight{0};        // delivery callbacks running (detach waits for 0)
    // cost accounting (nvrx_capture_stats): callbacks, headers, dispatch records handed to the
    // profiler, time inside our callback, flushes and their wall time
    std::atomic<uint64_t> n_cb{0}, n_rec{0}, n_pushed{0}, cb_ns{0}, n_flush{0}, flush_ns{0};
    // where a report-time flush's time goes: steady-clock ns of the flush in progress (0: none),
    // and per flush the time to the first delivery callback it saw, the callbacks it saw, and
    // the time from the end of its last callback to its return
    std::atomic<int64_t> flush_t0{0}, last_cb_end{0};
    std::atomic<uint64_t> flush_first_cb_ns{0}, flush_cbs{0}, flush_tail_ns{0};
    // delivery (NVRX_CAPTURE_DELIVERY): 3 = queue, the default (HSA intercept queues and device
    // completion records, no rocprofiler-sdk dispatch tracing; "Queue delivery" below); the
    // rocprofiler-sdk KERNEL_DISPATCH modes: 1 = callback (each completed dispatch handed over as
    // the runtime processes its completion), 0 = buffer (records batched by rocprofiler-sdk; a
    // flush also flushes the buffer, ~3.4-5 ms whenever records are pending), 2 = callback_counted
    // (1 + ENQUEUE callbacks on the launching thread, which count the dispatches when the marking
    // service below is off; kept for cost attribution).
    int delivery = 3;
    std::atomic<uint64_t> n_enqueued{0}, n_completed{0};
    // callback delivery runs on the runtime's completion (signal-handler) thread, which must never
    // wait for the profiler's lock: the caller's thread may hold it across a HIP call that needs
    // that very thread (a deadlock, seen at stop()'s drain).  Completed dispatches are therefore
    // queued under a lock held only for the append, and moved into the profiler by the caller's
    // thread (capture_drain: at every flush and stop).
    std::mutex qmu;
    std::vector<nvrx::DispatchRec> queue;
    std::atomic<uint64_t> n_runtime{0};  // runtime copy / fill dispatches left out (below)
    bool keep_runtime = false;           // NVRX_CAPTURE_RUNTIME_KERNELS=1 keeps them
    // the external-correlation-id request service (NVRX_CAPTURE_MARKING=0 turns it off, for cost
    // attribution): marks the library's own report kernels (left out) and counts job dispatches
    bool marking = false;
    std::atomic<uint64_t> n_own{0};
    std::atomic<int> n_marked{0};                  // threads currently marked
    std::atomic<uint64_t> marks[kMarks] = {};      // their rocprofiler thread ids (0: free)
    // flush epochs (see the top of the file); only a flush advances `epoch`, under flush_mu
    std::atomic<uint64_t> epoch{1};
    std::atomic<int64_t> owed[kEpochs] = {};
    std::mutex flush_mu;
    uint64_t settled = 1;  // lowest epoch that may still be owed (flush_mu)
    int64_t flush_timeout_ms = 1000;
    std::atomic<uint64_t> n_requested{0}, n_counted_flush{0}, n_quiet_flush{0}, n_timeouts{0},
        n_abandoned{0};
    // queue delivery (3, see "Queue delivery" below): every kernel dispatch packet of an
    // intercepted queue gets a completion signal of ours while started; pending = dispatches not
    // harvested yet (enqueue order), pool = free signals (value 1); both under pmu
    struct Pending {
        hsa_signal_t sig;   // a pool signal, or the address of a ring record (slot >= 0)
        const void* queue;  // its QueueInfo
        uint64_t obj;       // kernel_object of the packet
        uint32_t bx, by, bz, gx, gy, gz;
        int64_t slot;       // ring slot, -1: pool signal
        uint64_t seq;       // ring hand-out number (slot = seq % ring_n)
        int64_t want;       // the ring record's value once this dispatch has completed
    };
    std::mutex pmu;
    std::vector<Pending> pending;
    std::vector<hsa_signal_t> pool;
    // bounds: at most max_pending dispatches wait for a harvest (NVRX_CAPTURE_MAX_PENDING,
    // default 2^20); past it a dispatch goes out without a completion record and counts as dropped,
    // as the CUPTI buffer pool drops records when every buffer is in use (BufferPool.cpp:44-52).
    // The pool holds at most kPoolMax signals; a harvest destroys free ones above kPoolKeep.
    static constexpr size_t kPoolMax = 65536, kPoolKeep = 1024;
    size_t max_pending = (size_t)1 << 20;
    size_t pool_total = 0;  // signals created and not destroyed (pmu)
    std::atomic<uint64_t> n_dropped{0};
    std::atomic<bool> qactive{false};     // the profiler is started
    std::atomic<bool> q_installed{false}; // hsa_queue_create is ours
    std::atomic<uint64_t> n_queues{0}, n_signals{0}, n_signal_fail{0}, n_chained{0};
    std::atomic<bool> q_table_incomplete{false};  // the HSA table lacked an entry: no queue delivery
    double tick_ns = 0.0;                 // ns per HSA system timestamp tick (first harvest; ring_copy_mu)
    // NVRX_CAPTURE_QUEUE_DIAG (cost attribution only; outputs wrong): 1 = intercept, no signals;
    // 2 = signals on queues without profiling (no timestamps)
    int qdiag = 0;
    // raw timestamps: the CP's start_ts / end_ts read from the signal itself (amd_signal_t) in GPU
    // ticks, checked against hsa_amd_profiling_get_dispatch_time on the first harvest (-1: not yet;
    // ring_copy_mu)
    int raw_ok = -1;
    // the ring of completion records in device memory (queue delivery, "Completion records" below):
    // ring_val = the value each record holds once its last hand-out has completed (host, pmu)
    amd_signal_t* ring = nullptr;
    int64_t ring_n = 0;
    int64_t ring_pci = -2;  // the ring's device (QueueInfo::pci): only its queues take ring records
    std::vector<int64_t> ring_val;
    std::vector<uint8_t> ring_busy;
    std::vector<uint64_t> ring_last_end;  // end_ts of each record's last harvested hand-out
    uint64_t ring_next = 0;
    amd_signal_t* ring_host = nullptr;  // pinned mirror the harvest copies into
    hipStream_t ring_stream = nullptr;
    bool ring_tried = false;
    std::mutex ring_copy_mu;            // one harvest copy at a time
    std::atomic<uint64_t> n_ring{0}, n_ring_full{0}, n_ring_bad{0}, n_ring_torn{0};
    rocprofiler_client_id_t* client = nullptr;
};

inline Capture& cap() {  // one instance per process (an inline function's static)
    static Capture c;
    return c;
}

// the calling thread's marking (capture_self_begin / _end nest on one thread)
struct SelfMark {
    int depth = 0;
    int slot = -1;
};
extern thread_local SelfMark t_mark;

int64_t env_int(const char* name, int64_t dflt);  // an integer environment setting


// capture.cpp: kernel names and records
bool runtime_blit(uint64_t kernel_id);
std::string composite_name(const nvrx::DispatchKey& k);
enum class Kind { job, own, runtime };
Kind to_dispatch(const rocprofiler_kernel_dispatch_info_t& di, uint64_t start, uint64_t end,
                 uint64_t external, nvrx::DispatchRec& d);

// capture_queue.cpp: queue delivery
void hsa_table_cb(rocprofiler_intercept_table_t type, uint64_t, uint64_t, void** tables, uint64_t num,
                  void*);
void ring_setup();                 // on a caller's thread (HIP calls allowed), before the first hand-out
void q_harvest(nvrx_profiler* p);  // the completed pending dispatches into p

}  // namespace capture_detail
}  // namespace nvrx
