// Live-capture cost microbenchmark (not part of the library): the host cost
// per kernel dispatch of an empty kernel, and the report-time flush latency, in one mode per
// process:
//   none     the rocprofiler-sdk tool never configured (nvrx_capture_configure not called)
//   stopped  configured, profiler handle created, never started
//   started  configured and started: every dispatch becomes a record in the handle
//   cycle    started for the dispatch loop, then stopped before the flush measurements (how
//            Detector.generate_report finds it: between detection sections)
// For "started" the library's own share is nvrx_capture_stats().callback_ns (time inside our
// delivery callback), so (started - callback) is rocprofiler-sdk's interception alone.  The
// services are toggled by the environment, one process per setting (tools/gpu_r05_cost.sh):
// NVRX_CAPTURE_DELIVERY (buffer | callback | callback_counted), NVRX_CAPTURE_MARKING=0 (no
// external-correlation-id request: no self-marking, no enqueue count), NVRX_CAPTURE_SYMBOLS=0
// (no code-object tracing).
// Build: hipcc --offload-arch=gfx950 -O2 tools/capture_cost.cpp -I include
//        -L nvidia-resiliency-ext-x_amd/nvidia_resiliency_ext/straggler -lnvrx_hip -Wl,-rpath,...
// Output: one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nvrx_straggler.h"

__global__ void empty_kernel(int* p) {
    if (p && threadIdx.x == 1024) p[0] = 1;  // never true: keeps the kernel from being folded
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const char* mode = argc > 1 ? argv[1] : "none";
    const int n = argc > 2 ? atoi(argv[2]) : 20000;
    const bool configure = strcmp(mode, "none") != 0;
    const bool start = strcmp(mode, "started") == 0 || strcmp(mode, "cycle") == 0;
    const bool cycle = strcmp(mode, "cycle") == 0;
    if (configure && nvrx_capture_configure() != NVRX_OK) {
        printf("{\"error\": \"configure: %s\"}\n", nvrx_last_error());
        return 1;
    }
    (void)hipFree(nullptr);  // runtime (and the tool) initialise here
    nvrx_profiler* p = nullptr;
    nvrx_profiler_config cfg{1 << 20, 8, 1024, 0, NVRX_STATS_EXACT};
    if (configure) {
        if (nvrx_profiler_create(&cfg, &p) != NVRX_OK || nvrx_profiler_initialize(p) != NVRX_OK) {
            printf("{\"error\": \"profiler: %s\"}\n", nvrx_last_error());
            return 1;
        }
        if (start) nvrx_profiler_start(p);
    }
    const int avail = nvrx_profiler_capture_available();
    // warm up, then the timed dispatch loop (host time per launch; the device drains after)
    for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0, nullptr);
    (void)hipDeviceSynchronize();
    nvrx_capture_counters c0{}, c1{};
    nvrx_capture_stats(&c0);
    const double t0 = now_us();
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0, nullptr);
    const double t1 = now_us();
    (void)hipDeviceSynchronize();
    const double t2 = now_us();
    double stop_us = 0;
    if (cycle) {
        const double s0 = now_us();
        nvrx_profiler_stop(p);
        stop_us = now_us() - s0;
    }
    nvrx_capture_stats(&c1);
    nvrx_capture_counters cf0{}, cf1{};
    nvrx_capture_stats(&cf0);
    // report-time flush latency against the records waiting (0, 100, 1000, 10000 dispatches)
    std::vector<double> flush_us;
    const int waits[] = {0, 100, 1000, 10000};
    for (int m : waits) {
        for (int i = 0; i < m; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0, nullptr);
        (void)hipDeviceSynchronize();
        const double f0 = now_us();
        nvrx_capture_flush();
        flush_us.push_back(now_us() - f0);
    }
    nvrx_capture_stats(&cf1);
    const double nf = (double)std::max<int64_t>(1, cf1.flushes - cf0.flushes);
    // the profiler's get_stats (flush + device bucketing + EXACT stats + download)
    double gs_us = 0, gs2_us = 0;
    int64_t kernels = 0;
    if (p) {  // the first call loads the library's kernels (code objects); the second is steady
        double g0 = now_us();
        nvrx_profiler_get_stats(p, 0, &kernels, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
        gs_us = now_us() - g0;
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0, nullptr);  // invalidate the cache
        (void)hipDeviceSynchronize();
        g0 = now_us();
        nvrx_profiler_get_stats(p, 0, &kernels, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
        gs2_us = now_us() - g0;
    }
    nvrx_capture_counters c2{};
    nvrx_capture_stats(&c2);
    printf("{\"mode\": \"%s\", \"capture_available\": %d, \"dispatches\": %d, "
           "\"launch_us_per_dispatch\": %.4f, \"drain_us_per_dispatch\": %.4f, "
           "\"records_delivered\": %lld, \"callback_us_per_record\": %.4f, "
           "\"flush_us\": {\"0\": %.1f, \"100\": %.1f, \"1000\": %.1f, \"10000\": %.1f}, "
           "\"get_stats_us_first\": %.1f, \"get_stats_us\": %.1f, \"stop_us\": %.1f, \"kernels\": %lld, "
           "\"flushes\": %lld, \"flush_ms_total\": %.3f, \"delivery\": \"%s\", "
           "\"flush_first_callback_us\": %.1f, \"flush_callbacks\": %.1f, \"flush_tail_us\": %.1f, "
           "\"marking\": %d, \"delivery_mode\": %d, \"symbols\": \"%s\", \"enqueues_counted\": %lld, "
           "\"counted_flushes\": %lld, \"quiet_flushes\": %lld, \"flush_timeouts\": %lld}\n",
           mode, avail, n, (t1 - t0) / n, (t2 - t0) / n, (long long)(c1.dispatches - c0.dispatches),
           c1.dispatches > c0.dispatches ? (c1.callback_ns - c0.callback_ns) * 1e-3 / (double)(c1.dispatches - c0.dispatches) : 0.0,
           flush_us[0], flush_us[1], flush_us[2], flush_us[3], gs_us, gs2_us, stop_us, (long long)kernels,
           (long long)c2.flushes, c2.flush_ns * 1e-6,
           getenv("NVRX_CAPTURE_DELIVERY") ? getenv("NVRX_CAPTURE_DELIVERY") : "callback",
           (cf1.flush_first_cb_ns - cf0.flush_first_cb_ns) * 1e-3 / nf,
           (cf1.flush_callbacks - cf0.flush_callbacks) / nf, (cf1.flush_tail_ns - cf0.flush_tail_ns) * 1e-3 / nf,
           (int)c2.marking, (int)c2.delivery, getenv("NVRX_CAPTURE_SYMBOLS") ? getenv("NVRX_CAPTURE_SYMBOLS") : "1",
           (long long)(c1.enqueues_counted - c0.enqueues_counted), (long long)c2.counted_flushes,
           (long long)c2.quiet_flushes, (long long)c2.flush_timeouts);
    if (p) nvrx_profiler_destroy(p);
    return 0;
}
