// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/libnvrx_ref.so).
//
// Exposes the REFERENCE computeStats / CircularBuffer, compiled from the reference
// sources where they lie under /root/reference (nothing is copied into this repo),
// through a tiny extern "C" surface so tests/golden/make_golden.py can record
// known-answer vectors with ctypes.  The translation unit #includes the reference
// CuptiProfiler.cpp by path (REF_CUPTI_SRC, set by oracle/Makefile) because
// computeStats is a file-static function there (CuptiProfiler.cpp:44).
//
// Built only in the survey/dev container, where /root/reference and the cupti /
// pybind11 headers of the image exist; never used on the GPU box.
#include REF_CUPTI_SRC  // .../straggler/cupti_src/CuptiProfiler.cpp

#include <cstdint>
#include <cstring>

extern "C" {

struct ref_kstats {
    int32_t num_calls;
    float min, max, median, avg, stddev;
};

// CuptiProfiler.cpp:44-74
void ref_compute_stats(const float* data, int64_t n, ref_kstats* out) {
    std::vector<float> v(data, data + n);
    KernelStats s = computeStats(v);
    out->num_calls = s.num_calls;
    out->min = s.min;
    out->max = s.max;
    out->median = s.median;
    out->avg = s.avg;
    out->stddev = s.stddev;
}

// CircularBuffer.h:53-69: push n values into a capacity-cap ring, then linearize.
int64_t ref_ring_linearize(const float* pushed, int64_t n, int64_t cap, float* out) {
    CircularBuffer<float> rb((size_t)cap);
    for (int64_t i = 0; i < n; ++i) rb.push_back(pushed[i]);
    std::vector<float> lin = rb.linearize();
    if (!lin.empty()) std::memcpy(out, lin.data(), lin.size() * sizeof(float));
    return (int64_t)lin.size();
}

// CuptiProfiler.cpp:187: const float duration = (kernel->end - kernel->start) / 1000.0f;
float ref_ns_to_us(uint64_t start, uint64_t end) {
    const float duration = (end - start) / 1000.0f;
    return duration;
}

}  // extern "C"

extern "C" {
// vectorised CuptiProfiler.cpp:187 over uint32 durations (start = 0)
void ref_ns_to_us_array(const uint32_t* ns, int64_t n, float* out) {
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t start = 0, end = ns[i];
        const float duration = (end - start) / 1000.0f;
        out[i] = duration;
    }
}

// The reference's per-kernel path over a matrix of integer-ns durations, segment s =
// ns[s*stride + begin : +len], threaded over segments: every duration converted as
// bufferCompleted does (CuptiProfiler.cpp:187) and pushed into that kernel's
// CircularBuffer<float>(cap) (:189-198), then getStats' linearize + computeStats (:140-144).
// bench.py times this as the host-CPU baseline (cpu_baseline.kind = "reference").
void ref_matrix_stats(const uint32_t* ns, int64_t nseg, int64_t stride, int64_t begin, int64_t len,
                      int64_t cap, int32_t* num, float* mn, float* mx, float* med, float* avg,
                      float* sd, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        th.emplace_back([=] {
            const int64_t lo = nseg * t / nthreads, hi = nseg * (t + 1) / nthreads;
            for (int64_t s = lo; s < hi; ++s) {
                CircularBuffer<float> rb((size_t)cap);
                const uint32_t* p = ns + s * stride + begin;
                for (int64_t i = 0; i < len; ++i) {
                    const uint64_t start = 0, end = p[i];
                    const float duration = (end - start) / 1000.0f;
                    rb.push_back(duration);
                }
                const KernelStats k = computeStats(rb.linearize());
                num[s] = k.num_calls;
                mn[s] = k.min;
                mx[s] = k.max;
                med[s] = k.median;
                avg[s] = k.avg;
                sd[s] = k.stddev;
            }
        });
    }
    for (auto& x : th) x.join();
}
}
