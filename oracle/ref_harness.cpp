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
}
