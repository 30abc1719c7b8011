// Timing harness of records_resident.hip (not part of the library): configs[3]-shaped record
// streams (R streams x 47,482 Zipf-interleaved records, 2048 slots, cap 8192), the kernel alone,
// built once per ablation (-DNVRX_AB_RR=mask, see records_resident.hip).  Usage: rr_bench [R] [reps]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>
#include "records_resident.hip"
int main(int argc, char** argv) {
    const int64_t R = argc > 1 ? atoll(argv[1]) : 16384, reps = argc > 2 ? atoll(argv[2]) : 5;
    const int64_t K = 2048, cap = 8192;
    std::vector<int64_t> cnt(K);
    struct E { double key; uint32_t slot; };
    std::vector<E> ev;
    for (int64_t k = 0; k < K; ++k) {
        cnt[k] = std::max<int64_t>(1, (int64_t)std::floor(8192.0 / std::pow((double)(k + 1), 1.1)));
        for (int64_t i = 0; i < cnt[k]; ++i) ev.push_back({(2.0 * i + 1) / (2.0 * cnt[k]), (uint32_t)k});
    }
    std::sort(ev.begin(), ev.end(), [](const E& a, const E& b) { return a.key < b.key || (a.key == b.key && a.slot < b.slot); });
    const int64_t N = (int64_t)ev.size();
    std::vector<nvrx_record> h((size_t)(R * N));
    uint64_t x = 7;
    for (int64_t t = 0; t < R; ++t)
        for (int64_t i = 0; i < N; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            const uint32_t base = 2000 + (uint32_t)(ev[i].slot * 977u % 1998000u);
            h[t * N + i] = {ev[i].slot, base + (uint32_t)((x >> 33) % (base / 10 + 1))};
        }
    std::vector<int64_t> off(R + 1);
    for (int64_t t = 0; t <= R; ++t) off[t] = t * N;
    nvrx_record* d_recs; int64_t* d_off; int32_t *num, *sl, *cn; float* f[5];
    hipMalloc(&d_recs, h.size() * 8); hipMemcpy(d_recs, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipMalloc(&d_off, off.size() * 8); hipMemcpy(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice);
    const int64_t ng = R * K;
    hipMalloc(&num, ng * 4); hipMalloc(&sl, ng * 4); hipMalloc(&cn, ng * 4);
    for (auto& p : f) hipMalloc(&p, ng * 4);
    nvrx_stats_soa o{num, f[0], f[1], f[2], f[3], f[4]};
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipError_t e = nvrx::records_resident_stats(d_recs, d_off, R, K, cap, sl, cn, o, nullptr);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) e = nvrx::records_resident_stats(d_recs, d_off, R, K, cap, sl, cn, o, nullptr);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    printf("ab=%d R=%ld ms=%.3f (%s)\n", NVRX_AB_RR, (long)R, ms / reps, hipGetErrorString(e));
    return 0;
}
