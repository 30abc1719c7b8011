/*
 * abi_host.c -- a native C11 host of the C ABI (include/nvrx_straggler.h), linked against
 * libnvrx_hip.so with no Python in the process.  It runs INTEGRATION.md section 3's sequence and
 * the profiler handle's lifecycle, and writes every input and output to one binary file that
 * tests/test_native_host.py checks against the oracle bit for bit:
 *
 *   A. a rank x kernel matrix of u32 ns in device memory -> nvrx_segment_stats_strided (with
 *      the fused per-kernel reference) -> nvrx_scores (history, in-kernel finalize, straggler
 *      masks): the reference's computeStats + ReportGenerator scoring (CuptiProfiler.cpp:44-74,
 *      reporting.py:219-314) for every rank at once;
 *   B. nvrx_profiler_*: the nvrx_cupti_module.CuptiProfiler lifecycle (cupti_module_py.cpp:33-54)
 *      -- create, a second create refused (singleton, CuptiProfiler.cpp:83-90), initialize,
 *      start, register + push records (a ring of 7 over 21 pushes, test_cupti_ext.py:107-127),
 *      stop, get_stats (name-sorted, getStats :136-146), reset (every kernel forgotten), shutdown,
 *      destroy, and a new create once the first is gone.
 *
 * Usage: abi_host OUT.bin        exit status 0 on success; a failed check prints why and exits 1.
 * Built by tests/native/Makefile (gcc -std=c11 -Wall -Wextra -pedantic -Werror).
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nvrx_straggler.h"

enum { R = 16, K = 96, S = 1500, CAP = 1024 };
enum { STRAGGLER_RANK = 5 };

#define CHECK(cond, ...)                                                   \
    do {                                                                   \
        if (!(cond)) {                                                     \
            fprintf(stderr, "abi_host:%d: ", __LINE__);                    \
            fprintf(stderr, __VA_ARGS__);                                  \
            fprintf(stderr, " (last error: %s)\n", nvrx_last_error());     \
            exit(1);                                                       \
        }                                                                  \
    } while (0)
#define OK(call) CHECK((call) == NVRX_OK, "%s failed", #call)
#define HIP(call) CHECK((call) == hipSuccess, "%s failed", #call)

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void put(FILE* f, const void* p, size_t n) { CHECK(fwrite(p, 1, n, f) == n, "write"); }

static void* dalloc(size_t n) {
    void* p = NULL;
    HIP(hipMalloc(&p, n));
    return p;
}

static void part_matrix(FILE* f) {
    const size_t nseg = (size_t)R * K, nsamp = nseg * S;
    uint32_t* ns = malloc(nsamp * sizeof(uint32_t));
    CHECK(ns, "malloc");
    for (size_t seg = 0; seg < nseg; ++seg) {
        const uint64_t r = seg / K, k = seg % K;
        const uint64_t base = 2000 + splitmix64(0xBA5Eull ^ k) % 200000;
        for (size_t i = 0; i < S; ++i) {
            uint64_t v = base + splitmix64(0x5EEDull ^ (seg * S + i)) % (base / 10 + 1);
            if (r == STRAGGLER_RANK) v = v * 13 / 10;
            ns[seg * S + i] = (uint32_t)v;
        }
    }
    hipStream_t st;
    HIP(hipStreamCreate(&st));
    uint32_t* d_ns = dalloc(nsamp * sizeof(uint32_t));
    HIP(hipMemcpy(d_ns, ns, nsamp * sizeof(uint32_t), hipMemcpyHostToDevice));
    nvrx_stats_soa soa = {dalloc(nseg * 4), dalloc(nseg * 4), dalloc(nseg * 4),
                          dalloc(nseg * 4), dalloc(nseg * 4), dalloc(nseg * 4)};
    uint32_t* col_ref = dalloc(2 * K * sizeof(uint32_t));
    float* hist = dalloc(nseg * sizeof(float));
    float* h_hist = malloc(nseg * sizeof(float));
    CHECK(h_hist, "malloc");
    for (size_t i = 0; i < nseg; ++i) h_hist[i] = INFINITY;  /* reporting.py:186-191 */
    HIP(hipMemcpy(hist, h_hist, nseg * sizeof(float), hipMemcpyHostToDevice));
    int32_t* err = dalloc(sizeof(int32_t));
    HIP(hipMemset(err, 0, sizeof(int32_t)));
    double* gpu_rel = dalloc(R * sizeof(double));
    double* gpu_ind = dalloc(R * sizeof(double));
    uint8_t* srel = dalloc(R);
    uint8_t* sind = dalloc(R);

    /* INTEGRATION.md section 3 */
    OK(nvrx_segment_stats_strided(d_ns, (int64_t)nseg, S, 0, S, CAP, NVRX_STATS_FAST, &soa, col_ref,
                                  K, st));
    nvrx_score_args a;
    memset(&a, 0, sizeof a);
    a.R = R;
    a.K = K;
    a.num = soa.num;
    a.med = soa.med;
    a.avg = soa.avg;
    a.ref = (const float*)col_ref;
    a.ref_missing = col_ref + K;
    a.hist = hist;
    a.err = err;
    a.thr_rel = 0.8;
    a.thr_ind = 0.8;
    a.gpu_rel = gpu_rel;
    a.gpu_ind = gpu_ind;
    a.strag_rel = srel;
    a.strag_ind = sind;
    OK(nvrx_scores(&a, st));
    OK(nvrx_sync(st));

    const int64_t hdr[4] = {R, K, S, CAP};
    put(f, hdr, sizeof hdr);
    put(f, ns, nsamp * sizeof(uint32_t));
    void* host = malloc(nseg * 4);
    CHECK(host, "malloc");
    void* fields[6] = {soa.num, soa.min, soa.max, soa.med, soa.avg, soa.std};
    for (int i = 0; i < 6; ++i) {
        HIP(hipMemcpy(host, fields[i], nseg * 4, hipMemcpyDeviceToHost));
        put(f, host, nseg * 4);
    }
    double h_sc[R];
    uint8_t h_m[R];
    HIP(hipMemcpy(h_sc, gpu_rel, sizeof h_sc, hipMemcpyDeviceToHost));
    put(f, h_sc, sizeof h_sc);
    HIP(hipMemcpy(h_sc, gpu_ind, sizeof h_sc, hipMemcpyDeviceToHost));
    put(f, h_sc, sizeof h_sc);
    HIP(hipMemcpy(h_m, srel, sizeof h_m, hipMemcpyDeviceToHost));
    put(f, h_m, sizeof h_m);
    CHECK(h_m[STRAGGLER_RANK] == 1, "rank %d not flagged", STRAGGLER_RANK);
    HIP(hipMemcpy(h_m, sind, sizeof h_m, hipMemcpyDeviceToHost));
    put(f, h_m, sizeof h_m);
    int32_t h_err = -1;
    HIP(hipMemcpy(&h_err, err, sizeof h_err, hipMemcpyDeviceToHost));
    put(f, &h_err, sizeof h_err);
    CHECK(h_err == 0, "err = %d", (int)h_err);

    for (int i = 0; i < 6; ++i) HIP(hipFree(fields[i]));
    HIP(hipFree(d_ns));
    HIP(hipFree(col_ref));
    HIP(hipFree(hist));
    HIP(hipFree(err));
    HIP(hipFree(gpu_rel));
    HIP(hipFree(gpu_ind));
    HIP(hipFree(srel));
    HIP(hipFree(sind));
    HIP(hipStreamDestroy(st));
    free(ns);
    free(h_hist);
    free(host);
}

#define NKER 3
#define NAME_LEN 96

static void part_profiler(FILE* f) {
    static const char* names[NKER] = {"gemm_tn_blk_256_1_1_grid_64_1_1",
                                      "attn_fwd_blk_128_1_1_grid_32_8_1",
                                      "layer_norm_blk_64_1_1_grid_16_1_1"};
    const int pushes[NKER] = {21, 5, 1};
    nvrx_profiler_config cfg = {8 << 20, 8, 7, 0, NVRX_STATS_EXACT};
    nvrx_profiler* p = NULL;
    nvrx_profiler* q = NULL;
    OK(nvrx_profiler_create(&cfg, &p));
    CHECK(nvrx_profiler_create(&cfg, &q) == NVRX_ERR_SINGLETON && q == NULL,
          "a second profiler instance was not refused");
    CHECK(strstr(nvrx_last_error(), "Only one") != NULL, "singleton message: %s", nvrx_last_error());
    OK(nvrx_profiler_initialize(p));
    OK(nvrx_profiler_start(p));
    uint32_t slot[NKER];
    for (int k = 0; k < NKER; ++k) OK(nvrx_profiler_register_kernel(p, names[k], &slot[k]));
    nvrx_record recs[64];
    int64_t n = 0;
    for (int i = 0; i < 21; ++i)  /* interleaved push order, as kernels launch */
        for (int k = 0; k < NKER; ++k)
            if (i < pushes[k]) {
                recs[n].slot = slot[k];
                recs[n].ns = (uint32_t)(1000 * (k + 1) + (uint32_t)(splitmix64((uint64_t)(i * 7 + k)) % 997));
                ++n;
            }
    OK(nvrx_profiler_push(p, recs, n));
    OK(nvrx_profiler_stop(p));
    nvrx_record late = {slot[0], 5};
    OK(nvrx_profiler_push(p, &late, 1));  /* stopped: dropped */
    int64_t count = -1;
    OK(nvrx_profiler_get_stats(p, 0, &count, NULL, NULL, NULL, NULL, NULL, NULL, NULL));
    CHECK(count == NKER, "get_stats size query: %lld kernels", (long long)count);
    uint32_t s_slot[NKER];
    int32_t s_num[NKER];
    float s_min[NKER], s_max[NKER], s_med[NKER], s_avg[NKER], s_std[NKER];
    OK(nvrx_profiler_get_stats(p, NKER, &count, s_slot, s_num, s_min, s_max, s_med, s_avg, s_std));
    char sorted_names[NKER][NAME_LEN];
    memset(sorted_names, 0, sizeof sorted_names);
    for (int i = 0; i < NKER; ++i)
        OK(nvrx_profiler_kernel_name(p, s_slot[i], sorted_names[i], NAME_LEN));
    for (int i = 1; i < NKER; ++i)
        CHECK(strcmp(sorted_names[i - 1], sorted_names[i]) < 0, "get_stats not name-sorted");
    CHECK(s_num[0] >= 1 && (s_num[0] == 7 || s_num[1] == 7 || s_num[2] == 7), "ring of 7 not kept");

    const int64_t hdr[2] = {n, NKER};
    put(f, hdr, sizeof hdr);
    put(f, recs, (size_t)n * sizeof(nvrx_record));
    char slot_names[NKER][NAME_LEN];  /* the name of every slot, slot order */
    memset(slot_names, 0, sizeof slot_names);
    for (int k = 0; k < NKER; ++k) strncpy(slot_names[slot[k]], names[k], NAME_LEN - 1);
    put(f, slot_names, sizeof slot_names);
    put(f, s_slot, sizeof s_slot);
    put(f, s_num, sizeof s_num);
    put(f, s_min, sizeof s_min);
    put(f, s_max, sizeof s_max);
    put(f, s_med, sizeof s_med);
    put(f, s_avg, sizeof s_avg);
    put(f, s_std, sizeof s_std);
    put(f, sorted_names, sizeof sorted_names);

    OK(nvrx_profiler_reset(p));  /* CuptiProfiler.cpp:148-152 */
    OK(nvrx_profiler_get_stats(p, 0, &count, NULL, NULL, NULL, NULL, NULL, NULL, NULL));
    CHECK(count == 0, "%lld kernels after reset", (long long)count);
    OK(nvrx_profiler_shutdown(p));
    OK(nvrx_profiler_destroy(p));
    OK(nvrx_profiler_create(&cfg, &q));  /* the singleton is free again */
    OK(nvrx_profiler_destroy(q));
}

int main(int argc, char** argv) {
    CHECK(argc == 2, "usage: abi_host OUT.bin");
    CHECK(nvrx_abi_version() == NVRX_ABI_VERSION, "ABI %d, header %d", nvrx_abi_version(),
          NVRX_ABI_VERSION);
    int ndev = 0;
    OK(nvrx_device_count(&ndev));
    CHECK(ndev >= 1, "no HIP device");
    FILE* f = fopen(argv[1], "wb");
    CHECK(f != NULL, "open %s", argv[1]);
    part_matrix(f);
    part_profiler(f);
    CHECK(fclose(f) == 0, "close");
    printf("abi_host ok\n");
    return 0;
}
