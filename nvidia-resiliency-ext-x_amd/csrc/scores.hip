// scores.hip -- relative / individual performance scores on gfx950.
//
// Reference semantics (straggler/reporting.py):
//   _all_reduce_times      :255-296  per-kernel reference = min over ranks of the float32
//                                    MED; a rank without the kernel packs -1 => NaN.
//   _update_local_min_times:298-314  hist = min(hist, MED), BEFORE the individual score.
//   _compute_gpu_perf_score:219-253  score = sum_k (ref_k / MED_k) * (NUM_k * AVG_k) / sum_k w_k
//                                    over kernels with a non-NaN reference, f64; NaN when
//                                    there is none.
//   _compute_sections_perf_scores :196-217  score = ref_s / MED_s (no weights).
//   _get_tensor_from_scores :338-361 gather_on_rank0 packs scores as float32.
//   Report.identify_stragglers :84-151  straggler iff score < threshold (strict).
//
// Layout: stats are SoA [R][K] (row = rank, column = kernel), the same arrays the
// segment_stats kernels write.  Each per-element term is computed in f64 with
// separately rounded multiply/divide/add (-ffp-contract=off, no FMA), exactly as
// CPython evaluates it; the per-row sums use a fixed lane-stride + xor-butterfly
// order (deterministic; differs from Python's left-to-right order only by f64
// rounding, ~1e-16 relative).
#include "nvrx_common.h"
#include "nvrx_internal.h"

namespace nvrx {

__device__ __forceinline__ float bits_f32(uint32_t b) { return __uint_as_float(b); }

// ---------------------------------------------------------------------------
// Column reference: ref[k] = min_r med[r][k] if every rank has k, else NaN.
// ---------------------------------------------------------------------------
__global__ void kref_init_kernel(uint32_t* minbits, uint32_t* missing, int64_t K) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < K) {
        minbits[k] = 0x7F800000u;  // +inf; non-negative floats order like their bit patterns
        missing[k] = 0u;
    }
}

// grid.x over column tiles of 256, grid.y over row chunks of `rows` rows.
__global__ __launch_bounds__(256) void kref_reduce_kernel(const int32_t* __restrict__ num,
                                                          const float* __restrict__ med,
                                                          int64_t R, int64_t K, int64_t rows,
                                                          uint32_t* minbits, uint32_t* missing) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    const int64_t r0 = (int64_t)blockIdx.y * rows;
    const int64_t r1 = min(R, r0 + rows);
    uint32_t m = 0x7F800000u;
    bool miss = false;
#pragma unroll 8
    for (int64_t r = r0; r < r1; ++r) {  // unrolled: 8 independent loads in flight per thread
        const int64_t e = r * K + k;
        const int32_t c = num[e];
        const uint32_t b = __float_as_uint(med[e]);
        miss |= c <= 0;
        m = c > 0 ? min(m, b) : m;
    }
    if (miss) atomicOr(&missing[k], 1u);
    atomicMin(&minbits[k], m);
}

__global__ void kref_final_kernel(const uint32_t* minbits, const uint32_t* missing, int64_t K,
                                  int64_t R, float* ref) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < K) ref[k] = (missing[k] || R <= 0) ? __builtin_nanf("") : bits_f32(minbits[k]);
}

hipError_t kernel_ref(const int32_t* num, const float* med, int64_t R, int64_t K, float* ref,
                      uint32_t* scratch, hipStream_t st) {
    if (K <= 0) return hipSuccess;
    uint32_t* minbits = scratch;
    uint32_t* missing = scratch + K;
    const unsigned kb = (unsigned)((K + 255) / 256);
    hipLaunchKernelGGL(kref_init_kernel, dim3(kb), dim3(256), 0, st, minbits, missing, K);
    if (R > 0) {
        // 32 rows per thread: R/32 atomics per column, grid >> 256 CUs at scale
        const int64_t rows = 32;
        const unsigned rb = (unsigned)((R + rows - 1) / rows);
        hipLaunchKernelGGL(kref_reduce_kernel, dim3(kb, rb), dim3(256), 0, st, num, med, R, K,
                           rows, minbits, missing);
    }
    if (ref)  // NULL: the caller consumes the [minbits | missing] words of `scratch`
        hipLaunchKernelGGL(kref_final_kernel, dim3(kb), dim3(256), 0, st, minbits, missing, K, R, ref);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// _all_reduce_times pack: times = -1; times[id] = float32(MED)
// ---------------------------------------------------------------------------
__global__ void fill_f32_kernel(float* p, int64_t n, float v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}
__global__ void pack_times_kernel(const double* med, const int32_t* ids, int64_t n, float* times) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) times[ids[i]] = (float)med[i];  // RN to float32, as the torch float32 store
}

hipError_t pack_min_times(const double* med, const int32_t* ids, int64_t n, float* times,
                          int64_t total, hipStream_t st) {
    if (total > 0) {
        const int64_t gb = (total + 255) / 256;
        const unsigned g = (unsigned)(gb < 1024 ? gb : 1024);
        hipLaunchKernelGGL(fill_f32_kernel, dim3(g), dim3(256), 0, st, times, total, -1.0f);
    }
    if (n > 0) {
        const unsigned g = (unsigned)((n + 255) / 256);
        hipLaunchKernelGGL(pack_times_kernel, dim3(g), dim3(256), 0, st, med, ids, n, times);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per-row weighted score partials: one 64-lane wave per row.
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T tmin(T a, T b) { return b < a ? b : a; }  // Python min(a, b)

// score = n > 0 ? sum(s*w)/sum(w) : NaN (reporting.py:251-253); returns true when the
// total weight is 0 (Python raises ZeroDivisionError there).
__device__ __forceinline__ bool finish(double sw, double w, double n, double& out) {
    out = __builtin_nan("");
    if (n > 0.0) {
        out = sw / w;
        return w == 0.0;
    }
    return false;
}

// One 256-thread workgroup per row (rank): lanes stride over the kernels, each wave
// reduces with DPP, the 4 wave results are added in wave order (deterministic).
template <typename T>
__global__ __launch_bounds__(256) void scores_kernel(nvrx_score_args a) {
    __shared__ double red[4][6];
    __shared__ int zflag[4];
    __shared__ bool last;
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    const int64_t r = blockIdx.x;
    const int64_t K = a.K;
    const int64_t hs = a.hist_stride > 0 ? a.hist_stride : K;
    const bool do_rel = a.ref != nullptr;
    const bool do_ind = a.hist != nullptr;
    double swr = 0.0, wr = 0.0, nr = 0.0, swi = 0.0, wi = 0.0, ni = 0.0;
    bool zero_med = false;
    const int32_t* __restrict__ num = a.num + r * K;
    const T* __restrict__ med = (const T*)a.med + r * K;
    const T* __restrict__ avg = (const T*)a.avg + r * K;
    T* hist = (T*)a.hist;
    // Elements are taken SC at a time per thread, every load of a batch issued before any
    // is used (one memory latency per batch instead of one per element: at R = 64 one row per
    // workgroup is only 256 waves, so the kernel is latency-bound).  Each thread still visits
    // k = tid, tid + 256, ... in increasing order, so the sums are the ones of the
    // element-at-a-time loop, bit for bit.
    constexpr int SC = 8;
    for (int64_t k0 = tid; k0 < K; k0 += 256 * SC) {
        int32_t nm[SC];
        T mt[SC], av[SC], hv[SC];
        float rf[SC];
        bool ok[SC], rok[SC];
#pragma unroll
        for (int c = 0; c < SC; ++c) {
            const int64_t k = k0 + c * 256;
            const bool in = k < K;
            nm[c] = in ? num[k] : 0;
            ok[c] = in && (!a.col_valid || a.col_valid[k]);  // "ncclDev" filter (reporting.py:330-336)
            mt[c] = in ? med[k] : (T)1;
            av[c] = in ? avg[k] : (T)0;
            hv[c] = (in && do_ind) ? hist[r * hs + (a.hist_index ? a.hist_index[k] : k)] : (T)0;
            rf[c] = -1.0f;
            rok[c] = false;
            if (in && do_rel) {
                const int64_t ri = a.ref_index ? a.ref_index[k] : k;
                rf[c] = a.ref[ri];
                rok[c] = !(a.ref_missing && a.ref_missing[ri]);
            }
        }
#pragma unroll
        for (int c = 0; c < SC; ++c) {
            const int64_t k = k0 + c * 256;
            if (!ok[c] || nm[c] <= 0) continue;  // kernel not in this rank's summaries
            const double m = (double)mt[c];
            const double w = (double)nm[c] * (double)av[c];  // NUM * AVG (reporting.py:248)
            if (do_ind) {
                const T h = tmin(hv[c], mt[c]);  // min(hist, MED) (reporting.py:310)
                hist[r * hs + (a.hist_index ? a.hist_index[k] : k)] = h;
                zero_med |= (m == 0.0);
                const double sc = (double)h / m;
                const double t = sc * w;
                swi = swi + t;
                wi = wi + w;
                ni += 1.0;
            }
            if (do_rel && rf[c] >= 0.0f && rok[c]) {  // -1 / NaN => no reference (reporting.py:290, 244-245)
                zero_med |= (m == 0.0);
                const double sc = (double)rf[c] / m;
                const double t = sc * w;
                swr = swr + t;
                wr = wr + w;
                nr += 1.0;
            }
        }
    }
    swr = wave_sum_f64(swr);
    wr = wave_sum_f64(wr);
    nr = wave_sum_f64(nr);
    swi = wave_sum_f64(swi);
    wi = wave_sum_f64(wi);
    ni = wave_sum_f64(ni);
    const bool anyzero = __ballot(zero_med) != 0;
    if (lane == 0) {
        red[wave][0] = swr;
        red[wave][1] = wr;
        red[wave][2] = nr;
        red[wave][3] = swi;
        red[wave][4] = wi;
        red[wave][5] = ni;
        zflag[wave] = anyzero;
    }
    __syncthreads();
    if (tid == 0) {
        double p[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) p[i] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
        int errbits = (zflag[0] | zflag[1] | zflag[2] | zflag[3]) ? 1 : 0;
        if (a.partials) {
#pragma unroll
            for (int i = 0; i < 6; ++i) a.partials[r * 6 + i] = p[i];
        }
        if (a.gpu_rel || a.gpu_ind || a.strag_rel || a.strag_ind) {
            double sr, si;
            bool zw = finish(p[0], p[1], p[2], sr);
            zw |= finish(p[3], p[4], p[5], si);
            if (zw) errbits |= 2;
            if (a.round_f32) {
                sr = (double)(float)sr;
                si = (double)(float)si;
            }
            if (a.gpu_rel) a.gpu_rel[r] = sr;
            if (a.gpu_ind) a.gpu_ind[r] = si;
            if (a.strag_rel) a.strag_rel[r] = sr < a.thr_rel;  // NaN compares false
            if (a.strag_ind) a.strag_ind[r] = si < a.thr_ind;
        }
        if (!a.done) {
            if (errbits && a.err) atomicOr(a.err, errbits);
        } else {
            if (errbits) atomicOr(&a.done[1], (uint32_t)errbits);
            __threadfence();  // this row's results (and reads of the reference) come first
            last = atomicAdd(&a.done[0], 1u) == gridDim.x - 1;
        }
    }
    if (!a.done) return;
    __syncthreads();
    if (!last) return;
    // the last workgroup: every other one has finished reading the column reference
    __threadfence();
    for (int64_t i = tid; i < 2 * a.reset_ncols; i += 256)
        a.reset_col_ref[i] = i < a.reset_ncols ? 0x7F800000u : 0u;
    if (tid == 0) {
        const uint32_t e = atomicExch(&a.done[1], 0u);
        if (a.err) *a.err = (int32_t)e;
        a.done[0] = 0u;
    }
}

hipError_t scores(const nvrx_score_args& a, hipStream_t st) {
    if (a.R <= 0) return hipSuccess;
    if (a.R > 0x7FFFFFFF) return hipErrorInvalidValue;
    const unsigned g = (unsigned)a.R;
    if (a.value_f64)
        hipLaunchKernelGGL(scores_kernel<double>, dim3(g), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(scores_kernel<float>, dim3(g), dim3(256), 0, st, a);
    return hipGetLastError();
}

__global__ void finalize_kernel(const double* partials, int64_t R, int64_t nshards, int round_f32,
                                double thr_rel, double thr_ind, double* gpu_rel, double* gpu_ind,
                                uint8_t* strag_rel, uint8_t* strag_ind, int32_t* err) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    double p[6] = {0, 0, 0, 0, 0, 0};
    for (int64_t g = 0; g < nshards; ++g) {  // fixed shard order
        const double* q = partials + (g * R + r) * 6;
#pragma unroll
        for (int i = 0; i < 6; ++i) p[i] = p[i] + q[i];
    }
    const double qnan = __builtin_nan("");
    double sr = qnan, si = qnan;
    bool zero_w = false;
    if (p[2] > 0.0) {
        zero_w |= (p[1] == 0.0);
        sr = p[0] / p[1];
    }
    if (p[5] > 0.0) {
        zero_w |= (p[4] == 0.0);
        si = p[3] / p[4];
    }
    if (round_f32) {
        sr = (double)(float)sr;
        si = (double)(float)si;
    }
    if (gpu_rel) gpu_rel[r] = sr;
    if (gpu_ind) gpu_ind[r] = si;
    if (strag_rel) strag_rel[r] = sr < thr_rel;  // NaN compares false
    if (strag_ind) strag_ind[r] = si < thr_ind;
    if (zero_w && err) atomicOr(err, 2);
}

hipError_t finalize_scores(const double* partials, int64_t R, int64_t nshards, int round_f32,
                           double thr_rel, double thr_ind, double* gpu_rel, double* gpu_ind,
                           uint8_t* strag_rel, uint8_t* strag_ind, int32_t* err, hipStream_t st) {
    if (R <= 0) return hipSuccess;
    const unsigned g = (unsigned)((R + 255) / 256);
    hipLaunchKernelGGL(finalize_kernel, dim3(g), dim3(256), 0, st, partials, R, nshards, round_f32,
                       thr_rel, thr_ind, gpu_rel, gpu_ind, strag_rel, strag_ind, err);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Sections
// ---------------------------------------------------------------------------
__global__ void section_ref_kernel(const double* med, const uint8_t* present, int64_t R,
                                   int64_t S, float* ref) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    float m = __builtin_inff();
    bool miss = R <= 0;
    for (int64_t r = 0; r < R; ++r) {
        if (!present[r * S + s]) {
            miss = true;
            break;
        }
        m = fminf(m, (float)med[r * S + s]);  // packed as float32 (reporting.py:273-279)
    }
    ref[s] = miss ? __builtin_nanf("") : m;
}

__global__ void section_scores_kernel(const double* med, const uint8_t* present, int64_t R,
                                      int64_t S, const float* ref, const int32_t* ref_index,
                                      double* hist, int round_f32, double* out_rel,
                                      double* out_ind, int32_t* err) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= R * S) return;
    const int64_t s = e % S;
    const double qnan = __builtin_nan("");
    double rel = qnan, ind = qnan;
    if (present[e]) {
        const double m = med[e];
        bool zero = false;
        if (out_ind && hist) {
            double h = hist[e];
            h = m < h ? m : h;  // min(hist, MED), f64 (reporting.py:313)
            hist[e] = h;
            zero |= (m == 0.0);
            ind = h / m;
        }
        if (out_rel && ref) {
            const float rf = ref[ref_index ? ref_index[s] : s];
            const double rd = (rf >= 0.0f) ? (double)rf : qnan;  // -1 => NaN (reporting.py:295)
            zero |= (m == 0.0);
            rel = rd / m;
        }
        if (zero && err) atomicOr(err, 1);
    }
    if (round_f32) {
        rel = (double)(float)rel;
        ind = (double)(float)ind;
    }
    if (out_rel) out_rel[e] = rel;
    if (out_ind) out_ind[e] = ind;
}

hipError_t section_scores(const double* med, const uint8_t* present, int64_t R, int64_t S,
                          const float* ref_in, const int32_t* ref_index, float* ref_work,
                          double* hist, int round_f32, double* out_rel, double* out_ind,
                          int32_t* err, hipStream_t st) {
    if (R <= 0 || S <= 0) return hipSuccess;
    const float* ref = ref_in;
    if (out_rel && !ref_in) {
        if (!ref_work) return hipErrorInvalidValue;
        hipLaunchKernelGGL(section_ref_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st,
                           med, present, R, S, ref_work);
        ref = ref_work;
        ref_index = nullptr;
    }
    const unsigned g = (unsigned)((R * S + 255) / 256);
    hipLaunchKernelGGL(section_scores_kernel, dim3(g), dim3(256), 0, st, med, present, R, S, ref,
                       ref_index, hist, round_f32, out_rel, out_ind, err);
    return hipGetLastError();
}

__global__ void stragglers_kernel(const double* score, int64_t n, double thr, uint8_t* mask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) mask[i] = score[i] < thr;
}

hipError_t stragglers(const double* score, int64_t n, double thr, uint8_t* mask, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(stragglers_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       score, n, thr, mask);
    return hipGetLastError();
}

}  // namespace nvrx
