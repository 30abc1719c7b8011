/*
 * nvrx_synth.h -- TEST / BENCH INFRASTRUCTURE: device-side synthetic duration generator.
 * Not part of the product ABI (nvrx_straggler.h).  Bit-identical to the C oracle's
 * generator (oracle/nvrx_oracle.c: oracle_sample_ns), SURVEY.md 8(d):
 *   u    = splitmix64(seed ^ ((r*K + k)*S_push + i))
 *   base = 2000 + splitmix64(seed2 ^ k) % 1998000                 (2 us .. 2 ms)
 *   ns   = base + (((u >> 32) * (base / 10)) >> 32)               (0..10% jitter)
 *   ns   = ns * 13 / 10 on straggler ranks
 */
#ifndef NVRX_SYNTH_H
#define NVRX_SYNTH_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* out[r][kk][i] for r < R, kk < K_local, i < s_push, where the global kernel index of
 * local column kk is kmap[kk] (kmap NULL: kk) and K_global is used in the sample hash. */
int nvrx_synth_matrix(uint32_t* out, int64_t R, int64_t K_local, int64_t K_global,
                      const int64_t* kmap, int64_t s_push, uint64_t seed, uint64_t seed2,
                      const uint8_t* straggler, void* stream);
/* Record streams (configs[3]): out[r*N + j] = {slot[j], ns}, ns the occ[j]-th sample of
 * global kernel kglob[j] (kglob NULL: slot[j]) on rank r under the hash above with
 * S_push = s_push and K = K (the global kernel count). */
int nvrx_synth_records(uint32_t* out, int64_t R, int64_t N, const uint32_t* slot,
                       const uint32_t* kglob, const uint32_t* occ, int64_t K, int64_t s_push,
                       uint64_t seed, uint64_t seed2, const uint8_t* straggler, void* stream);
#ifdef __cplusplus
}
#endif
#endif
