// segment_ragged_big.hip -- the wave-per-segment class kernels of PL 64 / 128 and the
// workgroup-per-segment (EXACT) kernels of segment_ragged.hip, in their own translation unit
// (parallel build).
#include "segment_ragged_kernels.h"

namespace nvrx {

void ragged_launch_list_big(int pl, const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                            const nvrx_stats_soa& out, hipStream_t st) {
    using namespace ragged;
    if (pl == 64)
        launch_list<64>(segs, list, cls, out, st);
    else
        launch_list<128>(segs, list, cls, out, st);
}

hipError_t ragged_launch_exact(const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                               int64_t max_len, const nvrx_stats_soa& out,
                               hipStream_t st) {
    return ragged::launch_exact_list(segs, list, cls, max_len, out, st);
}

}  // namespace nvrx
