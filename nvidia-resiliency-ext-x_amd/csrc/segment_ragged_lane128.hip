// segment_ragged_lane128.hip -- the lane-per-segment class kernel of n <= 128 (the
// 128-register sorting network: the slowest instantiation to compile) of segment_ragged.hip,
// in its own translation unit (parallel build).
#include "segment_ragged_kernels.h"

namespace nvrx {

void ragged_launch_lane128(const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                           bool aligned16, const nvrx_stats_soa& out, hipStream_t st) {
    ragged::launch_lane<128>(segs, list, cls, aligned16, out, st);
}

}  // namespace nvrx
