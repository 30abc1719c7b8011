// segment_ragged_lane.hip -- the lane-per-segment class kernels (n <= 8/16/32/64/128) of
// segment_ragged.hip, in their own translation unit (parallel build).
#include "segment_ragged_kernels.h"

namespace nvrx {

void ragged_launch_lane128(const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                           bool aligned16, const nvrx_stats_soa& out, hipStream_t st);

void ragged_launch_lane(int n, const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                        bool aligned16, const nvrx_stats_soa& out, hipStream_t st) {
    using namespace ragged;
    switch (n) {
        case 8: launch_lane<8>(segs, list, cls, aligned16, out, st); break;
        case 16: launch_lane<16>(segs, list, cls, aligned16, out, st); break;
        case 32: launch_lane<32>(segs, list, cls, aligned16, out, st); break;
        case 64: launch_lane<64>(segs, list, cls, aligned16, out, st); break;
        default: ragged_launch_lane128(segs, list, cls, aligned16, out, st); break;
    }
}

}  // namespace nvrx
