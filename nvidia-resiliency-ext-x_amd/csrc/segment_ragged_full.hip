// segment_ragged_full.hip -- the FULL class kernels (exactly 64 * PL samples, 16-B aligned, FAST)
// of segment_ragged.hip, in their own translation unit (parallel build).
#include "segment_ragged_kernels.h"

namespace nvrx {

void ragged_launch_full(int pl, const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                        const nvrx_stats_soa& out, hipStream_t st) {
    using namespace ragged;
    switch (pl) {
        case 16: launch_list_full<16>(segs, list, cls, out, st); break;
        case 32: launch_list_full<32>(segs, list, cls, out, st); break;
        case 64: launch_list_full<64>(segs, list, cls, out, st); break;
        default: launch_list_full<128>(segs, list, cls, out, st); break;
    }
}

}  // namespace nvrx
