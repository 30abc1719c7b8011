// segment_ragged_list.hip -- the wave-per-segment class kernels (PL 4..32) of
// segment_ragged.hip, in their own translation unit (parallel build).
#include "segment_ragged_kernels.h"

namespace nvrx {

void ragged_launch_list_big(int pl, const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                            const nvrx_stats_soa& out, hipStream_t st);

void ragged_launch_list(int pl, const RaggedSegs& segs, const uint32_t* list, const uint32_t* cls,
                        const nvrx_stats_soa& out, hipStream_t st) {
    using namespace ragged;
    switch (pl) {
        case 4: launch_list<4>(segs, list, cls, out, st); break;
        case 8: launch_list<8>(segs, list, cls, out, st); break;
        case 16: launch_list<16>(segs, list, cls, out, st); break;
        case 32: launch_list<32>(segs, list, cls, out, st); break;
        default: ragged_launch_list_big(pl, segs, list, cls, out, st); break;
    }
}

}  // namespace nvrx
