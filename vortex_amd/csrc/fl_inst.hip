// K1 explicit instantiation unit.  Compiled several times by the Makefile with
//   -DFL_KIND_PLAIN -DFL_T=<8|16|32|64>   plain / FoR / FoR+ZigZag epilogues
//   -DFL_KIND_ALP                          BitPacked->FoR->ALP (u32->f32, u64->f64)
//   -DFL_KIND_DICT -DFL_VW=<1|2|4|8|16>    Dict(codes=BitPacked) gather, codes W <= 16
// so the ~800 kernel instantiations build in parallel.  Every K1 launch takes a chunk table
// (one array, or up to kArgChunks chunks of a ChunkedArray).
#include "fl_unpack_impl.hpp"

namespace vxg {

#if defined(FL_KIND_PLAIN)
#define FL_CAT2(a, b) a##b
#define FL_CAT(a, b) FL_CAT2(a, b)
vxg_status FL_CAT(fl_plain_, FL_T)(int W, Epi epi, const ChunkTable& t, uint64_t g, hipStream_t s) {
    switch (epi) {
    case Epi::Plain: return dispatch_w<FL_T, Epi::Plain, 0, FL_T>(W, t, g, s);
    case Epi::For: return dispatch_w<FL_T, Epi::For, 0, FL_T>(W, t, g, s);
    case Epi::ForZigZag: return dispatch_w<FL_T, Epi::ForZigZag, 0, FL_T>(W, t, g, s);
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
}
#elif defined(FL_KIND_ALP)
vxg_status fl_alp(int T, int W, Epi epi, const ChunkTable& t, uint64_t g, hipStream_t s) {
    if (epi == Epi::AlpF32 && T == 32) return dispatch_w<32, Epi::AlpF32, 0, 32>(W, t, g, s);
    if (epi == Epi::AlpF64 && T == 64) return dispatch_w<64, Epi::AlpF64, 0, 64>(W, t, g, s);
    return VXG_ERR_INVALID_ARGUMENT;
}
#elif defined(FL_KIND_DICT)
#define FL_CAT2(a, b) a##b
#define FL_CAT(a, b) FL_CAT2(a, b)
constexpr int kDictMaxW = 16;

template <int T>
static vxg_status dict_w(int W, const ChunkTable& t, uint64_t g, hipStream_t s) {
    constexpr int WM = T < kDictMaxW ? T : kDictMaxW;
    return dispatch_w<T, Epi::Dict, FL_VW, WM>(W, t, g, s);
}
vxg_status FL_CAT(fl_dict_, FL_VW)(int T, int W, const ChunkTable& t, uint64_t g, hipStream_t s) {
    switch (T) {
    case 8: return dict_w<8>(W, t, g, s);
    case 16: return dict_w<16>(W, t, g, s);
    case 32: return dict_w<32>(W, t, g, s);
    case 64: return dict_w<64>(W, t, g, s);
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
}
#else
#error "fl_inst.hip needs FL_KIND_PLAIN, FL_KIND_ALP or FL_KIND_DICT"
#endif

}  // namespace vxg
