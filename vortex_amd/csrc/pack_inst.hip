// K15 explicit instantiation unit, compiled once per T (-DPK_T=8|16|32|64) by the Makefile so the
// pack kernels (W = 1..T-1, plain or fused FoR) build in parallel.
#include "fl_pack_impl.hpp"

namespace vxg {

#define PK_CAT2(a, b) a##b
#define PK_CAT(a, b) PK_CAT2(a, b)
vxg_status PK_CAT(fl_pack_, PK_T)(int W, bool for_, uint64_t ref, unsigned shift, bool sgn, const void* v, uint64_t n,
                                  void* packed, hipStream_t s) {
    return pack_dispatch<PK_T>(W, for_, ref, shift, sgn, v, n, packed, s, std::make_integer_sequence<int, PK_T - 1>{});
}

}  // namespace vxg
