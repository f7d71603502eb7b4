// take.hpp — arguments of the compute::take kernels (take.hip); internal, not the C ABI.
#pragma once

#include "fl_unpack_impl.hpp"  // EpiParams, Epi

namespace vxg {

// Sorted Sparse patch indices (SparseArray::resolved_indices = idx - off) and their values.
struct TakePatches {
    const void* idx = nullptr;
    const void* values = nullptr;
    uint64_t n = 0;
    uint64_t off = 0;
    int iw = 8;
    int isg = 0;
};

// take(indices) of a BitPacked-rooted cascade: BitPacked(T, W, offset, len) [+ inner patches]
// -> epilogue (FoR / FoR+ZigZag / ALP) [+ outer (ALP) patches].
struct TakePacked {
    const uint8_t* packed;
    unsigned W;
    unsigned offset;
    uint64_t len;
    const void* idx;  // indices (iw bytes each, signed if isg)
    int iw;
    int isg;
    uint64_t n;
    void* out;
    EpiParams ep;
    TakePatches inner;  // raw T values, applied before the epilogue
    TakePatches outer;  // output-typed values, applied after it
    uint32_t* err;
};

vxg_status launch_take_packed(int T, Epi epi, const TakePacked& a, hipStream_t s);

}  // namespace vxg
