// take.hip — compute::take on compressed arrays (compute-on-compressed).
//
// Reference: vortex-array/src/compute/take.rs:10-34 dispatches to the encoding's TakeFn.
// BitPackedArray's take (encodings/fastlanes/src/bitpacking/compute/take.rs:21-125) decodes only
// the 1024-blocks the indices touch (unpack_single for sparse blocks, bitpacking/compress.rs:
// 295-306) and patches the taken values from the Sparse patches (take.rs:127-200); FoRArray's
// take (for/compute.rs:39-48) takes the child and keeps the FoR; ALP's take (alp/compute.rs)
// takes the encoded child and its patches.  Every taken value here is the same bits the
// reference produces; the GPU does each index independently: one thread per index locates
// (block, row, lane) of the FastLanes layout, reads the one or two packed words holding it,
// applies the cascade's epilogue (FoR / ZigZag / ALP) and overrides it from the sorted patch
// indices by binary search (inner BitPacked patches before the epilogue, ALP patches after).
#include "fl_unpack_impl.hpp"
#include "take.hpp"

namespace vxg {

namespace {

constexpr int kTakeBlock = 256;

__device__ __forceinline__ uint64_t ld_uint(const void* p, int width, bool sgn, uint64_t i) {
    switch (width) {
    case 1: return sgn ? uint64_t(int64_t(static_cast<const int8_t*>(p)[i])) : static_cast<const uint8_t*>(p)[i];
    case 2: return sgn ? uint64_t(int64_t(static_cast<const int16_t*>(p)[i])) : static_cast<const uint16_t*>(p)[i];
    case 4: return sgn ? uint64_t(int64_t(static_cast<const int32_t*>(p)[i])) : static_cast<const uint32_t*>(p)[i];
    default: return static_cast<const uint64_t*>(p)[i];
    }
}

// fastlanes unchecked_unpack_single (bitpacking/compress.rs:295-306): value `pos` of the packed
// array (pos counts from the first packed block, i.e. includes the BitPacked offset).
template <int T>
__device__ __forceinline__ typename Fl<T>::E unpack_single(const uint8_t* __restrict__ packed, unsigned W, uint64_t pos) {
    using E = typename Fl<T>::E;
    constexpr unsigned LANES = 1024 / T;
    if (W == 0) return E(0);
    const unsigned k = unsigned(pos & 1023);
    const unsigned lane = k % LANES;
    const unsigned s = k / 128;
    const unsigned fl = (k - s * 128 - lane) / 16;
    const unsigned row = unsigned(fl_order(int(fl))) * 8 + s;  // FL_ORDER is an involution
    const E* __restrict__ blk = reinterpret_cast<const E*>(packed + (pos >> 10) * (128ull * W));
    if (W == unsigned(T)) return blk[LANES * row + lane];
    const unsigned start = row * W, w0 = start / T, sh = start % T;
    uint64_t v = uint64_t(blk[LANES * w0 + lane]) >> sh;
    if (sh + W > unsigned(T)) v |= uint64_t(blk[LANES * (w0 + 1) + lane]) << (T - sh);
    return E(W >= 64 ? v : (v & ((1ull << W) - 1ull)));
}

// index k of the sorted patch indices with (idx[k] - off) == pos, or -1
__device__ __forceinline__ int64_t find_patch(const TakePatches& p, uint64_t pos) {
    uint64_t lo = 0, hi = p.n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (ld_uint(p.idx, p.iw, p.isg != 0, mid) - p.off < pos) lo = mid + 1; else hi = mid;
    }
    return lo < p.n && ld_uint(p.idx, p.iw, p.isg != 0, lo) - p.off == pos ? int64_t(lo) : -1;
}

template <int T, Epi EPI>
__global__ __launch_bounds__(kTakeBlock) void take_packed_kernel(TakePacked a) {
    using E = typename Fl<T>::E;
    using O = typename EpiOut<T, EPI, 0>::type;
    O* __restrict__ out = static_cast<O*>(a.out);
    bool oob = false;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < a.n; j += stride) {
        uint64_t i = ld_uint(a.idx, a.iw, a.isg != 0, j);  // negative indices wrap -> out of bounds
        if (i >= a.len) {
            oob = true;
            i = 0;
        }
        E raw;
        const int64_t pk = a.inner.n ? find_patch(a.inner, i) : -1;
        if (pk >= 0) raw = static_cast<const E*>(a.inner.values)[pk];
        else raw = unpack_single<T>(a.packed, a.W, i + a.offset);
        O v = apply_epi<T, EPI, 0>(raw, a.ep);
        if (a.outer.n) {
            const int64_t qk = find_patch(a.outer, i);
            if (qk >= 0) v = static_cast<const O*>(a.outer.values)[qk];
        }
        out[j] = v;
    }
    if (oob) __hip_atomic_fetch_or(a.err, kErrTakeOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

unsigned take_grid(uint64_t n) {
    uint64_t g = (n + kTakeBlock - 1) / kTakeBlock;
    return unsigned(g > 65536 ? 65536 : (g ? g : 1));
}

}  // namespace

vxg_status launch_take_packed(int T, Epi epi, const TakePacked& a, hipStream_t s) {
    if (a.n == 0) return VXG_OK;
    const dim3 grid(take_grid(a.n)), block(kTakeBlock);
#define VXG_TAKE(TT, EE)                                                                     \
    if (T == TT && epi == EE) {                                                              \
        hipLaunchKernelGGL((take_packed_kernel<TT, EE>), grid, block, 0, s, a);              \
        return hip_check(hipGetLastError(), "take_packed_kernel");                            \
    }
    VXG_TAKE(8, Epi::Plain) VXG_TAKE(16, Epi::Plain) VXG_TAKE(32, Epi::Plain) VXG_TAKE(64, Epi::Plain)
    VXG_TAKE(8, Epi::For) VXG_TAKE(16, Epi::For) VXG_TAKE(32, Epi::For) VXG_TAKE(64, Epi::For)
    VXG_TAKE(8, Epi::ForZigZag) VXG_TAKE(16, Epi::ForZigZag) VXG_TAKE(32, Epi::ForZigZag)
    VXG_TAKE(64, Epi::ForZigZag) VXG_TAKE(32, Epi::AlpF32) VXG_TAKE(64, Epi::AlpF64)
#undef VXG_TAKE
    return set_error(VXG_ERR_NOT_IMPLEMENTED, "take: unsupported BitPacked cascade");
}

}  // namespace vxg
