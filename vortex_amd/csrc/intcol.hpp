// intcol.hpp — device-side readers for IntCol (vxg_internal.hpp): integer columns that a
// consumer kernel (FSST offsets/lengths, Sparse patch indices) reads in place — a plain
// array, or a patch-free [FoR](BitPacked) FastLanes column unpacked per element
// (fastlanes unpack_single, bitpacking/compress.rs:295-306; layout SURVEY.md Appendix A).
#pragma once
#include <type_traits>

#include "vxg_internal.hpp"

namespace vxg {

// Integer load with compile-time width/signedness.  (A runtime width switch compiles to a
// branch nest that waits vmcnt(0) after every load.)
// (Column pointers address global memory; they are often read from a device table, where the
// compiler would otherwise emit flat loads: gload.)
template <int WIDTH, bool SGN>
__device__ __forceinline__ int64_t ld(const void* p, uint64_t i) {
    if constexpr (WIDTH == 1) return SGN ? int64_t(gload(static_cast<const int8_t*>(p) + i)) : int64_t(gload(static_cast<const uint8_t*>(p) + i));
    else if constexpr (WIDTH == 2) return SGN ? int64_t(gload(static_cast<const int16_t*>(p) + i)) : int64_t(gload(static_cast<const uint16_t*>(p) + i));
    else if constexpr (WIDTH == 4) return SGN ? int64_t(gload(static_cast<const int32_t*>(p) + i)) : int64_t(gload(static_cast<const uint32_t*>(p) + i));
    else return gload(static_cast<const int64_t*>(p) + i);
}

// Value `idx` (< 1024) of the FastLanes block at `blk` (T-bit words, bit width 0 < W <= T):
// unpack_single's (lane, row) -> bit offset row * W in the lane's words.  Both candidate words are
// loaded unconditionally (they retire under one wait; no branch the compiler could sink the
// second load into), the T = 32 pair is one funnel shift (v_alignbit), row * W a 24-bit multiply.
template <int T>
__device__ __forceinline__ std::conditional_t<T == 32, uint32_t, uint64_t> fl_word_pair(
    const std::conditional_t<T == 32, uint32_t, uint64_t>* blk, uint32_t idx, uint32_t W) {
    using E = std::conditional_t<T == 32, uint32_t, uint64_t>;
    constexpr uint32_t LANES = 1024 / T;
    const uint32_t lane = idx % LANES, s = idx >> 7;
    const uint32_t fl = ((idx & 127) - lane) >> 4;
    const uint32_t row = (((fl & 1) << 2) | (fl & 2) | (fl >> 2)) * 8 + s;  // FL_ORDER[fl]*8 + s
    const uint32_t start = __umul24(row, W), word = start / T, sh = start % T;
    const uint32_t word2 = word + 1 < W ? word + 1 : word;
    const E lo = gload(blk + LANES * word + lane), hi = gload(blk + LANES * word2 + lane);
    const E mask = W >= uint32_t(T) ? E(~E(0)) : E((E(1) << W) - 1);
    if constexpr (T == 32) {
        return __builtin_amdgcn_alignbit(hi, lo, sh) & mask;
    } else {
        return (sh ? (lo >> sh) | (hi << (64 - sh)) : lo) & mask;
    }
}

// Element i of a T-bit FastLanes column of bit width W, then FoR (wrapping in T), sign-extended
// when the logical type is signed.
template <int T>
__device__ __forceinline__ int64_t fl_get(const void* packed, uint32_t W, uint32_t shift, uint32_t offset,
                                          uint64_t reference, bool sgn, uint64_t i) {
    using E = std::conditional_t<T == 32, uint32_t, uint64_t>;
    constexpr uint32_t LANES = 1024 / T;
    E v = 0;
    if (W != 0) {
        const uint64_t g = i + offset;
        v = fl_word_pair<T>(static_cast<const E*>(packed) + (g >> 10) * (uint64_t(LANES) * W), uint32_t(g & 1023), W);
    }
    const E r = E(E(v << shift) + E(reference));
    if constexpr (T == 64) return int64_t(r);
    else return sgn ? int64_t(int32_t(r)) : int64_t(r);
}

// Compile-time readers (hot loops): Plain<WIDTH> and Packed<T>.
template <int WIDTH> struct PlainCol {
    const void* p;
    bool sgn;
    __host__ __device__ explicit PlainCol(const IntCol& c) : p(c.p), sgn(c.sgn) {}
    __device__ __forceinline__ int64_t operator()(uint64_t i) const {
        const int64_t u = ld<WIDTH, false>(p, i);
        if constexpr (WIDTH == 8) return u;
        else return sgn ? ((u << (64 - 8 * WIDTH)) >> (64 - 8 * WIDTH)) : u;
    }
};
template <int T> struct PackedCol {
    const void* p;
    uint32_t W, shift, offset;
    uint64_t reference;
    bool sgn;
    __host__ __device__ explicit PackedCol(const IntCol& c)
        : p(c.p), W(c.W), shift(c.shift), offset(c.offset), reference(c.reference), sgn(c.sgn) {}
    __device__ __forceinline__ int64_t operator()(uint64_t i) const {
        return fl_get<T>(p, W, shift, offset, reference, sgn, i);
    }
};

// Runtime reader (one element per thread, e.g. patch indices): uniform branches only.
__device__ __forceinline__ int64_t intcol_get(const IntCol& c, uint64_t i) {
    if (c.packed) {
        return c.width == 4 ? fl_get<32>(c.p, c.W, c.shift, c.offset, c.reference, c.sgn, i)
                            : fl_get<64>(c.p, c.W, c.shift, c.offset, c.reference, c.sgn, i);
    }
    switch (c.width) {
    case 1: return c.sgn ? ld<1, true>(c.p, i) : ld<1, false>(c.p, i);
    case 2: return c.sgn ? ld<2, true>(c.p, i) : ld<2, false>(c.p, i);
    case 4: return c.sgn ? ld<4, true>(c.p, i) : ld<4, false>(c.p, i);
    default: return ld<8, true>(c.p, i);
    }
}

}  // namespace vxg
