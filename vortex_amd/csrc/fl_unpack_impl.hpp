// fl_unpack_impl.hpp — K1: FastLanes bit-unpack for CDNA4 (gfx950) with fused epilogues.
//
// Restates fastlanes 0.1.8 `BitPacking::unchecked_unpack` as used by
// encodings/fastlanes/src/bitpacking/compress.rs:209-273 (unpack_primitive), fused with the
// cascades the reference runs as separate materialised passes:
//   FoR       for/compress.rs:100-117           out = (v << shift) wrapping_add reference
//   ZigZag    zigzag/compress.rs:35-57          out = (u >> 1) ^ -(u & 1)
//   ALP       alp/mod.rs:161-163, compress.rs:98-106   out = ((float)enc * F10[f]) * IF10[e]
//   Dict      dict/array.rs:68-73 -> primitive/compute/take.rs:58-67   out = values[code]
//
// Work decomposition (MI355X-first):
//   * A FastLanes block (1024 values of T bits) stores W "word rows" of 128 bytes each
//     (word w of lane l at packed[l + LANES*w]).  Every word row is 1024 bits for every T.
//   * 8 threads own one block; thread t owns byte slice [16t, 16t+16) of every word row,
//     i.e. 16/sizeof(T) adjacent lanes.  It issues W independent 16-byte loads (one
//     global_load_dwordx4 per word row; 8 threads = one full 128-byte line) and keeps them in
//     VGPRs for the whole block: every packed byte is read from HBM exactly once.
//   * Rows are extracted lane-parallel inside 32-bit (T<=32) or 64-bit (T=64) registers
//     (SWAR: T-bit lanes never leak because every shift is followed by a per-lane mask).
//   * Row r of the thread's lanes lands at out[index(r, lane0) .. +16/sizeof(T)) — 16
//     contiguous bytes — so every output row is one global_store_dwordx4 and 8 threads write
//     one full 128-byte line.  A 64-lane wave covers 8 blocks = 8 KiB of u32 output.
//   * W and T are template parameters: all shifts/masks fold to immediates, the packed words
//     stay in registers (no scratch), and the row loop is fully unrolled.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "vxg_internal.hpp"
#include "intcol.hpp"

namespace vxg {

template <int T> struct Fl;
template <> struct Fl<8> {
    using E = uint8_t;  using U = uint32_t;
    static constexpr uint32_t rep(uint32_t m) { return m * 0x01010101u; }
};
template <> struct Fl<16> {
    using E = uint16_t; using U = uint32_t;
    static constexpr uint32_t rep(uint32_t m) { return m * 0x00010001u; }
};
template <> struct Fl<32> {
    using E = uint32_t; using U = uint32_t;
    static constexpr uint32_t rep(uint32_t m) { return m; }
};
template <> struct Fl<64> {
    using E = uint64_t; using U = uint64_t;
    static constexpr uint64_t rep(uint64_t m) { return m; }
};

template <typename U> __host__ __device__ constexpr U low_mask(int bits) {
    return bits >= int(8 * sizeof(U)) ? ~U(0) : ((U(1) << bits) - U(1));
}

template <int VW> struct VType;
template <> struct VType<0> { using t = uint8_t; };  // placeholder for non-Dict epilogues
template <> struct VType<1> { using t = uint8_t; };
template <> struct VType<2> { using t = uint16_t; };
template <> struct VType<4> { using t = uint32_t; };
template <> struct VType<8> { using t = uint64_t; };
template <> struct VType<16> { using t = uint4; };

// 16 bytes of lane data held as NV words of U.
template <int T> struct Vec16 {
    using U = typename Fl<T>::U;
    static constexpr int NV = 16 / sizeof(U);
    U w[NV];
    __device__ __forceinline__ typename Fl<T>::E elem(int j) const {
        using E = typename Fl<T>::E;
        if constexpr (T == 64) {
            return w[j];
        } else {
            constexpr int PER = 32 / T;
            return E((w[j / PER] >> ((j % PER) * T)) & low_mask<uint32_t>(T));
        }
    }
};

template <int T>
__device__ __forceinline__ Vec16<T> load16(const uint8_t* p) {
    Vec16<T> v;
    uint4 q = *reinterpret_cast<const uint4*>(p);
    static_assert(sizeof(v.w) == 16, "");
    __builtin_memcpy(v.w, &q, 16);
    return v;
}
// load16 from global memory through a pointer the compiler cannot place (read from a table)
template <int T>
__device__ __forceinline__ Vec16<T> load16_global(const uint8_t* p) {
    Vec16<T> v;
    const uint4 q = gload(reinterpret_cast<const uint4*>(p));
    __builtin_memcpy(v.w, &q, 16);
    return v;
}


// Extract row R of W-bit values from the register-resident word rows (SWAR over lanes).
template <int T, int W, int R>
__device__ __forceinline__ Vec16<T> extract_row(const Vec16<T>* p) {
    using U = typename Fl<T>::U;
    constexpr int NV = Vec16<T>::NV;
    Vec16<T> v;
    if constexpr (W == 0) {
#pragma unroll
        for (int k = 0; k < NV; k++) v.w[k] = 0;
    } else if constexpr (W == T) {
        v = p[R];
    } else {
        constexpr int start = R * W, word = start / T, shift = start % T;
        if constexpr (shift + W <= T) {
            constexpr U m = Fl<T>::rep(low_mask<U>(W));
#pragma unroll
            for (int k = 0; k < NV; k++) v.w[k] = (p[word].w[k] >> shift) & m;
        } else {
            constexpr int cur = T - shift;
            constexpr U mlo = Fl<T>::rep(low_mask<U>(cur));
            constexpr U mhi = Fl<T>::rep(low_mask<U>(W - cur));
#pragma unroll
            for (int k = 0; k < NV; k++)
                v.w[k] = ((p[word].w[k] >> shift) & mlo) | ((p[word + 1].w[k] & mhi) << cur);
        }
    }
    return v;
}

struct EpiParams {
    uint64_t reference;
    uint32_t shift;
    double alp_a, alp_b;
    const void* dict;
    uint64_t dict_len;
    uint32_t* err;
    bool dict_lds = false;  // dict points into LDS (a staged dictionary), else global memory
};

inline EpiParams to_epi(const UnpackArgs& a) {
    EpiParams ep;
    ep.reference = a.reference;
    ep.shift = a.shift;
    ep.alp_a = a.alp_a;
    ep.alp_b = a.alp_b;
    ep.dict = a.dict;
    ep.dict_len = a.dict_len;
    ep.err = a.err;
    return ep;
}

template <int T, Epi EPI, int VW> struct EpiOut {
    using type = typename Fl<T>::E;
};
template <int T, int VW> struct EpiOut<T, Epi::AlpF32, VW> { using type = float; };
template <int T, int VW> struct EpiOut<T, Epi::AlpF64, VW> { using type = double; };
template <int T, int VW> struct EpiOut<T, Epi::Dict, VW> { using type = typename VType<VW>::t; };

// Apply the epilogue to one element.  Dict: an out-of-range code reads entry 0 and sets `oob`
// (reported once per thread, not one branch + atomic per element).
template <int T, Epi EPI, int VW>
__device__ __forceinline__ typename EpiOut<T, EPI, VW>::type apply_epi(typename Fl<T>::E e,
                                                                      const EpiParams& ep, bool& oob) {
    using E = typename Fl<T>::E;
    if constexpr (EPI == Epi::Plain) {
        return e;
    } else if constexpr (EPI == Epi::For || EPI == Epi::ForZigZag) {
        E v = E(E(e << ep.shift) + E(ep.reference));  // wrapping in T
        if constexpr (EPI == Epi::ForZigZag) v = E((v >> 1) ^ E(E(0) - E(v & 1)));
        return v;
    } else if constexpr (EPI == Epi::AlpF32) {
        static_assert(T == 32, "ALP f32 decodes i32");
        E v = E(E(e << ep.shift) + E(ep.reference));
        float x = float(int32_t(v));                 // v_cvt_f32_i32: RN
        x = __fmul_rn(x, float(ep.alp_a));           // F10[f]
        return __fmul_rn(x, float(ep.alp_b));        // IF10[e]
    } else if constexpr (EPI == Epi::AlpF64) {
        static_assert(T == 64, "ALP f64 decodes i64");
        E v = E(E(e << ep.shift) + E(ep.reference));
        double x = double(int64_t(v));               // exact hi*2^32 + lo, one RN rounding
        x = __dmul_rn(x, ep.alp_a);
        return __dmul_rn(x, ep.alp_b);
    } else {  // Dict gather
        using VT = typename VType<VW>::t;
        const uint64_t c = uint64_t(e);
        const bool bad = c >= ep.dict_len;
        oob |= bad;
        const VT* p = static_cast<const VT*>(ep.dict) + (bad ? 0 : c);
        return ep.dict_lds ? lds_load(p) : gload(p);
    }
}

template <int T, Epi EPI, int VW>
__device__ __forceinline__ typename EpiOut<T, EPI, VW>::type apply_epi(typename Fl<T>::E e,
                                                                      const EpiParams& ep) {
    bool oob = false;
    const auto r = apply_epi<T, EPI, VW>(e, ep, oob);
    if (oob) __hip_atomic_fetch_or(ep.err, kErrTakeOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return r;
}

// Thread-per-output extraction from LDS-staged blocks with a RUNTIME bit width (K1g, K14): thread
// t produces values i = 256 k + t (k < 4) of every block.  For LANES <= 256 the lane (i % LANES)
// and the FL_ORDER group of i do not depend on k, and the row advances by 2 per k, so the bit
// offset is start0 + 2 k W: one 24-bit multiply per thread instead of one per value.  Both words
// of a value are read and combined branch-free (v_alignbit for T <= 32).
template <int T>
struct RtRows {
    using E = typename Fl<T>::E;
    static constexpr uint32_t LANES = 1024 / T;
    uint32_t lane, start0, W;
    E mask;
    __device__ __forceinline__ explicit RtRows(uint32_t w) : W(w) {
        const uint32_t t = threadIdx.x;  // value t of the block (k = 0)
        lane = t % LANES;
        const uint32_t fl = ((t & 127) - lane) >> 4;
        const uint32_t row = (((fl & 1) << 2) | (fl & 2) | (fl >> 2)) * 8 + (t >> 7);  // FL_ORDER[fl]*8 + s
        start0 = __umul24(row, w);
        mask = w >= uint32_t(T) ? E(~E(0)) : E((E(1) << w) - E(1));
    }
    // value 256 k + threadIdx.x of the block whose words start at pw (LDS)
    __device__ __forceinline__ E get(const E* __restrict__ pw, uint32_t k) const {
        if constexpr (T == 64) {
            const uint32_t start = start0 + 2 * k * W, w0 = start >> 6, sh = start & 63;
            const uint32_t w1 = w0 + 1 < W ? w0 + 1 : w0;
            const uint64_t lo = pw[LANES * w0 + lane], hi = pw[LANES * w1 + lane];
            return (sh ? (lo >> sh) | (hi << (64 - sh)) : lo) & mask;
        } else {
            constexpr uint32_t LT = T == 32 ? 5 : (T == 16 ? 4 : 3);
            const uint32_t start = start0 + 2 * k * W, w0 = start >> LT, sh = start & (T - 1);
            const uint32_t w1 = w0 + 1 < W ? w0 + 1 : w0;
            const uint32_t lo = pw[LANES * w0 + lane], hi = pw[LANES * w1 + lane];
            if constexpr (T == 32) return E(__builtin_amdgcn_alignbit(hi, lo, sh) & mask);
            else return E(((lo | (hi << T)) >> sh) & mask);
        }
    }
};

// Output store policy of the K1 launches (1 = non-temporal streaming stores; a
// -DVXG_OUT_NT=0 build is the A/B variant with plain stores).
#ifndef VXG_OUT_NT
#define VXG_OUT_NT 1
#endif
constexpr int kOutNT = VXG_OUT_NT;

// Store N bytes (compile-time) from a register array using the widest aligned stores.
// NT = 1: non-temporal (streaming) 16-byte stores for the decoded output.
template <int NBYTES, int NT = 0>
__device__ __forceinline__ void store_bytes(uint8_t* dst, const void* src) {  // dst: global memory
    using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
    if constexpr (NBYTES >= 16) {
#pragma unroll
        for (int i = 0; i < NBYTES / 16; i++) {
            u32x4 vv;
            __builtin_memcpy(&vv, static_cast<const uint8_t*>(src) + 16 * i, 16);
            if constexpr (NT) __builtin_nontemporal_store(vv, (gptr<u32x4>)dst + i);
            else ((gptr<u32x4>)dst)[i] = vv;
        }
    } else if constexpr (NBYTES == 8) {
        uint64_t q; __builtin_memcpy(&q, src, 8); *(gptr<uint64_t>)dst = q;
    } else if constexpr (NBYTES == 4) {
        uint32_t q; __builtin_memcpy(&q, src, 4); *(gptr<uint32_t>)dst = q;
    } else if constexpr (NBYTES == 2) {
        uint16_t q; __builtin_memcpy(&q, src, 2); *(gptr<uint16_t>)dst = q;
    } else {
        *(gptr<uint8_t>)dst = *static_cast<const uint8_t*>(src);
    }
}

// One output row R of this thread's 16-byte lane slice.  FULL (compile time): the block lands
// entirely inside [0, len) with 16-byte alignment -> one unconditional 16-byte store.
template <int T, int W, Epi EPI, int VW, int NT, int R, bool FULL>
__device__ __forceinline__ void process_row(const Vec16<T>* p, int lane0,
                                            typename EpiOut<T, EPI, VW>::type* __restrict__ out,
                                            int64_t out_base, uint64_t len, const EpiParams& ep, bool& oob) {
    using E = typename Fl<T>::E;
    using O = typename EpiOut<T, EPI, VW>::type;
    constexpr int EPV = 16 / int(sizeof(E));  // elements per 16-byte lane slice
    const Vec16<T> v = extract_row<T, W, R>(p);
    const int idx = fl_index(R, lane0);
    if constexpr (FULL) {
        O* dst = out + (out_base + idx);
        if constexpr (EPI == Epi::Plain) {
            store_bytes<16, NT>(reinterpret_cast<uint8_t*>(dst), v.w);
        } else {
            O o[EPV];
#pragma unroll
            for (int j = 0; j < EPV; j++) o[j] = apply_epi<T, EPI, VW>(v.elem(j), ep, oob);
            store_bytes<EPV * int(sizeof(O)), NT>(reinterpret_cast<uint8_t*>(dst), o);
        }
    } else {
#pragma unroll
        for (int j = 0; j < EPV; j++) {
            const int64_t o = out_base + idx + j;
            if (o >= 0 && uint64_t(o) < len) gstore(out + o, apply_epi<T, EPI, VW>(v.elem(j), ep, oob));
        }
    }
}

template <int T, int W, Epi EPI, int VW, int NT, bool FULL, int... Rs>
__device__ __forceinline__ void process_rows(const Vec16<T>* p, int lane0,
                                             typename EpiOut<T, EPI, VW>::type* __restrict__ out,
                                             int64_t out_base, uint64_t len, const EpiParams& ep, bool& oob,
                                             std::integer_sequence<int, Rs...>) {
    (process_row<T, W, EPI, VW, NT, Rs, FULL>(p, lane0, out, out_base, len, ep, oob), ...);
}

// Decode one FastLanes block: this thread's 16-byte lane slice `t` of every word row.
// out_base = output index of the block's packed position 0 (negative for the first block of
// a slice with offset > 0); `full` = the whole block lands inside [0, len) with 16-B alignment.
template <int T, int W, Epi EPI, int VW, int NT = 0>
__device__ __forceinline__ void unpack_block(const uint8_t* __restrict__ blk_packed, int t,
                                             typename EpiOut<T, EPI, VW>::type* __restrict__ out,
                                             int64_t out_base, bool full, uint64_t len,
                                             const EpiParams& ep) {
    using E = typename Fl<T>::E;
    constexpr int EPV = 16 / int(sizeof(E));
    constexpr int NW = W > 0 ? W : 1;
    Vec16<T> p[NW];
    if constexpr (W > 0) {
#pragma unroll
        for (int w = 0; w < W; w++) p[w] = load16<T>(blk_packed + 128 * w + 16 * t);
    }
    bool oob = false;
    if (full)  // unswitched: the full-block path is straight-line code
        process_rows<T, W, EPI, VW, NT, true>(p, t * EPV, out, out_base, len, ep, oob,
                                              std::make_integer_sequence<int, T>{});
    else
        process_rows<T, W, EPI, VW, NT, false>(p, t * EPV, out, out_base, len, ep, oob,
                                               std::make_integer_sequence<int, T>{});
    if constexpr (EPI == Epi::Dict)
        if (oob) __hip_atomic_fetch_or(ep.err, kErrTakeOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Rows [Q*T/S, (Q+1)*T/S) of a block (row split S, quarter Q): only the word rows those rows
// read are loaded.  Used by small launches (few blocks) to put 4x more threads on the array.
template <int T, int W, Epi EPI, int VW, int NT, int S, int Q, bool FULL, int... Rs>
__device__ __forceinline__ void process_rows_part(const Vec16<T>* p, int lane0,
                                                  typename EpiOut<T, EPI, VW>::type* __restrict__ out,
                                                  int64_t out_base, uint64_t len, const EpiParams& ep, bool& oob,
                                                  std::integer_sequence<int, Rs...>) {
    (process_row<T, W, EPI, VW, NT, Q * (T / S) + Rs, FULL>(p, lane0, out, out_base, len, ep, oob), ...);
}

template <int T, int W, Epi EPI, int VW, int NT, int S, int Q>
__device__ __forceinline__ void unpack_block_part(const uint8_t* __restrict__ blk_packed, int t,
                                                  typename EpiOut<T, EPI, VW>::type* __restrict__ out,
                                                  int64_t out_base, bool full, uint64_t len,
                                                  const EpiParams& ep) {
    using E = typename Fl<T>::E;
    constexpr int EPV = 16 / int(sizeof(E));
    constexpr int NW = W > 0 ? W : 1;
    constexpr int R0 = Q * (T / S), R1 = (Q + 1) * (T / S);
    constexpr int WLO = W > 0 ? (R0 * W) / T : 0;
    constexpr int WHI = W > 0 ? (R1 * W - 1) / T : 0;  // inclusive
    Vec16<T> p[NW];
    if constexpr (W > 0) {
#pragma unroll
        for (int w = WLO; w <= WHI && w < W; w++) p[w] = load16<T>(blk_packed + 128 * w + 16 * t);
    }
    bool oob = false;
    if (full)
        process_rows_part<T, W, EPI, VW, NT, S, Q, true>(p, t * EPV, out, out_base, len, ep, oob,
                                                         std::make_integer_sequence<int, T / S>{});
    else
        process_rows_part<T, W, EPI, VW, NT, S, Q, false>(p, t * EPV, out, out_base, len, ep, oob,
                                                          std::make_integer_sequence<int, T / S>{});
    if constexpr (EPI == Epi::Dict)
        if (oob) __hip_atomic_fetch_or(ep.err, kErrTakeOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Dictionaries up to this size are staged into LDS by every workgroup of a Dict launch: a
// gather of 64 random 8-byte entries from global memory touches up to 64 cache lines (one
// TA cycle each), from LDS it is one ds_read_b64 with bank conflicts.
constexpr int kDictLdsBytes = 16 * 1024;

template <int VW>
__device__ __forceinline__ void stage_dict(uint8_t* s_dict, const void* dict, uint64_t dict_len) {
    // 16-byte aligned chunks (the last may run past the dictionary inside its aligned chunk)
    const int n16 = int((dict_len * VW + 15) / 16);
    for (int q = threadIdx.x; q < n16; q += blockDim.x)
        reinterpret_cast<uint4*>(s_dict)[q] = static_cast<const uint4*>(dict)[q];
    __syncthreads();
}

// One launch decodes up to kArgChunks independent arrays ("chunks": a single array, or the
// chunks of a ChunkedArray written straight into their output slices -- chunked/canonical.rs:
// 170-187 without the pack copy).  The chunk table travels as the kernel argument (no upload,
// no host synchronisation); each workgroup of 256 threads covers 32 FastLanes blocks of exactly
// one chunk, found by a workgroup-uniform binary search on first_group (no search for n = 1).
// S = 1: 8 threads per block, 32 blocks per workgroup (large launches).  S = 4 (T = 32/64):
// each wave takes one quarter of the rows of 8 blocks -> 8 blocks per workgroup and 4x the
// threads, for launches too small to fill 256 CUs (the quarter is wave-uniform, no divergence).
template <int T, int W, Epi EPI, int VW, bool LDSD, int S>
__device__ __forceinline__ void unpack_chunk(const ChunkDev& c, uint64_t g, uint32_t* err) {
    using O = typename EpiOut<T, EPI, VW>::type;
    constexpr int BPG = 32 / S;  // blocks per workgroup
    const uint64_t blk = (g - c.first_group) * BPG + ((threadIdx.x >> 3) % BPG);
    const int t = int(threadIdx.x & 7);
    EpiParams ep;
    ep.reference = c.reference;
    ep.shift = c.shift;
    ep.alp_a = c.alp_a;
    ep.alp_b = c.alp_b;
    ep.dict = c.dict;
    ep.dict_len = c.dict_len;
    ep.err = err;
    if constexpr (LDSD) {  // the whole workgroup is in this chunk
        __shared__ __attribute__((aligned(16))) uint8_t s_dict[kDictLdsBytes];
        stage_dict<VW>(s_dict, c.dict, c.dict_len);
        ep.dict = s_dict;
        ep.dict_lds = true;
    }
    if (blk >= c.n_blocks) return;
    const int64_t out_base = int64_t(blk * 1024) - int64_t(c.offset);
    // full: straight-line 16-byte stores (block inside [0, len), 16-byte aligned slice)
    const bool full =
        c.offset == 0 && (blk + 1) * 1024 <= c.len && (reinterpret_cast<uintptr_t>(c.out) & 15) == 0;
    // Decoded output is written once and never re-read by this launch: non-temporal 16-byte
    // stores (measured on C1: 51.1 us vs 63.0 us with plain stores = 80% vs 65% of 8 TB/s,
    // profiles/r01_ubench_k1.txt; a perfectly coalesced copy of the same bytes: 49.2 us).
    const uint8_t* bp = c.packed + blk * (128 * W);
    if constexpr (S == 1) {
        unpack_block<T, W, EPI, VW, kOutNT>(bp, t, static_cast<O*>(c.out), out_base, full, c.len, ep);
    } else {
        static_assert(S == 4, "row split 1 or 4");
        switch (threadIdx.x >> 6) {  // wave-uniform quarter
        case 0: unpack_block_part<T, W, EPI, VW, kOutNT, 4, 0>(bp, t, static_cast<O*>(c.out), out_base, full, c.len, ep); break;
        case 1: unpack_block_part<T, W, EPI, VW, kOutNT, 4, 1>(bp, t, static_cast<O*>(c.out), out_base, full, c.len, ep); break;
        case 2: unpack_block_part<T, W, EPI, VW, kOutNT, 4, 2>(bp, t, static_cast<O*>(c.out), out_base, full, c.len, ep); break;
        default: unpack_block_part<T, W, EPI, VW, kOutNT, 4, 3>(bp, t, static_cast<O*>(c.out), out_base, full, c.len, ep); break;
        }
    }
}

// ---------------------------------------------------------------------------- K1w
// The large-launch K1: burst read + wave-contiguous stores.  Measured on C1 (tools/ubench_k1.hip,
// profiles/r03_ubench_k1.txt): a copy of C1's bytes whose workgroups first read their whole
// input into LDS and then write their output 1 KiB per store instruction runs 54.6 us against
// 59.6 us for the same copy with reads and writes interleaved per wave, and K1 with this shape
// ran 57.1 us against 60.5 us for the register-resident K1 (whose store instruction writes
// 8 x 128 B at a 4 KiB stride).  So:
//   * a workgroup stages the packed words of BPW consecutive blocks of one chunk (~32 KiB) into
//     LDS with coalesced 16-byte loads, then decodes them: wave v takes BPW/4 consecutive
//     blocks (a contiguous output range);
//   * all 64 lanes of a wave work on ONE block at a time: in store k, lane group g (8 lanes)
//     produces the row whose 128 output bytes are slot 8k + g of the block and lane t its
//     16-byte slice, so every store instruction writes 1 KiB contiguous (T/8 stores per block);
//   * the row -- hence the bit offset -- differs per lane group: each 16-byte slice is funnel-
//     shifted out of the two LDS word rows holding it (runtime shift, per-lane SWAR masks).
//   * the packed words live in LDS, not VGPRs: T = 64, W = 24 (C2) drops from 110 VGPRs
//     (4 waves/SIMD) to a few dozen.
// blocks per workgroup: ~32 KiB of packed words (16 KiB when a dictionary shares the LDS)
constexpr int kw_bpw(int W, bool lds_dict = false) {
    const int b = ((lds_dict ? 16 : 32) * 1024) / (128 * (W > 0 ? W : 1));
    const int b4 = (b / 4) * 4;
    return b4 < 4 ? 4 : (b4 > 32 ? 32 : b4);
}

// Row whose 128 output bytes are 128-byte slot q of a block: row r = o*8 + s sits at slot
// FL_ORDER[o] * T/64 + s * T/8 (fl_index in bytes / 128), and FL_ORDER is its own inverse.
template <int T>
__device__ __forceinline__ int kw_row(int q) {
    constexpr int P = T / 8;
    const int s = q / P, f = (q % P) * (64 / T);
    const int o = ((f & 1) << 2) | (f & 2) | (f >> 2);
    return o * 8 + s;
}

template <typename U>
__device__ __forceinline__ U kw_mask(int n) {
    return n >= int(8 * sizeof(U)) ? ~U(0) : ((U(1) << n) - U(1));
}

// Row r of this lane's 16-byte lane slice t from a block's packed words in LDS.
template <int T, int W>
__device__ __forceinline__ Vec16<T> kw_extract(const uint8_t* blk, int r, int t) {
    using U = typename Fl<T>::U;
    constexpr int NV = Vec16<T>::NV;
    Vec16<T> v;
    if constexpr (W == 0) {
#pragma unroll
        for (int k = 0; k < NV; k++) v.w[k] = 0;
    } else {
        const int start = r * W, w0 = start / T, sh = start % T;
        const Vec16<T> lo = load16<T>(blk + w0 * 128 + 16 * t);  // ds_read_b128
        if constexpr (W == T) {
            v = lo;
        } else {
            // word w0 + 1 may be the next block's (or the LDS slack): its bits are masked off
            const Vec16<T> hi = load16<T>(blk + (w0 + 1) * 128 + 16 * t);
            const int cur = T - sh;                  // bits of the value held by word w0
            const int nlo = cur < W ? cur : W, nhi = W - nlo;
            const U mlo = Fl<T>::rep(kw_mask<U>(nlo)), mhi = Fl<T>::rep(kw_mask<U>(nhi));
            const int hs = cur & (int(8 * sizeof(U)) - 1);  // == cur whenever mhi != 0
#pragma unroll
            for (int k = 0; k < NV; k++) v.w[k] = ((lo.w[k] >> sh) & mlo) | ((hi.w[k] & mhi) << hs);
        }
    }
    return v;
}

template <int T, int W, Epi EPI, int VW, int NT>
__device__ __forceinline__ void kw_block(const uint8_t* pk, int gq, int t, typename EpiOut<T, EPI, VW>::type* __restrict__ out,
                                         int64_t out_base, bool full, uint64_t len, const EpiParams& ep, bool& oob) {
    using E = typename Fl<T>::E;
    using O = typename EpiOut<T, EPI, VW>::type;
    constexpr int EPV = 16 / int(sizeof(E));
#pragma unroll
    for (int k = 0; k < T / 8; k++) {
        const int q = 8 * k + gq;
        const Vec16<T> v = kw_extract<T, W>(pk, kw_row<T>(q), t);
        const int idx = q * (1024 / T) + t * EPV;  // element index of the slice in the block
        if (full) {
            O* dst = out + (out_base + idx);
            if constexpr (EPI == Epi::Plain) {
                store_bytes<16, NT>(reinterpret_cast<uint8_t*>(dst), v.w);
            } else {
                O o[EPV];
#pragma unroll
                for (int j = 0; j < EPV; j++) o[j] = apply_epi<T, EPI, VW>(v.elem(j), ep, oob);
                store_bytes<EPV * int(sizeof(O)), NT>(reinterpret_cast<uint8_t*>(dst), o);
            }
        } else {
#pragma unroll
            for (int j = 0; j < EPV; j++) {
                const int64_t o = out_base + idx + j;
                if (o >= 0 && uint64_t(o) < len) gstore(out + o, apply_epi<T, EPI, VW>(v.elem(j), ep, oob));
            }
        }
    }
}

// LDS of a K1w workgroup: the packed words (+ one word row of slack), then (LDSD) the dictionary
// -- dynamic, sized by the launch to the largest dictionary of its table.
template <int W, bool LDSD>
constexpr int kw_packed_lds() {
    return (W > 0 ? kw_bpw(W, LDSD) * 128 * W : 0) + 128;
}

// First patch (ascending keys idx[i] - idx_off) whose key is >= x: a 256-ary search by the whole
// workgroup, one memory round trip per round (3 rounds for 2^24 patches).  `s_cnt`: 4 LDS words.
__device__ __forceinline__ uint64_t patch_lower_bound(const PatchCol& pc, uint64_t x, uint32_t* s_cnt) {
    uint64_t lo = 0, hi = pc.n;  // the answer is in [lo, hi]
    while (lo < hi) {            // workgroup-uniform
        const uint64_t step = (hi - lo + 255) / 256;
        const uint64_t i = lo + uint64_t(threadIdx.x) * step;
        const bool below = i < hi && uint64_t(intcol_get(pc.idx, i)) - pc.idx_off < x;
        const uint32_t cw = uint32_t(__popcll(__ballot(below)));
        if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = cw;
        __syncthreads();
        const uint64_t cnt = uint64_t(s_cnt[0]) + s_cnt[1] + s_cnt[2] + s_cnt[3];
        __syncthreads();
        // samples 0 .. cnt-1 are below x: the answer is in (lo + (cnt-1) step, lo + cnt step]
        if (cnt == 0) {
            hi = lo;
        } else {
            const uint64_t nhi = lo + cnt * step;
            lo = lo + (cnt - 1) * step + 1;
            hi = nhi < hi ? nhi : hi;
        }
    }
    return lo;
}

template <int T, int W, Epi EPI, int VW, bool LDSD>
__device__ __forceinline__ void unpack_chunk_w(const ChunkDev& c, uint64_t g, uint32_t* err, const PatchCol& pc,
                                               uint32_t bpw_rt) {
    using O = typename EpiOut<T, EPI, VW>::type;
    constexpr int BPW_MAX = kw_bpw(W, LDSD);
    // blocks per workgroup: the width's maximum (~32 KiB of packed words), or fewer for a launch
    // too small to fill the chip with it (launch_w)
    const int BPW = bpw_rt ? int(bpw_rt) : BPW_MAX;
    extern __shared__ __attribute__((aligned(16))) uint8_t k1w_lds[];
    uint8_t* const s_pk = k1w_lds;
    EpiParams ep;
    ep.reference = c.reference;
    ep.shift = c.shift;
    ep.alp_a = c.alp_a;
    ep.alp_b = c.alp_b;
    ep.dict = c.dict;
    ep.dict_len = c.dict_len;
    ep.err = err;
    if constexpr (LDSD) {  // the whole workgroup is in this chunk
        uint8_t* const s_dict = k1w_lds + kw_packed_lds<W, LDSD>();
        stage_dict<VW>(s_dict, c.dict, c.dict_len);
        ep.dict = s_dict;
        ep.dict_lds = true;
    }
    const uint64_t blk0 = (g - c.first_group) * BPW;
    const int nb = c.n_blocks - blk0 < uint64_t(BPW) ? int(c.n_blocks - blk0) : BPW;
    // Fused patches: the raw words of a 256-patch window around where the workgroup's output
    // range [olo, ohi) falls if the patches are spread evenly, loaded before the burst and used
    // only after the decode (no wait in between: 8-byte index words, plain or FastLanes-packed,
    // loaded unconditionally).  When the window brackets the range, each thread holds at most one
    // of the workgroup's patches and stores it after the decode; otherwise the range is found by
    // patch_lower_bound.  Scratch: the LDS slack row, whose bytes kw_extract always masks off.
    uint32_t* const s_pscr = reinterpret_cast<uint32_t*>(k1w_lds + (W > 0 ? BPW * 128 * W : 0));
    const bool patched = pc.n != 0;
    uint64_t olo = 0, ohi = 0, pbase = 0, pw0 = 0, pw1 = 0;
    uint32_t psh = 0;
    O pval{};
    if (patched) {
        const uint64_t s0 = blk0 * 1024, s1 = (blk0 + uint64_t(nb)) * 1024;
        olo = s0 > c.offset ? s0 - c.offset : 0;
        ohi = s1 - c.offset < c.len ? s1 - c.offset : c.len;
        const uint64_t guess = uint64_t(double(olo) * double(pc.n) / double(c.len));
        pbase = guess > 128 ? guess - 128 : 0;
        if (pbase + 256 > pc.n) pbase = pc.n > 256 ? pc.n - 256 : 0;
        const uint64_t i0 = pbase + threadIdx.x, i = i0 < pc.n ? i0 : pc.n - 1;
        const uint64_t* ip = static_cast<const uint64_t*>(pc.idx.p);
        uint64_t a0 = i, a1 = i;
        if (pc.idx.packed) {  // fl_word_pair<64>'s two word indices
            const uint64_t g2 = i + pc.idx.offset;
            const uint32_t e = uint32_t(g2 & 1023), lane = e % 16, s = e >> 7;
            const uint32_t fl = ((e & 127) - lane) >> 4;
            const uint32_t row = (((fl & 1) << 2) | (fl & 2) | (fl >> 2)) * 8 + s;
            const uint32_t start = __umul24(row, pc.idx.W), word = start / 64;
            psh = start % 64;
            const uint64_t blk = (g2 >> 10) * (16ull * pc.idx.W);
            a0 = blk + 16ull * word + lane;
            a1 = blk + 16ull * (word + 1 < pc.idx.W ? word + 1 : word) + lane;
        }
        pw0 = ip[a0];
        pw1 = ip[a1];
        pval = static_cast<const O*>(pc.vals)[i];
    }
    if constexpr (W > 0) {  // burst: the workgroup's packed words, coalesced 16-byte loads
        // non-temporal: every packed byte is read once (a copy with this shape: 55.1 -> 53.0 us,
        // profiles/r03_ubench_k1.txt)
        using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
        const gptr<const u32x4> src = (gptr<const u32x4>)(c.packed + blk0 * (128 * W));
#if VXG_K1W_BURST
        // A/B variant (VXG_K1W_BURST=1 build): a full workgroup issues all PQ of its thread's
        // loads before any LDS write (PQ * 4 VGPRs; the default loop keeps one load in flight)
        constexpr int NQ = BPW_MAX * 8 * W, PQ = (NQ + 255) / 256;
        if (nb == BPW_MAX) {
            u32x4 v[PQ];
#pragma unroll
            for (int p = 0; p < PQ; p++) {
                const int q = int(threadIdx.x) + 256 * p;
                v[p] = __builtin_nontemporal_load(src + (q < NQ ? q : NQ - 1));
            }
#pragma unroll
            for (int p = 0; p < PQ; p++) {
                const int q = int(threadIdx.x) + 256 * p;
                if (q < NQ) reinterpret_cast<uint4*>(s_pk)[q] = make_uint4(v[p][0], v[p][1], v[p][2], v[p][3]);
            }
        } else
#endif
        for (int q = threadIdx.x; q < nb * 8 * W; q += 256) {
            const u32x4 v = __builtin_nontemporal_load(src + q);
            reinterpret_cast<uint4*>(s_pk)[q] = make_uint4(v[0], v[1], v[2], v[3]);
        }
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, gq = lane >> 3, t = lane & 7;
    O* const out = static_cast<O*>(c.out);
    const bool aligned = (reinterpret_cast<uintptr_t>(c.out) & 15) == 0;
    bool oob = false;
    const int PER = (BPW + 3) / 4;  // blocks per wave (the last waves may have fewer)
    for (int j = 0; j < PER; j++) {
        const int b = wave * PER + j;
        if (b >= nb) break;  // wave-uniform
        const uint64_t blk = blk0 + b;
        const int64_t out_base = int64_t(blk * 1024) - int64_t(c.offset);
        const bool full = c.offset == 0 && (blk + 1) * 1024 <= c.len && aligned;
        kw_block<T, W, EPI, VW, kOutNT>(s_pk + b * 128 * W, gq, t, out, out_base, full, c.len, ep, oob);
    }
    if constexpr (EPI == Epi::Dict)
        if (oob) __hip_atomic_fetch_or(err, kErrTakeOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (patched) {
        // the window's words are used from here on (keeps the compiler from hoisting their use,
        // and its wait, above the decode)
        asm volatile("" : "+v"(pw0), "+v"(pw1));
        uint64_t pkey = pw0;
        if (pc.idx.packed) {  // fl_get<64>
            const uint64_t mask = pc.idx.W >= 64 ? ~0ull : ((1ull << pc.idx.W) - 1);
            const uint64_t v = pc.idx.W ? ((psh ? (pw0 >> psh) | (pw1 << (64 - psh)) : pw0) & mask) : 0;
            pkey = (v << pc.idx.shift) + pc.idx.reference;
        }
        const bool valid = pbase + threadIdx.x < pc.n;
        pkey = valid ? pkey - pc.idx_off : ~0ull;
        const bool pin = pkey >= olo && pkey < ohi;
        // the window brackets [olo, ohi): nothing before it is >= olo, nothing after it < ohi
        if (threadIdx.x == 0) s_pscr[0] = pbase == 0 || pkey < olo;
        if (threadIdx.x == 255) s_pscr[1] = pbase + 256 >= pc.n || pkey >= ohi;
        // keys ascending inside the window (a cheap check of the invariant the search relies on)
        const uint64_t nk = __shfl_down(pkey, 1, 64);
        if ((threadIdx.x & 63) != 63 && pbase + threadIdx.x + 1 < pc.n && nk < pkey)
            __hip_atomic_fetch_or(err, kErrPatchOrder, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (g == c.first_group && threadIdx.x == 0) {  // sorted keys: all in [0, len) iff both ends are
            const uint64_t k0 = uint64_t(intcol_get(pc.idx, 0)) - pc.idx_off;
            const uint64_t k1 = uint64_t(intcol_get(pc.idx, pc.n - 1)) - pc.idx_off;
            if (k0 >= c.len || k1 >= c.len)
                __hip_atomic_fetch_or(err, kErrPatchOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // every block store of the workgroup is complete before any patch store
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (s_pscr[0] && s_pscr[1]) {
            if (pin) gstore(out + pkey, pval);
        } else {
            const uint64_t ps = patch_lower_bound(pc, olo, s_pscr + 4);
            const uint64_t pe = patch_lower_bound(pc, ohi, s_pscr + 4);
            // sorted keys in [ps, pe) all lie in [olo, ohi); one outside is unsorted input (a
            // malformed file) and is reported, never stored
            bool bad = false;
            for (uint64_t i = ps + threadIdx.x; i < pe; i += 256) {
                const uint64_t key = uint64_t(intcol_get(pc.idx, i)) - pc.idx_off;
                if (key >= olo && key < ohi) gstore(out + key, gload(static_cast<const O*>(pc.vals) + i));
                else bad = true;
            }
            if (bad) __hip_atomic_fetch_or(err, kErrPatchOrder, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int T, int W, Epi EPI, int VW, bool LDSD, bool EXT>
__global__ __launch_bounds__(256) void fl_unpack_w_kernel(ChunkTable tab) {
    const uint64_t g = blockIdx.x;
    if constexpr (EXT) {
        const ChunkDev& c =
            tab.ext[ext_chunk_index(tab.ext, tab.n, g, [](const ChunkDev& d) { return d.first_group; })];
        unpack_chunk_w<T, W, EPI, VW, LDSD>(c, g, tab.err, PatchCol{}, tab.bpw);
    } else {
        uint32_t lo = 0, hi = tab.n;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tab.c[mid].first_group <= g) lo = mid; else hi = mid;
        }
        unpack_chunk_w<T, W, EPI, VW, LDSD>(tab.c[lo], g, tab.err, tab.patch, tab.bpw);
    }
}

// EXT: the chunk table is a recorded plan's device table (any length; one wave-wide count
// finds the chunk) instead of the kernel argument -- a separate instantiation, so the kernarg
// path keeps its scalar-load code (a runtime branch cost C1 1 %).
template <int T, int W, Epi EPI, int VW, bool LDSD = false, int S = 1, bool EXT = false>
__global__ __launch_bounds__(256) void fl_unpack_kernel(ChunkTable tab) {
    const uint64_t g = blockIdx.x;
    if constexpr (EXT) {
        const ChunkDev& c =
            tab.ext[ext_chunk_index(tab.ext, tab.n, g, [](const ChunkDev& d) { return d.first_group; })];
        unpack_chunk<T, W, EPI, VW, LDSD, S>(c, g, tab.err);
    } else {
        uint32_t lo = 0, hi = tab.n;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tab.c[mid].first_group <= g) lo = mid; else hi = mid;
        }
        unpack_chunk<T, W, EPI, VW, LDSD, S>(tab.c[lo], g, tab.err);
    }
}


// Blocks per workgroup of a K1w launch over `blocks` FastLanes blocks whose width allows at most
// `bpw_max`: the maximum, or -- when that leaves the launch under `min_groups` workgroups (a C5
// column of 6 M values, 5,861 blocks, was 183 workgroups for 256 CUs, one 4-wave workgroup per
// CU) -- blocks / min_groups rounded down to a multiple of 4 (>= 4), so the 4 waves get equal
// shares; `forced` (VXG_OPT_K1W_BPW) > 0 takes min(forced, bpw_max) instead.  Every value in
// [1, bpw_max] is a valid launch shape (unpack_chunk_w: PER = ceil(BPW / 4) blocks per wave).
inline int k1w_pick_bpw(uint64_t blocks, int bpw_max, int64_t min_groups, int64_t forced) {
    if (forced > 0) return int(forced < bpw_max ? forced : bpw_max);
    if (min_groups <= 0 || blocks >= uint64_t(min_groups) * uint64_t(bpw_max)) return bpw_max;
    const uint64_t b = blocks / uint64_t(min_groups);
    const int bpw = int(b < 4 ? 4 : (b / 4) * 4);
    return bpw > bpw_max ? bpw_max : bpw;
}

template <int T, int W, Epi EPI, int VW, bool LDSD, bool EXT>
vxg_status launch_w(ChunkTable tab, hipStream_t s) {
    constexpr int BPW_MAX = kw_bpw(W, LDSD);
    ChunkDev* cs = tab.ext ? tab.host : tab.c;
    uint64_t blocks = 0;
    for (uint32_t k = 0; k < tab.n; k++) blocks += cs[k].n_blocks;
    // the dictionary stage (LDSD) keeps its fixed offset at any BPW
    const Options o = cur_options();
    const int BPW = k1w_pick_bpw(blocks, BPW_MAX, o.k1w_min_groups, o.k1w_bpw);
    tab.bpw = uint32_t(BPW);
    uint64_t groups = 0, dict_bytes = 0;
    for (uint32_t k = 0; k < tab.n; k++) {
        cs[k].first_group = groups;
        groups += (cs[k].n_blocks + BPW - 1) / BPW;
        const uint64_t db = (cs[k].dict_len * uint64_t(VW > 0 ? VW : 1) + 15) & ~15ull;
        dict_bytes = db > dict_bytes ? db : dict_bytes;
    }
    if (groups == 0) return VXG_OK;
    if (groups > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "array too long for one launch");
    const size_t shm = LDSD ? size_t(kw_packed_lds<W, LDSD>()) + size_t(dict_bytes)
                            : size_t(W > 0 ? BPW * 128 * W : 0) + 128;
    hipLaunchKernelGGL((fl_unpack_w_kernel<T, W, EPI, VW, LDSD, EXT>), dim3(unsigned(groups)), dim3(256), shm, s, tab);
    note_k1w_launch(uint32_t(BPW), uint32_t(BPW_MAX), groups);
    if constexpr (!EXT) {
        if (tab.patch.n) g_k1w_wrote_patches = true;  // only this kernel reads tab.patch
    }
    return hip_check(hipGetLastError(), "fl_unpack_w_kernel launch");
}

// k1_wave_mode() (vxg_internal.hpp): VXG_OPT_K1_WAVE, else VXG_K1_WAVE read at every launch --
// "0" keeps the register-resident K1 for large launches too; "force" takes K1w for small
// launches as well (parity tests of every width).

template <int T, int W, Epi EPI, int VW, bool LDSD, int S, bool EXT = false>
vxg_status launch_s(ChunkTable tab, hipStream_t s) {
    // first workgroup of each chunk at this launch's blocks per workgroup (a device table's
    // host mirror is completed here and uploaded when the plan is finalised)
    ChunkDev* cs = tab.ext ? tab.host : tab.c;
    uint64_t groups = 0;
    for (uint32_t k = 0; k < tab.n; k++) {
        cs[k].first_group = groups;
        groups += (cs[k].n_blocks + (32 / S) - 1) / (32 / S);
    }
    if (groups == 0) return VXG_OK;
    if (groups > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "array too long for one launch");
    hipLaunchKernelGGL((fl_unpack_kernel<T, W, EPI, VW, LDSD, S, EXT>), dim3(unsigned(groups)), dim3(256), 0, s, tab);
    return hip_check(hipGetLastError(), "fl_unpack_kernel launch");
}

// `groups32` = the table's workgroups at 32 blocks per workgroup (decides the row split).
template <int T, int W, Epi EPI, int VW>
vxg_status launch_one(const ChunkTable& tab, uint64_t groups32, hipStream_t s) {
    if (groups32 == 0) return VXG_OK;
    constexpr bool kSplit = (T == 32 || T == 64) && W > 0;
    const bool split = kSplit && groups32 < split_below_groups();
    bool lds = false;
    if constexpr (EPI == Epi::Dict) {
        const ChunkDev* cs = tab.ext ? tab.host : tab.c;
        lds = true;
        for (uint32_t k = 0; k < tab.n; k++)
            lds = lds && cs[k].dict_len * VW <= uint64_t(kDictLdsBytes) &&
                  (reinterpret_cast<uintptr_t>(cs[k].dict) & 15) == 0;
    }
    // Dict gathers keep the register-resident K1 by default: C3 (u64 codes W=10, 8-byte values,
    // dictionary in LDS) measured 0.65 of 8 TB/s with K1w against 0.70 with the row split
    // Device-table launches (a plan's chunked columns) take K1w from kExtWaveGroups workgroups of
    // 32 blocks: C5's 48 MB numeric columns (183) measured C5 0.52 -> 0.556 of 8 TB/s with K1w
    // instead of the row split (sessions r04kw, r04c), but the 2-GPU shard's halves (92) 0.506 ->
    // 0.429 (too few K1w workgroups for 256 CUs)
    constexpr uint64_t kExtWaveGroups = 128;
    const int mode = k1_wave_mode();
    const bool big = !split || (tab.ext && groups32 >= kExtWaveGroups);
    const bool wave = mode == 2 || (mode == 1 && big && EPI != Epi::Dict);  // large launches: K1w
    if (tab.ext) {  // device table (plans): K1w, or the register-resident K1 for Dict gathers
        if (wave) {
            if constexpr (EPI == Epi::Dict) {
                if (lds) return launch_w<T, W, EPI, VW, true, true>(tab, s);
            }
            return launch_w<T, W, EPI, VW, false, true>(tab, s);
        }
        constexpr int SX = kSplit ? 4 : 1;
        if constexpr (EPI == Epi::Dict) {
            if (lds) return launch_s<T, W, EPI, VW, true, SX, true>(tab, s);
        }
        return launch_s<T, W, EPI, VW, false, SX, true>(tab, s);
    }
    if constexpr (kSplit) {
        if (split && !wave) return lds ? launch_s<T, W, EPI, VW, true, 4>(tab, s) : launch_s<T, W, EPI, VW, false, 4>(tab, s);
    }
    if (wave) {
        if constexpr (EPI == Epi::Dict) {
            if (lds) return launch_w<T, W, EPI, VW, true, false>(tab, s);
        }
        return launch_w<T, W, EPI, VW, false, false>(tab, s);
    }
    if constexpr (EPI == Epi::Dict) {
        if (lds) return launch_s<T, W, EPI, VW, true, 1>(tab, s);
    }
    return launch_s<T, W, EPI, VW, false, 1>(tab, s);
}

// Function-pointer table over W = 0..WMAX.
template <int T, Epi EPI, int VW, int... Ws>
vxg_status dispatch_w_impl(int W, const ChunkTable& tab, uint64_t groups, hipStream_t s,
                           std::integer_sequence<int, Ws...>) {
    using Fn = vxg_status (*)(const ChunkTable&, uint64_t, hipStream_t);
    static constexpr Fn table[] = {&launch_one<T, Ws, EPI, VW>...};
    if (W < 0 || W >= int(sizeof...(Ws))) return VXG_ERR_NOT_IMPLEMENTED;
    return table[W](tab, groups, s);
}

template <int T, Epi EPI, int VW, int WMAX>
vxg_status dispatch_w(int W, const ChunkTable& tab, uint64_t groups, hipStream_t s) {
    return dispatch_w_impl<T, EPI, VW>(W, tab, groups, s, std::make_integer_sequence<int, WMAX + 1>{});
}

}  // namespace vxg
