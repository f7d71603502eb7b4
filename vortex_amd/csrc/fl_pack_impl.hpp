// fl_pack_impl.hpp — K15: fastlanes BitPacking::unchecked_pack (+ FoR compress_primitive) on the
// GPU; instantiated per T by pack_inst.hip.  See encode_gpu.hip for the design notes.
#pragma once

#include <type_traits>

#include "encode_gpu.hpp"
#include "fl_unpack_impl.hpp"

namespace vxg {

constexpr int kPackBlock = 256;

// value x of the input, FoR-transformed ((x - ref) wrapping, >> shift: arithmetic for signed
// ptypes, for/compress.rs:61-84) and masked to W bits; zero for the padding of the last block
// (bitpacking/compress.rs:121-135 pads the ENCODED values with zeros)
template <int T, int W, bool FOR>
__device__ __forceinline__ uint64_t pack_in(typename Fl<T>::E x, bool valid, uint64_t ref, unsigned shift, bool sgn) {
    using E = typename Fl<T>::E;
    if (!valid) return 0;
    if constexpr (FOR) {
        E d = E(x - E(ref));
        if (shift) {
            if (sgn) {
                using S = std::make_signed_t<E>;
                d = E(S(d) >> shift);
            } else {
                d = E(d >> shift);
            }
        }
        x = d;
    }
    return uint64_t(x) & (W >= 64 ? ~0ull : ((1ull << W) - 1ull));
}

template <int T, int W, bool FOR, int R>
__device__ __forceinline__ void pack_row(Vec16<T>* p, const Vec16<T>& in, uint32_t valid, uint64_t ref,
                                         unsigned shift, bool sgn) {
    using U = typename Fl<T>::U;
    constexpr int EPV = 16 / (T / 8);
    constexpr int PER = T == 64 ? 1 : 32 / T;  // elements per U word
    constexpr int start = R * W, word = start / T, sh = start % T;
#pragma unroll
    for (int j = 0; j < EPV; j++) {
        const uint64_t x = pack_in<T, W, FOR>(in.elem(j), (valid >> j) & 1u, ref, shift, sgn);
        const int k = j / PER, b = (j % PER) * T;  // U word and bit position of lane j
        const uint64_t lo = (x << sh) & (T == 64 ? ~0ull : ((1ull << T) - 1ull));
        p[word].w[k] |= U(lo << b);
        if constexpr (sh + W > T) p[word + 1].w[k] |= U((x >> (T - sh)) << b);
    }
}

template <int T, int W, bool FOR, int... Rs>
__device__ __forceinline__ void pack_rows(Vec16<T>* p, const uint8_t* __restrict__ vals, uint64_t blk, int t,
                                          uint64_t n, uint64_t ref, unsigned shift, bool sgn, bool full,
                                          std::integer_sequence<int, Rs...>) {
    using E = typename Fl<T>::E;
    constexpr int EPV = 16 / (T / 8);
    auto one = [&](auto rc) {
        constexpr int R = decltype(rc)::value;
        const uint64_t i0 = blk * 1024 + uint64_t(fl_index(R, t * EPV));
        Vec16<T> in;
        uint32_t valid = (1u << EPV) - 1u;
        if (full) {
            in = load16<T>(vals + i0 * sizeof(E));
        } else {
            E e[EPV];
            valid = 0;
#pragma unroll
            for (int j = 0; j < EPV; j++) {
                const bool ok = i0 + j < n;
                e[j] = ok ? reinterpret_cast<const E*>(vals)[i0 + j] : E(0);
                valid |= uint32_t(ok) << j;
            }
            __builtin_memcpy(in.w, e, 16);
        }
        pack_row<T, W, FOR, R>(p, in, valid, ref, shift, sgn);
    };
    (one(std::integral_constant<int, Rs>{}), ...);
}

template <int T, int W, bool FOR>
__global__ __launch_bounds__(kPackBlock) void fl_pack_kernel(const uint8_t* __restrict__ vals, uint64_t n,
                                                             uint8_t* __restrict__ packed, uint64_t ref,
                                                             unsigned shift, bool sgn) {
    const uint64_t gid = uint64_t(blockIdx.x) * kPackBlock + threadIdx.x;
    const uint64_t blk = gid >> 3;
    const int t = int(gid & 7);
    if (blk * 1024 >= n) return;
    const bool full = (blk + 1) * 1024 <= n && (reinterpret_cast<uintptr_t>(vals) & 15) == 0;
    Vec16<T> p[W];
#pragma unroll
    for (int w = 0; w < W; w++)
#pragma unroll
        for (int k = 0; k < Vec16<T>::NV; k++) p[w].w[k] = 0;
    pack_rows<T, W, FOR>(p, vals, blk, t, n, ref, shift, sgn, full, std::make_integer_sequence<int, T>{});
#pragma unroll
    for (int w = 0; w < W; w++) {
        uint4 q;
        __builtin_memcpy(&q, p[w].w, 16);
        nt_store(reinterpret_cast<uint4*>(packed + blk * (128ull * W) + 128 * w + 16 * t), q);
    }
}

template <int T, int W>
vxg_status launch_pack_w(bool for_, uint64_t ref, unsigned shift, bool sgn, const void* v, uint64_t n, void* packed,
                         hipStream_t s) {
    const uint64_t threads = ((n + 1023) / 1024) * 8;
    const dim3 grid(unsigned((threads + kPackBlock - 1) / kPackBlock));
    if (for_)
        hipLaunchKernelGGL((fl_pack_kernel<T, W, true>), grid, dim3(kPackBlock), 0, s, static_cast<const uint8_t*>(v), n,
                           static_cast<uint8_t*>(packed), ref, shift, sgn);
    else
        hipLaunchKernelGGL((fl_pack_kernel<T, W, false>), grid, dim3(kPackBlock), 0, s, static_cast<const uint8_t*>(v),
                           n, static_cast<uint8_t*>(packed), ref, shift, sgn);
    return hip_check(hipGetLastError(), "fl_pack_kernel");
}

template <int T, int... Ws>
vxg_status pack_dispatch(int W, bool for_, uint64_t ref, unsigned shift, bool sgn, const void* v, uint64_t n,
                         void* packed, hipStream_t s, std::integer_sequence<int, Ws...>) {
    using Fn = vxg_status (*)(bool, uint64_t, unsigned, bool, const void*, uint64_t, void*, hipStream_t);
    static constexpr Fn table[] = {&launch_pack_w<T, Ws + 1>...};
    if (W < 1 || W > int(sizeof...(Ws))) return set_error(VXG_ERR_INVALID_ARGUMENT, "pack: bit width out of range");
    return table[W - 1](for_, ref, shift, sgn, v, n, packed, s);
}

}  // namespace vxg
