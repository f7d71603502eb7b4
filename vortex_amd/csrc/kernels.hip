// kernels.hip — the non-bitpacking decode kernels of the engine (gfx950).
//
//   K2 patch scatter     sparse/mod.rs:132-144 + primitive/mod.rs:168-185 (+ cascade epilogue)
//   FoR / ZigZag / ALP   for/compress.rs:86-117, zigzag/compress.rs:35-57, alp/compress.rs:98-106
//                        (standalone forms, used when the child is not BitPacked)
//   K5 take              primitive/compute/take.rs:58-67, varbinview/compute.rs:68-76 (16-B views)
//   K4 ALP-RD combine    alp_rd/mod.rs:260-301
//   K3 Delta             delta/compress.rs:100-166 (undelta + untranspose fused, + slice :111)
//   K8 RunEnd expand     runend/compress.rs:115-148
//   K10 fill             array/constant/canonical.rs (broadcast)
//   views                arrow-cast 53.2 Utf8->Utf8View (varbin/flatten.rs:10-17)
// All of them are HBM-streaming kernels: 16-byte-per-lane accesses where the layout allows it,
// grid-stride loops capped at 8 workgroups per CU, no LDS except where a re-layout needs it.
#include "fl_unpack_impl.hpp"
#include "intcol.hpp"
#include "runend_runs.hpp"

namespace vxg {

namespace {

constexpr int kBlock = 256;

inline unsigned grid_for(uint64_t n_threads) {
    uint64_t g = (n_threads + kBlock - 1) / kBlock;
    const uint64_t cap = 256ull * 8 * 16;  // grid-stride beyond 32K workgroups
    if (g > cap) g = cap;
    if (g == 0) g = 1;
    return unsigned(g);
}

__device__ __forceinline__ uint64_t load_uint(const void* p, int width, bool sgn, uint64_t i) {
    switch (width) {
    case 1: return sgn ? uint64_t(int64_t(gload(static_cast<const int8_t*>(p) + i))) : gload(static_cast<const uint8_t*>(p) + i);
    case 2: return sgn ? uint64_t(int64_t(gload(static_cast<const int16_t*>(p) + i))) : gload(static_cast<const uint16_t*>(p) + i);
    case 4: return sgn ? uint64_t(int64_t(gload(static_cast<const int32_t*>(p) + i))) : gload(static_cast<const uint32_t*>(p) + i);
    default: return gload(static_cast<const uint64_t*>(p) + i);
    }
}

template <int W> struct UInt;
template <> struct UInt<1> { using t = uint8_t; };
template <> struct UInt<2> { using t = uint16_t; };
template <> struct UInt<4> { using t = uint32_t; };
template <> struct UInt<8> { using t = uint64_t; };
template <> struct UInt<16> { using t = uint4; };

}  // namespace

// ------------------------------------------------------------------ K2 patch scatter
template <int T, Epi EPI, int VW>
__global__ __launch_bounds__(kBlock) void patch_kernel(typename EpiOut<T, EPI, VW>::type* __restrict__ out,
                                                       uint64_t out_len, IntCol idx, uint64_t idx_off,
                                                       const typename Fl<T>::E* __restrict__ vals,
                                                       uint64_t n, EpiParams ep) {
    // indices read in place (a packed FoR/BitPacked index column is unpacked per patch)
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += uint64_t(gridDim.x) * blockDim.x) {
        const uint64_t p = uint64_t(intcol_get(idx, i)) - idx_off;
        if (p >= out_len) {
            __hip_atomic_fetch_or(ep.err, kErrPatchOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            continue;
        }
        out[p] = apply_epi<T, EPI, VW>(vals[i], ep);
    }
}

template <int T, Epi EPI, int VW>
static vxg_status patch_launch(void* out, uint64_t out_len, const IntCol& idx, uint64_t ioff,
                               const void* vals, uint64_t n, const UnpackArgs& a, hipStream_t s) {
    using O = typename EpiOut<T, EPI, VW>::type;
    hipLaunchKernelGGL((patch_kernel<T, EPI, VW>), dim3(grid_for(n)), dim3(kBlock), 0, s,
                       static_cast<O*>(out), out_len, idx, ioff,
                       static_cast<const typename Fl<T>::E*>(vals), n, to_epi(a));
    return hip_check(hipGetLastError(), "patch_kernel");
}

template <int T, Epi EPI>
static vxg_status patch_vw(int vw, void* out, uint64_t out_len, const IntCol& idx, uint64_t ioff,
                           const void* vals, uint64_t n, const UnpackArgs& a, hipStream_t s) {
    switch (vw) {
    case 1: return patch_launch<T, EPI, 1>(out, out_len, idx, ioff, vals, n, a, s);
    case 2: return patch_launch<T, EPI, 2>(out, out_len, idx, ioff, vals, n, a, s);
    case 4: return patch_launch<T, EPI, 4>(out, out_len, idx, ioff, vals, n, a, s);
    case 8: return patch_launch<T, EPI, 8>(out, out_len, idx, ioff, vals, n, a, s);
    case 16: return patch_launch<T, EPI, 16>(out, out_len, idx, ioff, vals, n, a, s);
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
}

template <int T>
static vxg_status patch_t(Epi epi, int vw, void* out, uint64_t out_len, const IntCol& idx, uint64_t ioff,
                          const void* vals, uint64_t n, const UnpackArgs& a, hipStream_t s) {
    switch (epi) {
    case Epi::Plain: return patch_launch<T, Epi::Plain, 0>(out, out_len, idx, ioff, vals, n, a, s);
    case Epi::For: return patch_launch<T, Epi::For, 0>(out, out_len, idx, ioff, vals, n, a, s);
    case Epi::ForZigZag: return patch_launch<T, Epi::ForZigZag, 0>(out, out_len, idx, ioff, vals, n, a, s);
    case Epi::AlpF32:
        if constexpr (T == 32) return patch_launch<32, Epi::AlpF32, 0>(out, out_len, idx, ioff, vals, n, a, s);
        return VXG_ERR_INVALID_ARGUMENT;
    case Epi::AlpF64:
        if constexpr (T == 64) return patch_launch<64, Epi::AlpF64, 0>(out, out_len, idx, ioff, vals, n, a, s);
        return VXG_ERR_INVALID_ARGUMENT;
    case Epi::Dict: return patch_vw<T, Epi::Dict>(vw, out, out_len, idx, ioff, vals, n, a, s);
    }
    return VXG_ERR_INVALID_ARGUMENT;
}

vxg_status launch_patch(int val_width, const IntCol& indices, Epi epi, int T, void* out, uint64_t out_len,
                        uint64_t indices_offset, const void* values, uint64_t n, const UnpackArgs& ep,
                        hipStream_t s) {
    if (n == 0) return VXG_OK;
    switch (T) {
    case 8: return patch_t<8>(epi, val_width, out, out_len, indices, indices_offset, values, n, ep, s);
    case 16: return patch_t<16>(epi, val_width, out, out_len, indices, indices_offset, values, n, ep, s);
    case 32: return patch_t<32>(epi, val_width, out, out_len, indices, indices_offset, values, n, ep, s);
    case 64: return patch_t<64>(epi, val_width, out, out_len, indices, indices_offset, values, n, ep, s);
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
}

// ------------------------------------------------------------------ FoR / ZigZag (16 B / lane)
template <typename E, bool ZZ>
__global__ __launch_bounds__(kBlock) void for_kernel(const E* __restrict__ in, uint64_t n, E ref,
                                                     unsigned shift, E* __restrict__ out) {
    constexpr int V = 16 / sizeof(E);
    const uint64_t nv = n / V;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nv; i += stride) {
        uint4 q = reinterpret_cast<const uint4*>(in)[i];
        E e[V];
        __builtin_memcpy(e, &q, 16);
#pragma unroll
        for (int j = 0; j < V; j++) {
            E v = E(E(e[j] << shift) + ref);
            if constexpr (ZZ) v = E((v >> 1) ^ E(E(0) - E(v & 1)));
            e[j] = v;
        }
        __builtin_memcpy(&q, e, 16);
        nt_store(reinterpret_cast<uint4*>(out) + i, q);
    }
    for (uint64_t i = nv * V + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        E v = E(E(in[i] << shift) + ref);
        if constexpr (ZZ) v = E((v >> 1) ^ E(E(0) - E(v & 1)));
        out[i] = v;
    }
}

template <typename E>
static vxg_status for_t(const void* in, uint64_t n, uint64_t ref, unsigned shift, bool zz, void* out,
                        hipStream_t s) {
    if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15)
        return set_error(VXG_ERR_INVALID_ARGUMENT, "FoR/ZigZag buffers must be 16-byte aligned");
    const unsigned g = grid_for(n / (16 / sizeof(E)) + 1);
    if (zz)
        hipLaunchKernelGGL((for_kernel<E, true>), dim3(g), dim3(kBlock), 0, s,
                           static_cast<const E*>(in), n, E(ref), shift, static_cast<E*>(out));
    else
        hipLaunchKernelGGL((for_kernel<E, false>), dim3(g), dim3(kBlock), 0, s,
                           static_cast<const E*>(in), n, E(ref), shift, static_cast<E*>(out));
    return hip_check(hipGetLastError(), "for_kernel");
}

vxg_status launch_for(int width, const void* in, uint64_t n, uint64_t ref, unsigned shift, bool zz,
                      void* out, hipStream_t s) {
    if (n == 0) return VXG_OK;
    switch (width) {
    case 1: return for_t<uint8_t>(in, n, ref, shift, zz, out, s);
    case 2: return for_t<uint16_t>(in, n, ref, shift, zz, out, s);
    case 4: return for_t<uint32_t>(in, n, ref, shift, zz, out, s);
    case 8: return for_t<uint64_t>(in, n, ref, shift, zz, out, s);
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
}

vxg_status launch_zigzag(int width, const void* in, uint64_t n, void* out, hipStream_t s) {
    return launch_for(width, in, n, 0, 0, true, out, s);
}

// ------------------------------------------------------------------ ALP (standalone)
template <typename I, typename F>
__global__ __launch_bounds__(kBlock) void alp_kernel(const I* __restrict__ in, uint64_t n, F a, F b,
                                                     F* __restrict__ out) {
    constexpr int V = 16 / sizeof(I);
    const uint64_t nv = n / V;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nv; i += stride) {
        uint4 q = reinterpret_cast<const uint4*>(in)[i];
        I e[V];
        F o[V];
        __builtin_memcpy(e, &q, 16);
#pragma unroll
        for (int j = 0; j < V; j++) {
            if constexpr (sizeof(F) == 4) o[j] = __fmul_rn(__fmul_rn(F(e[j]), a), b);
            else o[j] = __dmul_rn(__dmul_rn(F(e[j]), a), b);
        }
        __builtin_memcpy(&q, o, 16);
        nt_store(reinterpret_cast<uint4*>(out) + i, q);
    }
    for (uint64_t i = nv * V + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        if constexpr (sizeof(F) == 4) out[i] = __fmul_rn(__fmul_rn(F(in[i]), a), b);
        else out[i] = __dmul_rn(__dmul_rn(F(in[i]), a), b);
    }
}

vxg_status launch_alp(int float_ptype, const void* enc, uint64_t n, double a, double b, void* out,
                      hipStream_t s) {
    if (n == 0) return VXG_OK;
    if ((reinterpret_cast<uintptr_t>(enc) | reinterpret_cast<uintptr_t>(out)) & 15)
        return set_error(VXG_ERR_INVALID_ARGUMENT, "ALP buffers must be 16-byte aligned");
    if (float_ptype == VXG_F32) {
        hipLaunchKernelGGL((alp_kernel<int32_t, float>), dim3(grid_for(n / 4 + 1)), dim3(kBlock), 0, s,
                           static_cast<const int32_t*>(enc), n, float(a), float(b), static_cast<float*>(out));
    } else if (float_ptype == VXG_F64) {
        hipLaunchKernelGGL((alp_kernel<int64_t, double>), dim3(grid_for(n / 2 + 1)), dim3(kBlock), 0, s,
                           static_cast<const int64_t*>(enc), n, a, b, static_cast<double*>(out));
    } else {
        return set_error(VXG_ERR_MISMATCHED_TYPES, "ALP decodes to f32 or f64 only");
    }
    return hip_check(hipGetLastError(), "alp_kernel");
}

// ------------------------------------------------------------------ K5 take (gather)
template <typename C, typename V>
__global__ __launch_bounds__(kBlock) void take_kernel(const V* __restrict__ values, uint64_t n_values,
                                                      const C* __restrict__ codes, uint64_t n,
                                                      V* __restrict__ out, uint32_t* err) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t c = uint64_t(codes[i]);
        if (c >= n_values) {
            __hip_atomic_fetch_or(err, kErrTakeOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            c = 0;
        }
        nt_store(out + i, values[c]);
    }
}

template <typename C>
static vxg_status take_c(int vw, const void* values, uint64_t nv, const void* codes, uint64_t n,
                         void* out, uint32_t* err, hipStream_t s) {
    const unsigned g = grid_for(n);
    switch (vw) {
#define TAKE_CASE(W)                                                                                \
    case W:                                                                                         \
        hipLaunchKernelGGL((take_kernel<C, typename UInt<W>::t>), dim3(g), dim3(kBlock), 0, s,      \
                           static_cast<const typename UInt<W>::t*>(values), nv,                     \
                           static_cast<const C*>(codes), n, static_cast<typename UInt<W>::t*>(out), \
                           err);                                                                    \
        break;
        TAKE_CASE(1) TAKE_CASE(2) TAKE_CASE(4) TAKE_CASE(8) TAKE_CASE(16)
#undef TAKE_CASE
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
    return hip_check(hipGetLastError(), "take_kernel");
}

// Signed indices are sign-extended: a negative index becomes a huge usize and is OutOfBounds,
// as the reference's `as usize` conversion makes it (primitive/compute/take.rs:58-67).
vxg_status launch_take(int value_width, const void* values, uint64_t n_values, int code_width, bool code_signed,
                       const void* codes, uint64_t n, void* out, uint32_t* err, hipStream_t s) {
    if (n == 0) return VXG_OK;
    // every index is out of bounds of an empty array (and its values buffer may be null)
    if (n_values == 0) return set_error(VXG_ERR_OUT_OF_BOUNDS, "take: index out of bounds");
    switch (code_width * (code_signed ? -1 : 1)) {
    case 1: return take_c<uint8_t>(value_width, values, n_values, codes, n, out, err, s);
    case 2: return take_c<uint16_t>(value_width, values, n_values, codes, n, out, err, s);
    case 4: return take_c<uint32_t>(value_width, values, n_values, codes, n, out, err, s);
    case 8: case -8: return take_c<uint64_t>(value_width, values, n_values, codes, n, out, err, s);
    case -1: return take_c<int8_t>(value_width, values, n_values, codes, n, out, err, s);
    case -2: return take_c<int16_t>(value_width, values, n_values, codes, n, out, err, s);
    case -4: return take_c<int32_t>(value_width, values, n_values, codes, n, out, err, s);
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
}

// ------------------------------------------------------------------ K4 ALP-RD
struct RdDict { uint16_t d[8]; };

template <typename UT>
__global__ __launch_bounds__(kBlock) void alprd_kernel(const uint16_t* __restrict__ left, RdDict dict,
                                                       unsigned dict_len, unsigned rbw,
                                                       const UT* __restrict__ right, uint64_t n,
                                                       UT* __restrict__ out) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        unsigned c = left[i];
        const UT l = UT(c < dict_len ? dict.d[c] : 0);
        out[i] = UT((l << rbw) | right[i]);
    }
}

template <typename UT>
__global__ __launch_bounds__(kBlock) void alprd_exc_kernel(const void* __restrict__ pos, int pos_width,
                                                           int pos_signed, uint64_t pos_off,
                                                           const uint16_t* __restrict__ exc, uint64_t n_exc,
                                                           unsigned rbw, const UT* __restrict__ right,
                                                           uint64_t n, UT* __restrict__ out, uint32_t* err) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n_exc; i += stride) {
        const uint64_t p = load_uint(pos, pos_width, pos_signed != 0, i) - pos_off;
        if (p < n) out[p] = UT((UT(exc[i]) << rbw) | right[p]);
        else __hip_atomic_fetch_or(err, kErrPatchOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

vxg_status launch_alprd(int float_ptype, const uint16_t* left, const uint16_t* dict, unsigned dict_len,
                        unsigned rbw, const void* right, uint64_t n, const void* exc_pos, int pos_width,
                        bool pos_signed, uint64_t pos_off, const uint16_t* exc, uint64_t n_exc, void* out,
                        uint32_t* err, hipStream_t s) {
    RdDict d{};
    for (unsigned i = 0; i < dict_len && i < 8; i++) d.d[i] = dict[i];
    if (float_ptype == VXG_F32) {
        if (n) hipLaunchKernelGGL((alprd_kernel<uint32_t>), dim3(grid_for(n)), dim3(kBlock), 0, s, left, d,
                                  dict_len, rbw, static_cast<const uint32_t*>(right), n, static_cast<uint32_t*>(out));
        if (n_exc) hipLaunchKernelGGL((alprd_exc_kernel<uint32_t>), dim3(grid_for(n_exc)), dim3(kBlock), 0, s,
                                      exc_pos, pos_width, int(pos_signed), pos_off, exc, n_exc, rbw,
                                      static_cast<const uint32_t*>(right), n, static_cast<uint32_t*>(out), err);
    } else if (float_ptype == VXG_F64) {
        if (n) hipLaunchKernelGGL((alprd_kernel<uint64_t>), dim3(grid_for(n)), dim3(kBlock), 0, s, left, d,
                                  dict_len, rbw, static_cast<const uint64_t*>(right), n, static_cast<uint64_t*>(out));
        if (n_exc) hipLaunchKernelGGL((alprd_exc_kernel<uint64_t>), dim3(grid_for(n_exc)), dim3(kBlock), 0, s,
                                      exc_pos, pos_width, int(pos_signed), pos_off, exc, n_exc, rbw,
                                      static_cast<const uint64_t*>(right), n, static_cast<uint64_t*>(out), err);
    } else {
        return set_error(VXG_ERR_MISMATCHED_TYPES, "ALP-RD decodes to f32 or f64 only");
    }
    return hip_check(hipGetLastError(), "alprd_kernel");
}

// ------------------------------------------------------------------ validity bit copy
// dst (pre-zeroed) bits [dst_off, dst_off+n) |= src bits [src_off, src_off+n); LSB order.
__global__ __launch_bounds__(kBlock) void copy_bits_kernel(uint32_t* __restrict__ dst, uint64_t dst_off,
                                                           const uint8_t* __restrict__ src, uint64_t src_off,
                                                           uint64_t n, int set_all) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t w = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; w * 32 < n; w += stride) {
        uint32_t bits = 0;
        for (int k = 0; k < 32; k++) {
            const uint64_t i = w * 32 + k;
            if (i >= n) break;
            const uint64_t si = src_off + i;
            const uint32_t b = set_all ? 1u : uint32_t((src[si >> 3] >> (si & 7)) & 1);
            bits |= b << k;
        }
        const uint64_t d = dst_off + w * 32;
        const uint64_t word = d >> 5;
        const int sh = int(d & 31);
        if (bits) {
            atomicOr(dst + word, bits << sh);
            if (sh) atomicOr(dst + word + 1, bits >> (32 - sh));
        }
    }
}

vxg_status launch_copy_bits(void* dst, uint64_t dst_off, const uint8_t* src, uint64_t src_off, uint64_t n,
                            bool set_all, hipStream_t s) {
    if (n == 0) return VXG_OK;
    hipLaunchKernelGGL(copy_bits_kernel, dim3(grid_for((n + 31) / 32)), dim3(kBlock), 0, s,
                       static_cast<uint32_t*>(dst), dst_off, src, src_off, n, int(set_all));
    return hip_check(hipGetLastError(), "copy_bits_kernel");
}

// Sparse validity: set bit (idx - off) for every index.
__global__ __launch_bounds__(kBlock) void set_bits_at_kernel(uint32_t* __restrict__ dst, const void* idx,
                                                             int iw, int isg, uint64_t off, uint64_t n,
                                                             uint64_t len) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t p = load_uint(idx, iw, isg != 0, i) - off;
        if (p < len) atomicOr(dst + (p >> 5), 1u << (p & 31));
    }
}

vxg_status launch_set_bits_at(void* dst, const void* idx, int iw, bool isg, uint64_t off, uint64_t n,
                              uint64_t len, hipStream_t s) {
    if (n == 0) return VXG_OK;
    hipLaunchKernelGGL(set_bits_at_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       static_cast<uint32_t*>(dst), idx, iw, int(isg), off, n, len);
    return hip_check(hipGetLastError(), "set_bits_at_kernel");
}

// Sum of an integer column (FSST heap size), int64 result.
__global__ __launch_bounds__(kBlock) void sum_kernel(const void* p, int w, int sg, uint64_t n,
                                                     unsigned long long* out) {
    unsigned long long acc = 0;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        acc += (unsigned long long)load_uint(p, w, sg != 0, i);
    for (int d = 32; d > 0; d >>= 1) acc += __shfl_down(acc, d, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

vxg_status launch_sum(const void* p, int w, bool sg, uint64_t n, void* out_u64, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out_u64, 0, 8, s);
    if (e != hipSuccess) return hip_check(e, "memset");
    if (n == 0) return VXG_OK;
    hipLaunchKernelGGL(sum_kernel, dim3(grid_for(n) > 1024 ? 1024 : grid_for(n)), dim3(kBlock), 0, s, p, w,
                       int(sg), n, static_cast<unsigned long long*>(out_u64));
    return hip_check(hipGetLastError(), "sum_kernel");
}

// ------------------------------------------------------------------ K3 Delta
// For lane l of a full block, the untransposed output positions of rows 0..T-1 form the
// contiguous run out[base_l .. base_l+T) with base_l = transpose(index(0, l)) (SURVEY App. A,
// invariant 3), so undelta + untranspose is one serial wrapping prefix per lane whose result
// is written as a contiguous T-element run: thread per (block, lane).
template <typename E>
__global__ __launch_bounds__(kBlock) void delta_kernel(const E* __restrict__ bases,
                                                       const E* __restrict__ deltas, uint64_t n_full_blocks,
                                                       uint64_t offset, uint64_t len, E* __restrict__ out) {
    constexpr int T = 8 * sizeof(E), LANES = 1024 / T;
    const uint64_t gid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t blk = gid / LANES;
    const int l = int(gid % LANES);
    if (blk >= n_full_blocks) return;
    const E* d = deltas + blk * 1024;
    // transpose(i) = (i%16)*64 + FL_ORDER[(i/16)%8]*8 + i/128 at i = index(0, l) = l
    const int base_l = (l % 16) * 64 + fl_order((l / 16) % 8) * 8;
    E prev = bases[blk * LANES + l];
    E run[T];
#pragma unroll
    for (int r = 0; r < T; r++) {
        prev = E(d[fl_index(r, l)] + prev);
        run[r] = prev;
    }
    const int64_t o0 = int64_t(blk * 1024 + base_l) - int64_t(offset);
    constexpr int RUN_BYTES = T * int(sizeof(E));  // 8 B for u8, 32/128/512 B otherwise
    constexpr int ALIGN = RUN_BYTES < 16 ? RUN_BYTES : 16;
    if (o0 >= 0 && uint64_t(o0) + T <= len && ((reinterpret_cast<uintptr_t>(out + o0) & (ALIGN - 1)) == 0)) {
        if constexpr (RUN_BYTES < 16) {
            uint2 q;
            __builtin_memcpy(&q, run, 8);
            *reinterpret_cast<uint2*>(out + o0) = q;
        } else {
#pragma unroll
            for (int k = 0; k < RUN_BYTES / 16; k++) {
                uint4 q;
                __builtin_memcpy(&q, reinterpret_cast<const uint8_t*>(run) + 16 * k, 16);
                nt_store(reinterpret_cast<uint4*>(out + o0) + k, q);
            }
        }
    } else {
#pragma unroll
        for (int r = 0; r < T; r++) {
            const int64_t o = o0 + r;
            if (o >= 0 && uint64_t(o) < len) out[o] = run[r];
        }
    }
}

template <typename E>
__global__ void delta_tail_kernel(const E* __restrict__ bases, const E* __restrict__ deltas,
                                  uint64_t n_full_blocks, uint64_t n_deltas, uint64_t offset,
                                  uint64_t len, E* __restrict__ out) {
    // remainder block: scalar running sum from bases[last] (delta/compress.rs:153-163)
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    constexpr int LANES = 1024 / (8 * sizeof(E));
    E base = bases[n_full_blocks * LANES];
    for (uint64_t i = n_full_blocks * 1024; i < n_deltas; i++) {
        base = E(deltas[i] + base);
        if (i >= offset && i - offset < len) out[i - offset] = base;
    }
}

template <typename E>
static vxg_status delta_t(const void* bases, const void* deltas, uint64_t n_deltas, uint64_t offset,
                          uint64_t len, void* out, hipStream_t s) {
    constexpr int LANES = 1024 / (8 * sizeof(E));
    const uint64_t full = n_deltas / 1024;
    if (full) {
        const uint64_t threads = full * LANES;
        hipLaunchKernelGGL((delta_kernel<E>), dim3(unsigned((threads + kBlock - 1) / kBlock)), dim3(kBlock),
                           0, s, static_cast<const E*>(bases), static_cast<const E*>(deltas), full, offset,
                           len, static_cast<E*>(out));
    }
    if (n_deltas % 1024)
        hipLaunchKernelGGL((delta_tail_kernel<E>), dim3(1), dim3(64), 0, s, static_cast<const E*>(bases),
                           static_cast<const E*>(deltas), full, n_deltas, offset, len, static_cast<E*>(out));
    return hip_check(hipGetLastError(), "delta_kernel");
}

vxg_status launch_delta(int width, const void* bases, const void* deltas, uint64_t n_deltas,
                        uint64_t offset, uint64_t len, void* out, hipStream_t s) {
    switch (width) {
    case 1: return delta_t<uint8_t>(bases, deltas, n_deltas, offset, len, out, s);
    case 2: return delta_t<uint16_t>(bases, deltas, n_deltas, offset, len, out, s);
    case 4: return delta_t<uint32_t>(bases, deltas, n_deltas, offset, len, out, s);
    case 8: return delta_t<uint64_t>(bases, deltas, n_deltas, offset, len, out, s);
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
}

// ------------------------------------------------------------------ K8 RunEnd expand
// (kernels below: runend_runs_kernel for short runs, runend_chunks_kernel for long ones; a
// single array is a one-chunk table, launch_runend at the end of this section)
// Chunk-table form.  A workgroup expands outputs [j0, j0 + 2048) of one chunk:
//   * wave 0 finds the runs holding j0 and the range's last output with 64-ary searches over the
//     ends (3-4 dependent loads, not a 14-step binary search per thread);
//   * every run of the range writes its index at its first output position (a run head) into
//     LDS, an inclusive max-scan fills the positions between heads;
//   * outputs are written coalesced: out[j] = values[run(j)].
// Ends are trimmed as the reference does: min(ends[r] - offset, len) (runend/compress.rs:140).
__device__ __forceinline__ uint64_t runend_first_gt(const void* ends, int ew, uint64_t offset, uint64_t n_runs,
                                                    uint64_t j) {
    // first run r with ends[r] - offset > j (n_runs if none); wave-uniform result, one wave
    const int lane = threadIdx.x & 63;
    uint64_t lo = 0, hi = n_runs;
    while (hi - lo > 64) {
        const uint64_t step = (hi - lo + 63) / 64;
        const uint64_t idx = lo + step * uint64_t(lane);
        const bool gt = idx < hi ? load_uint(ends, ew, false, idx) - offset > j : true;
        const unsigned long long bm = __ballot(gt);
        const int k = bm ? __ffsll(bm) - 1 : 64;
        const uint64_t nlo = k == 0 ? lo : lo + step * uint64_t(k - 1) + 1;
        const uint64_t nhi = k == 64 ? hi : (lo + step * uint64_t(k) < hi ? lo + step * uint64_t(k) : hi);
        lo = nlo;
        hi = nhi;
    }
    const uint64_t idx = lo + uint64_t(lane);
    const bool gt = idx < hi ? load_uint(ends, ew, false, idx) - offset > j : false;
    const unsigned long long bm = __ballot(gt);
    return bm ? lo + uint64_t(__ffsll(bm) - 1) : hi;
}

// First run r in [lo, hi) with ends[r] - offset > j (hi if none), one wave, wave-uniform result.
__device__ __forceinline__ uint64_t runend_first_gt_in(const void* ends, int ew, uint64_t offset, uint64_t lo,
                                                       uint64_t hi, uint64_t j) {
    const int lane = threadIdx.x & 63;
    while (hi - lo > 64) {
        const uint64_t step = (hi - lo + 63) / 64;
        const uint64_t idx = lo + step * uint64_t(lane);
        const bool gt = idx < hi ? load_uint(ends, ew, false, idx) - offset > j : true;
        const unsigned long long bm = __ballot(gt);
        const int k = bm ? __ffsll(bm) - 1 : 64;
        const uint64_t nlo = k == 0 ? lo : lo + step * uint64_t(k - 1) + 1;
        const uint64_t nhi = k == 64 ? hi : (lo + step * uint64_t(k) < hi ? lo + step * uint64_t(k) : hi);
        lo = nlo;
        hi = nhi;
    }
    const uint64_t idx = lo + uint64_t(lane);
    const bool gt = idx < hi ? load_uint(ends, ew, false, idx) - offset > j : false;
    const unsigned long long bm = __ballot(gt);
    return bm ? lo + uint64_t(__ffsll(bm) - 1) : hi;
}

// The run holding output j: an interpolated guess (j * n_runs / len) probed by one wave at 64
// points 64 runs apart, then the 64 runs of the bracket -- two dependent loads when the run
// lengths are near-uniform (the usual case), a 64-ary search of the rest otherwise.
__device__ __forceinline__ uint64_t runend_locate(const void* ends, int ew, uint64_t offset, uint64_t n_runs,
                                                  uint64_t len, uint64_t j) {
    const int lane = threadIdx.x & 63;
    constexpr uint64_t S = 64;
    const uint64_t guess = uint64_t(double(j) / double(len) * double(n_runs));
    const uint64_t base = guess > 32 * S ? guess - 32 * S : 0;
    if (base >= n_runs) return runend_first_gt_in(ends, ew, offset, 0, n_runs, j);
    const uint64_t idx = base + S * uint64_t(lane);
    const bool gt = idx < n_runs ? load_uint(ends, ew, false, idx) - offset > j : true;
    const unsigned long long bm = __ballot(gt);
    if (bm & 1ull) return base == 0 ? 0 : runend_first_gt_in(ends, ew, offset, 0, base + 1, j);
    if (bm == 0) return runend_first_gt_in(ends, ew, offset, base + 63 * S + 1, n_runs, j);
    const int k = __ffsll(bm) - 1;  // probe k is > j, probe k - 1 is not
    const uint64_t lo = base + S * uint64_t(k - 1) + 1;
    const uint64_t hi = base + S * uint64_t(k) < n_runs ? base + S * uint64_t(k) + 1 : n_runs;
    return runend_first_gt_in(ends, ew, offset, lo, hi, j);
}

// A workgroup expands outputs [j0, j0 + kRunEndSpan) of one chunk:
//   * wave 0 locates r0, the run holding j0 (runend_locate); the chunk's last end is checked
//     to cover the chunk (an independent load);
//   * every thread loads the ends of 4 runs at once (r0 + t + 256 i): the run after run r starts
//     at ends[r] - offset, and each start inside the range records its run index (a run head) in
//     LDS -- repeated while the last start is still inside, so no search for the range's end;
//   * an inclusive max-scan fills the positions between heads;
//   * outputs are written coalesced: out[j] = values[run(j)] (non-temporal).
// Ends are trimmed as the reference does: min(ends[r] - offset, len) (runend/compress.rs:140).
template <typename V>
__global__ __launch_bounds__(kBlock) void runend_chunks_kernel(RunEndTable tab) {
    constexpr int SPAN = int(kRunEndSpan), PER = SPAN / kBlock;
    __shared__ uint32_t s_head[SPAN];
    __shared__ uint32_t s_wmax[kBlock / 64];
    __shared__ uint64_t s_r0;
    __shared__ int s_bad;
    const uint64_t g = blockIdx.x;
    RunEndChunk c;  // this workgroup's chunk: kernarg table (binary search) or a plan's device table
    if (tab.ext) {
        c = tab.ext[ext_chunk_index(tab.ext, tab.n, g, [](RunEndChunk const& d) { return d.first_group; })];
    } else {
        uint32_t lo = 0, hi = tab.n;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tab.c[mid].first_group <= g) lo = mid; else hi = mid;
        }
        c = tab.c[lo];
    }
    const V* __restrict__ values = static_cast<const V*>(c.values.p);  // plain columns only
    const void* ends = c.ends.p;
    V* __restrict__ out = static_cast<V*>(c.out);
    const int ew = c.ends.width, tid = threadIdx.x;
    const uint64_t j0 = (g - c.first_group) * SPAN;
    const int jn = int(c.len - j0 < uint64_t(SPAN) ? c.len - j0 : uint64_t(SPAN));
    const uint64_t jend = j0 + uint64_t(jn);
    if (tid < 64) {
        const uint64_t r0 = runend_locate(ends, ew, c.offset, c.n_runs, c.len, j0);
        if (tid == 0) s_r0 = r0;
    } else if (tid == 64) {  // the last run must reach the chunk's end
        s_bad = c.n_runs == 0 || load_uint(ends, ew, false, c.n_runs - 1) - c.offset < c.len;
    }
#pragma unroll
    for (int k = 0; k < PER; k++) s_head[tid + k * kBlock] = 0;
    __syncthreads();
    if (s_bad) {  // the ends do not reach the end of the array
        if (tid == 0) __hip_atomic_fetch_or(tab.err, kErrRunEnd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const uint64_t r0 = s_r0;
    // run heads: run r + 1 starts at ends[r] - offset (> j0 for r >= r0)
    constexpr int Q = 4;
    for (uint64_t rb = r0;; rb += uint64_t(Q) * kBlock) {
        uint64_t st[Q];
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const uint64_t r = rb + uint64_t(q) * kBlock + uint64_t(tid);
            st[q] = r + 1 < c.n_runs ? load_uint(ends, ew, false, r) - c.offset : ~0ull;
        }
#pragma unroll
        for (int q = 0; q < Q; q++)
            if (st[q] < jend) s_head[st[q] - j0] = uint32_t(rb + uint64_t(q) * kBlock + uint64_t(tid) + 1 - r0);
        if (!__syncthreads_or(st[Q - 1] < jend)) break;
    }
    __syncthreads();
    // inclusive max-scan of s_head: thread t owns entries [PER t, PER t + PER)
    uint32_t v[PER];
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        m = max(m, s_head[tid * PER + k]);
        v[k] = m;
    }
    uint32_t x = m;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if ((tid & 63) >= d) x = max(x, y);
    }
    if ((tid & 63) == 63) s_wmax[tid >> 6] = x;
    __syncthreads();
    uint32_t before = __shfl_up(x, 1, 64);
    if ((tid & 63) == 0) before = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; w++)
        if (w < (tid >> 6)) before = max(before, s_wmax[w]);
#pragma unroll
    for (int k = 0; k < PER; k++) s_head[tid * PER + k] = max(v[k], before);
    __syncthreads();
    for (int i = tid; i < jn; i += kBlock) nt_store(out + j0 + i, gload(values + r0 + s_head[i]));
}

template <typename V>
__global__ __launch_bounds__(kBlock) void runend_runs_kernel(RunEndTable tab) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[runs_lds_bytes<V>()];
    const uint64_t g = blockIdx.x;
    RunEndChunk c;
    if (tab.ext) {
        c = tab.ext[ext_chunk_index(tab.ext, tab.n, g, [](RunEndChunk const& d) { return d.first_group; })];
    } else {
        uint32_t lo = 0, hi = tab.n;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tab.c[mid].first_group <= g) lo = mid; else hi = mid;
        }
        c = tab.c[lo];
    }
    runend_runs_body<V>(c, g, tab.err, lds);
}

vxg_status launch_runend_runs(int value_width, const RunEndTable& t, uint64_t groups, hipStream_t s) {
    if (groups == 0) return VXG_OK;
    switch (value_width) {
#define RR_CASE(W)                                                                                                \
    case W:                                                                                                       \
        hipLaunchKernelGGL((runend_runs_kernel<typename UInt<W>::t>), dim3(unsigned(groups)), dim3(kBlock), 0, s, t); \
        break;
        RR_CASE(1) RR_CASE(2) RR_CASE(4) RR_CASE(8) RR_CASE(16)
#undef RR_CASE
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
    return hip_check(hipGetLastError(), "runend_runs_kernel");
}

vxg_status launch_runend_chunks(int value_width, const RunEndTable& t, uint64_t groups, hipStream_t s) {
    if (groups == 0) return VXG_OK;
    switch (value_width) {
#define RE_CASE(W)                                                                                  \
    case W:                                                                                         \
        hipLaunchKernelGGL((runend_chunks_kernel<typename UInt<W>::t>), dim3(unsigned(groups)), dim3(kBlock), 0, s, t); \
        break;
        RE_CASE(1) RE_CASE(2) RE_CASE(4) RE_CASE(8) RE_CASE(16)
#undef RE_CASE
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
    return hip_check(hipGetLastError(), "runend_chunks_kernel");
}

vxg_status launch_runend(int value_width, const RunEndChunk& chunk, uint32_t* err, hipStream_t s) {
    if (chunk.len == 0) return VXG_OK;
    if (chunk.n_runs == 0) return set_error(VXG_ERR_INVALID_ARGUMENT, "RunEnd with len > 0 has no runs");
    RunEndTable t{};
    t.err = err;
    t.n = 1;
    t.c[0] = chunk;
    t.c[0].first_group = 0;
    if (chunk.len <= kRunEndShortRun * chunk.n_runs)
        return launch_runend_runs(value_width, t, (chunk.n_runs + kRunEndRunsPerGroup - 1) / kRunEndRunsPerGroup, s);
    if (chunk.ends.packed || chunk.values.packed)
        return set_error(VXG_ERR_INVALID_ARGUMENT, "long-run RunEnd expansion reads plain ends/values");
    return launch_runend_chunks(value_width, t, (chunk.len + kRunEndSpan - 1) / kRunEndSpan, s);
}

// ------------------------------------------------------------------ K10 fill
template <typename V>
__global__ __launch_bounds__(kBlock) void fill_kernel(V v, uint64_t n, V* __restrict__ out) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) nt_store(out + i, v);
}

vxg_status launch_fill(int value_width, const uint8_t* scalar16, uint64_t n, void* out, hipStream_t s) {
    if (n == 0) return VXG_OK;
    const unsigned g = grid_for(n);
    switch (value_width) {
#define FILL_CASE(W)                                                                                \
    case W: {                                                                                       \
        typename UInt<W>::t v;                                                                      \
        __builtin_memcpy(&v, scalar16, W);                                                          \
        hipLaunchKernelGGL((fill_kernel<typename UInt<W>::t>), dim3(g), dim3(kBlock), 0, s, v, n,   \
                           static_cast<typename UInt<W>::t*>(out));                                 \
    } break;
        FILL_CASE(1) FILL_CASE(2) FILL_CASE(4) FILL_CASE(8) FILL_CASE(16)
#undef FILL_CASE
    default: return VXG_ERR_INVALID_ARGUMENT;
    }
    return hip_check(hipGetLastError(), "fill_kernel");
}

// ------------------------------------------------------------------ K10 byte copy / zero
// dst[0, n) = src[0, n) (src null: zeros).  The planner's device-to-device copies and zero fills
// are kernels rather than hipMemcpyAsync / hipMemsetAsync: inside a recorded plan those become
// graph memcpy/memset nodes, and a memset node at the root of a replayed graph was measured to
// leave stale bits that the following kernels' atomic ORs then kept (profiles/r05_plan_memset.md);
// kernel nodes also keep a plan eligible for direct replay.  The body is 16-byte stores at dst's
// 16-byte alignment.  When src is misaligned against dst by r bytes (a chunked
// column's slice after a chunk whose byte length is not a multiple of 16, a sliced VarBin byte
// buffer), each 16-byte chunk is assembled from the two aligned 16-byte source words holding it
// with byte funnel shifts (v_alignbyte_b32; r is uniform over the launch, so the word select is a
// uniform branch).  Both words hold a byte of the source range, so neither load leaves its pages.
__device__ __forceinline__ uint32_t abyte(uint32_t hi, uint32_t lo, uint32_t sh) {
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
template <int QD>
__device__ __forceinline__ uint4 funnel16(const uint4& lo, const uint4& hi, uint32_t rb) {
    const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    return make_uint4(abyte(w[QD + 1], w[QD], rb), abyte(w[QD + 2], w[QD + 1], rb), abyte(w[QD + 3], w[QD + 2], rb),
                      abyte(w[QD + 4], w[QD + 3], rb));
}

__global__ __launch_bounds__(kBlock) void copy_bytes_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                            uint64_t n, uint64_t head, uint64_t body, uint32_t r) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    const uint64_t t0 = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    uint4* const d16 = reinterpret_cast<uint4*>(dst + head);
    if (!src) {
        for (uint64_t q = t0; q < body; q += stride) gstore(d16 + q, make_uint4(0, 0, 0, 0));
    } else if (r == 0) {  // 16-byte chunks after the head
        const uint4* const s16 = reinterpret_cast<const uint4*>(src + head);
        for (uint64_t q = t0; q < body; q += stride) gstore(d16 + q, gload(s16 + q));
    } else {
        const uint4* const s16 = reinterpret_cast<const uint4*>(src + head - r);  // aligned
        const uint32_t qd = r >> 2, rb = r & 3;
        for (uint64_t q = t0; q < body; q += stride) {
            const uint4 lo = gload(s16 + q), hi = gload(s16 + q + 1);
            uint4 v;
            if (qd == 0) v = funnel16<0>(lo, hi, rb);
            else if (qd == 1) v = funnel16<1>(lo, hi, rb);
            else if (qd == 2) v = funnel16<2>(lo, hi, rb);
            else v = funnel16<3>(lo, hi, rb);
            gstore(d16 + q, v);
        }
    }
    const uint64_t tail0 = head + 16 * body, edge = head + (n - tail0);  // head bytes + tail bytes
    for (uint64_t k = t0; k < edge; k += stride) {
        const uint64_t i = k < head ? k : tail0 + (k - head);
        gstore(dst + i, src ? gload(src + i) : uint8_t(0));
    }
}

vxg_status launch_copy_bytes(void* dst, const void* src, uint64_t n, hipStream_t s) {
    if (n == 0) return VXG_OK;
    const uintptr_t d = reinterpret_cast<uintptr_t>(dst), a = reinterpret_cast<uintptr_t>(src);
    const uint64_t head = std::min<uint64_t>(n, (16 - (d & 15)) & 15);
    const uint64_t body = (n - head) / 16;
    const uint32_t r = src ? uint32_t((a + head) & 15) : 0u;
    const uint64_t work = std::max<uint64_t>(body, 32);
    hipLaunchKernelGGL(copy_bytes_kernel, dim3(grid_for(work)), dim3(kBlock), 0, s, static_cast<uint8_t*>(dst),
                       static_cast<const uint8_t*>(src), n, head, body, r);
    return hip_check(hipGetLastError(), "copy_bytes_kernel");
}

// ------------------------------------------------------------------ VarBin -> views
// arrow-array 53.2 make_view: len<=12 inline (zero padded), else {len, prefix, 0, offset};
// null rows -> all-zero view (GenericByteViewBuilder::append_null).
// Byte positions are compile-time (unrolled j) so nothing is a runtime-indexed register array
// (which hipcc places in scratch); reads are guarded by j < len.
__device__ __forceinline__ uint4 make_view(const uint8_t* __restrict__ heap, uint64_t start, uint32_t len,
                                          uint32_t bidx) {
    const uint8_t* p = heap + start;
    uint32_t w1 = 0, w2 = 0, w3 = 0;
    if (len <= 12) {
#pragma unroll
        for (int j = 0; j < 12; j++) {
            const uint32_t b = uint32_t(j) < len ? uint32_t(gload(p + j)) : 0u;
            if (j < 4) w1 |= b << (8 * j);
            else if (j < 8) w2 |= b << (8 * (j - 4));
            else w3 |= b << (8 * (j - 8));
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) w1 |= uint32_t(gload(p + j)) << (8 * j);
        w2 = bidx;
        w3 = uint32_t(start);
    }
    return make_uint4(len, w1, w2, w3);
}

// A row whose offsets are not a <= e <= heap_len gets an all-zero view and sets kErrVarBin.
__device__ __forceinline__ uint4 checked_view(const uint8_t* __restrict__ heap, uint64_t heap_len, uint64_t a,
                                              uint64_t e, uint32_t bidx, uint32_t* err) {
    if (a > e || e > heap_len) {
        __hip_atomic_fetch_or(err, kErrVarBin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return make_uint4(0, 0, 0, 0);
    }
    return make_view(heap, a, uint32_t(e - a), bidx);
}

__global__ __launch_bounds__(kBlock) void varbin_views_kernel(const uint8_t* __restrict__ heap, uint64_t heap_len,
                                                              const void* offs, int offs_width, uint64_t n,
                                                              const uint8_t* __restrict__ validity,
                                                              uint32_t bidx, uint4* __restrict__ views, uint32_t* err) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (validity && !((validity[i >> 3] >> (i & 7)) & 1)) {
            views[i] = make_uint4(0, 0, 0, 0);
            continue;
        }
        const uint64_t a = load_uint(offs, offs_width, offs_width < 8, i);
        const uint64_t b = load_uint(offs, offs_width, offs_width < 8, i + 1);
        views[i] = checked_view(heap, heap_len, a, b, bidx, err);
    }
}

vxg_status launch_varbin_views(const uint8_t* heap, uint64_t heap_len, int offs_width, const void* offsets, uint64_t n,
                               const uint8_t* validity, uint32_t bidx, uint8_t* views, uint32_t* err, hipStream_t s) {
    if (n == 0) return VXG_OK;
    hipLaunchKernelGGL(varbin_views_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, heap, heap_len, offsets,
                       offs_width, n, validity, bidx, reinterpret_cast<uint4*>(views), err);
    return hip_check(hipGetLastError(), "varbin_views_kernel");
}

// Chunk-table VarBin -> views: workgroup g of a chunk copies its share of the bytes into the
// output data buffer and builds the views of rows [256 (g - first_group), +256).
__global__ __launch_bounds__(kBlock) void varbin_chunks_kernel(VarBinTable tab) {
    const uint64_t g = blockIdx.x;
    VarBinChunk c;  // this workgroup's chunk: kernarg table (binary search) or a plan's device table
    if (tab.ext) {
        c = tab.ext[ext_chunk_index(tab.ext, tab.n, g, [](VarBinChunk const& d) { return d.first_group; })];
    } else {
        uint32_t lo = 0, hi = tab.n;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tab.c[mid].first_group <= g) lo = mid; else hi = mid;
        }
        c = tab.c[lo];
    }
    const uint64_t lg = g - c.first_group;
    const uint64_t ng = (c.n + kBlock - 1) / kBlock > 0 ? (c.n + kBlock - 1) / kBlock : 1;
    const uint64_t per = (c.bytes + ng - 1) / ng;
    for (uint64_t b = lg * per + threadIdx.x; b < c.bytes && b < (lg + 1) * per; b += kBlock) gstore(c.dst + b, gload(c.src + b));
    const uint64_t i = lg * kBlock + threadIdx.x;
    if (i < c.n) {
        const uint64_t a = load_uint(c.offsets, int(c.offs_width), c.offs_width < 8, i);
        const uint64_t e = load_uint(c.offsets, int(c.offs_width), c.offs_width < 8, i + 1);
        gstore(reinterpret_cast<uint4*>(c.views) + i, checked_view(c.src, c.bytes, a, e, c.bidx, tab.err));
    }
}

vxg_status launch_varbin_chunks(const VarBinTable& t, uint64_t groups, hipStream_t s) {
    if (groups == 0) return VXG_OK;
    hipLaunchKernelGGL(varbin_chunks_kernel, dim3(unsigned(groups)), dim3(kBlock), 0, s, t);
    return hip_check(hipGetLastError(), "varbin_chunks_kernel");
}

// pack_views (chunked/canonical.rs:214-231): copy views, adding `add` to the buffer_index of
// every non-inlined view (len > 12); inlined views are copied unchanged.
__global__ __launch_bounds__(kBlock) void views_rebase_kernel(const uint4* __restrict__ src, uint64_t n, uint32_t add,
                                                              uint4* __restrict__ dst) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint4 v = src[i];
        if (v.x > 12) v.z += add;
        dst[i] = v;
    }
}

vxg_status launch_views_rebase(const uint8_t* src, uint64_t n, uint32_t add, uint8_t* dst, hipStream_t s) {
    if (n == 0) return VXG_OK;
    hipLaunchKernelGGL(views_rebase_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       reinterpret_cast<const uint4*>(src), n, add, reinterpret_cast<uint4*>(dst));
    return hip_check(hipGetLastError(), "views_rebase_kernel");
}

// ---- Bool canonical: LSB bit buffers (arrow BooleanBuffer) ------------------------------
// Every bool producer ORs 32-bit words into a zeroed bit buffer at an arbitrary bit position
// (a chunk of a ChunkedArray starts anywhere); a full word at a 32-aligned position is owned
// by its producer and stored plainly, ragged ones are split over two words with atomics.
__device__ __forceinline__ void put_bits(uint32_t* __restrict__ dst, uint64_t pos, uint32_t word, bool full) {
    const uint64_t w = pos >> 5;
    const int sh = int(pos & 31);
    if (full && sh == 0) {
        dst[w] = word;
        return;
    }
    if (!word) return;
    atomicOr(dst + w, word << sh);
    if (sh) {
        const uint32_t hi = word >> (32 - sh);
        if (hi) atomicOr(dst + w + 1, hi);
    }
}

// RunEndBool (runend-bool/src/compress.rs:46-93): the value flips at every trimmed run end, so
// a workgroup of 8192 bits finds the run holding its first bit (one wave, 64-ary search), XORs
// a flip bit at every run end inside its span into LDS (zero-length runs flip twice = not at
// all, like the reference's empty appends), and turns flips into values with an in-word
// prefix XOR plus a block XOR-scan of word parities.  Writes are whole words.
constexpr int kBoolSpan = 32 * kBlock;
__global__ __launch_bounds__(kBlock) void runend_bool_kernel(const void* __restrict__ ends, int ew, uint64_t n_runs,
                                                             uint64_t offset, int start, uint64_t len,
                                                             uint32_t* __restrict__ dst, uint64_t dst_off,
                                                             uint32_t* __restrict__ err) {
    __shared__ uint32_t s_flip[kBlock];
    __shared__ uint32_t s_wpar[kBlock / 64];
    __shared__ uint64_t s_r0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t j0 = uint64_t(blockIdx.x) * kBoolSpan;
    const uint64_t jend = len - j0 < uint64_t(kBoolSpan) ? len : j0 + kBoolSpan;
    s_flip[tid] = 0;
    if (tid < 64) {
        const uint64_t r0 = runend_first_gt(ends, ew, offset, n_runs, j0);
        if (tid == 0) s_r0 = r0;
        // the trimmed ends must reach len (the reference appends exactly len bits)
        if (blockIdx.x == 0 && tid == 0 && load_uint(ends, ew, false, n_runs - 1) - offset < len)
            __hip_atomic_fetch_or(err, kErrRunEnd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const uint64_t r0 = s_r0;
    if (r0 >= n_runs) {  // bits past the last run end (flagged above)
        return;
    }
    for (uint64_t r = r0 + tid; r < n_runs; r += kBlock) {
        const uint64_t e = load_uint(ends, ew, false, r) - offset;
        if (e >= jend) break;  // ends increase: so do all later ones
        const uint32_t p = uint32_t(e - j0);  // > 0: ends[r] - offset > j0 for r >= r0
        atomicXor(&s_flip[p >> 5], 1u << (p & 31));
    }
    __syncthreads();
    const uint32_t f = s_flip[tid];
    uint32_t x = f;  // inclusive prefix XOR inside the word
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    x ^= x << 16;
    const unsigned long long bal = __ballot(__popc(f) & 1);
    const uint32_t below = uint32_t(__popcll(bal & ((1ull << lane) - 1ull)) & 1);
    if (lane == 0) s_wpar[wave] = uint32_t(__popcll(bal) & 1);
    __syncthreads();
    uint32_t carry = below ^ uint32_t(start != 0) ^ uint32_t(r0 & 1);  // value_at_index(r0, start)
    for (int w = 0; w < wave; w++) carry ^= s_wpar[w];
    uint32_t word = x ^ (carry ? 0xFFFFFFFFu : 0u);
    const uint64_t p0 = j0 + uint64_t(tid) * 32;
    if (p0 >= jend) return;
    const uint64_t nb = jend - p0;
    if (nb < 32) word &= (1u << nb) - 1u;
    put_bits(dst, dst_off + p0, word, nb >= 32);
}

vxg_status launch_runend_bool(const void* ends, int ew, uint64_t n_runs, uint64_t offset, bool start, uint64_t len,
                              void* dst, uint64_t dst_off, uint32_t* err, hipStream_t s) {
    if (len == 0) return VXG_OK;
    if (n_runs == 0) return set_error(VXG_ERR_INVALID_ARGUMENT, "Ends array must have at least one element");
    const uint64_t groups = (len + kBoolSpan - 1) / kBoolSpan;
    if (groups > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "RunEndBool too long");
    hipLaunchKernelGGL(runend_bool_kernel, dim3(unsigned(groups)), dim3(kBlock), 0, s, ends, ew, n_runs, offset,
                       int(start), len, static_cast<uint32_t*>(dst), dst_off, err);
    return hip_check(hipGetLastError(), "runend_bool_kernel");
}

// ByteBool (bytebool/src/array.rs:138-146): 32 bytes -> one word per thread (byte != 0).
__device__ __forceinline__ uint32_t nonzero_nibble(uint32_t v) {
    const uint32_t m = (((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;  // bit 7 of each byte != 0
    const uint32_t b = m >> 7;                                                  // bits 0, 8, 16, 24
    return (b | (b >> 7) | (b >> 14) | (b >> 21)) & 0xFu;
}

__global__ __launch_bounds__(kBlock) void bytebool_kernel(const uint8_t* __restrict__ src, uint64_t n,
                                                          uint32_t* __restrict__ dst, uint64_t dst_off) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t w = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; w * 32 < n; w += stride) {
        const uint64_t p0 = w * 32;
        uint32_t word = 0;
        if (p0 + 32 <= n && (reinterpret_cast<uintptr_t>(src + p0) & 15) == 0) {
            const uint4 a = reinterpret_cast<const uint4*>(src + p0)[0];
            const uint4 b = reinterpret_cast<const uint4*>(src + p0)[1];
            const uint32_t q[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int k = 0; k < 8; k++) word |= nonzero_nibble(q[k]) << (4 * k);
        } else {
            for (int k = 0; k < 32 && p0 + k < n; k++) word |= uint32_t(src[p0 + k] != 0) << k;
        }
        put_bits(dst, dst_off + p0, word, p0 + 32 <= n);
    }
}

vxg_status launch_bytebool(const uint8_t* src, uint64_t n, void* dst, uint64_t dst_off, hipStream_t s) {
    if (n == 0) return VXG_OK;
    hipLaunchKernelGGL(bytebool_kernel, dim3(grid_for((n + 31) / 32)), dim3(kBlock), 0, s, src, n,
                       static_cast<uint32_t*>(dst), dst_off);
    return hip_check(hipGetLastError(), "bytebool_kernel");
}

// Sparse bools (sparse/flatten.rs:41-61): bit (dst_off + idx - ioff) = values bit i.
__global__ __launch_bounds__(kBlock) void assign_bits_at_kernel(uint32_t* __restrict__ dst, uint64_t dst_off,
                                                                const void* idx, int iw, int isg, uint64_t ioff,
                                                                uint64_t n, uint64_t len,
                                                                const uint8_t* __restrict__ vals) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t p = load_uint(idx, iw, isg != 0, i) - ioff;
        if (p >= len) continue;
        const uint64_t q = dst_off + p;
        const uint32_t bit = 1u << (q & 31);
        if ((vals[i >> 3] >> (i & 7)) & 1) atomicOr(dst + (q >> 5), bit);
        else atomicAnd(dst + (q >> 5), ~bit);
    }
}

vxg_status launch_assign_bits_at(void* dst, uint64_t dst_off, const void* idx, int iw, bool isg, uint64_t ioff,
                                 uint64_t n, uint64_t len, const uint8_t* vals, hipStream_t s) {
    if (n == 0) return VXG_OK;
    hipLaunchKernelGGL(assign_bits_at_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, static_cast<uint32_t*>(dst),
                       dst_off, idx, iw, int(isg), ioff, n, len, vals);
    return hip_check(hipGetLastError(), "assign_bits_at_kernel");
}

// Validity of take(values, codes) (primitive/compute/take.rs:58-67 -> Validity::take): bit i =
// values_valid[codes[i]], 32 rows per thread, whole words into a zeroed bitmap at bit 0.
__global__ __launch_bounds__(kBlock) void gather_bits_kernel(uint32_t* __restrict__ dst, const void* codes, int cw,
                                                             bool csg, uint64_t n, const uint8_t* __restrict__ src,
                                                             uint64_t n_values, uint32_t* __restrict__ err) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t w = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; w * 32 < n; w += stride) {
        uint32_t word = 0;
        bool oob = false;
        for (int k = 0; k < 32; k++) {
            const uint64_t i = w * 32 + k;
            if (i >= n) break;
            const uint64_t c = load_uint(codes, cw, csg, i);  // negative -> huge -> out of bounds
            oob |= c >= n_values;
            word |= (c < n_values ? uint32_t((src[c >> 3] >> (c & 7)) & 1) : 0u) << k;
        }
        if (oob) __hip_atomic_fetch_or(err, kErrTakeOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dst[w] = word;
    }
}

vxg_status launch_gather_bits(void* dst, const void* codes, int cw, bool csg, uint64_t n, const uint8_t* src,
                              uint64_t n_values, uint32_t* err, hipStream_t s) {
    if (n == 0) return VXG_OK;
    hipLaunchKernelGGL(gather_bits_kernel, dim3(grid_for((n + 31) / 32)), dim3(kBlock), 0, s,
                       static_cast<uint32_t*>(dst), codes, cw, csg, n, src, n_values, err);
    return hip_check(hipGetLastError(), "gather_bits_kernel");
}

}  // namespace vxg
