// encode_gpu.hip — the compressor side on the GPU: the encoders whose
// output the decode path consumes, restated as CDNA4 kernels.
//
//   int stats    min / max / trailing zeros / bit-width histogram of a primitive column:
//                vortex-array/src/stats (trailing_zeros stats/mod.rs:178-189, bit_width_freq),
//                what for_compress (for/compress.rs:13-58) and the BitPacked compressor's
//                best_bit_width (bitpacking/compress.rs; compressors/bitpacked.rs) decide on
//   K15 pack     fastlanes BitPacking::unchecked_pack as used by bitpack_primitive
//                (bitpacking/compress.rs:82-137), optionally fused with FoR's compress_primitive
//                ((v - min) >> shift, for/compress.rs:61-84): the inverse of K1 — 8 threads per
//                1024-value block, each owning 16 bytes of every row, rows read with 16-byte loads
//                at index(row, lane), packed words built in registers (W, T template
//                parameters), W 16-byte stores per thread
//   patches      gather_patches (bitpacking/compress.rs:138-163): the sorted indices and values of
//                the elements wider than W (ordered stream compaction: tile counts, one-workgroup
//                scan, ordered scatter)
//   ALP encode   ALPFloat::encode (alp/mod.rs:114-246): find_best_exponents over the reference's
//                strided sample (every (e, f) pair scored by one thread; the host picks in the
//                reference's iteration order), encode_single_unchecked / decode_single round trip
//                per value, exceptions compacted, and the reference's fill-forward (every
//                exception's slot takes the first non-exception's encoded value)
// Float arithmetic uses explicit round-to-nearest intrinsics (no contraction), so every encoded
// integer and every exception decision is the host encoder's (vortex_amd/csrc/encode.cpp).
#include <limits>
#include <type_traits>
#include <vector>

#include "encode_gpu.hpp"
#include "fl_unpack_impl.hpp"

#define VXG_TRY_E(expr)              \
    do {                             \
        vxg_status _s = (expr);      \
        if (_s != VXG_OK) return _s; \
    } while (0)

namespace vxg {

namespace {

constexpr int kEB = 256;

inline unsigned egrid(uint64_t n_threads, uint64_t cap = 256ull * 8 * 16) {
    uint64_t g = (n_threads + kEB - 1) / kEB;
    if (g > cap) g = cap;
    return unsigned(g ? g : 1);
}

// ------------------------------------------------------------------ stats
struct StatsDev {
    unsigned long long min_key, max_key;  // order-preserving keys (sign bit flipped for signed)
    unsigned long long or_bits;
    unsigned long long freq[65];
};

template <typename E, bool SGN>
__global__ __launch_bounds__(kEB) void int_stats_kernel(const E* __restrict__ v, uint64_t n, StatsDev* out) {
    constexpr int T = 8 * sizeof(E);
    __shared__ unsigned long long s_freq[65];
    for (int i = threadIdx.x; i < 65; i += kEB) s_freq[i] = 0;
    __syncthreads();
    unsigned long long mn = ~0ull, mx = 0, orb = 0;
    const uint64_t stride = uint64_t(gridDim.x) * kEB;
    for (uint64_t i = uint64_t(blockIdx.x) * kEB + threadIdx.x; i < n; i += stride) {
        const uint64_t x = uint64_t(v[i]) & (T == 64 ? ~0ull : ((1ull << T) - 1));
        const unsigned long long key = SGN ? (x ^ (1ull << (T - 1))) : x;
        mn = key < mn ? key : mn;
        mx = key > mx ? key : mx;
        orb |= x;
        // histogram: one LDS add per distinct bit width in the wave (values of a column share a
        // handful of widths; per-lane atomics on one address would serialize 64-way)
        const unsigned b = x ? unsigned(64 - __clzll(x)) : 0u;
        unsigned long long todo = __ballot(true);
        while (todo) {
            const int leader = __ffsll(todo) - 1;
            const unsigned b0 = __shfl(b, leader, 64);
            const unsigned long long same = __ballot(b == b0) & todo;
            if ((threadIdx.x & 63) == unsigned(leader)) atomicAdd(&s_freq[b0], (unsigned long long)__popcll(same));
            todo &= ~same;
        }
    }
    // wave reductions, then one atomic per wave
    for (int d = 32; d > 0; d >>= 1) {
        const unsigned long long a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64), c = __shfl_xor(orb, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
        orb |= c;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&out->min_key, mn);
        atomicMax(&out->max_key, mx);
        atomicOr(&out->or_bits, orb);
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= T; i += kEB)
        if (s_freq[i]) atomicAdd(&out->freq[i], s_freq[i]);
}

// ------------------------------------------------------------------ FoR compress_primitive
// (for/compress.rs:61-84): (v wrapping_sub min) >> shift, arithmetic for signed ptypes
template <typename E, bool SGN>
__global__ __launch_bounds__(kEB) void for_encode_kernel(const E* __restrict__ v, uint64_t n, E ref, unsigned shift,
                                                         E* __restrict__ out) {
    const uint64_t stride = uint64_t(gridDim.x) * kEB;
    for (uint64_t i = uint64_t(blockIdx.x) * kEB + threadIdx.x; i < n; i += stride) {
        E d = E(v[i] - ref);
        if (shift) d = SGN ? E(std::make_signed_t<E>(d) >> shift) : E(d >> shift);
        out[i] = d;
    }
}

// ------------------------------------------------------------------ ordered compaction
// Tiles of kCTile elements: count the flagged ones, exclusive-scan the counts in one workgroup,
// then each tile writes its flagged (index, value) pairs in order at its offset.
constexpr int kCTile = 1024;

template <class Pred>
__global__ __launch_bounds__(kEB) void compact_count(Pred pred, uint64_t n, uint32_t* __restrict__ counts) {
    const uint64_t tile = blockIdx.x;
    uint32_t c = 0;
    for (int k = 0; k < kCTile / kEB; k++) {
        const uint64_t i = tile * kCTile + uint64_t(k) * kEB + threadIdx.x;
        c += i < n && pred(i);
    }
    __shared__ uint32_t s[kEB / 64];
    for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d, 64);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[tile] = s[0] + s[1] + s[2] + s[3];
}

// exclusive scan of counts[0..m) into offs (64-bit), total into offs[m]; one workgroup
__global__ __launch_bounds__(kEB) void compact_scan(const uint32_t* __restrict__ counts, uint64_t m,
                                                   unsigned long long* __restrict__ offs) {
    __shared__ unsigned long long s_ws[kEB / 64];
    __shared__ unsigned long long s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t base = 0; base < m; base += kEB) {
        const uint64_t i = base + threadIdx.x;
        const unsigned long long v = i < m ? counts[i] : 0ull;
        unsigned long long x = v;
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) s_ws[wave] = x;
        __syncthreads();
        unsigned long long before = s_carry, tot = 0;
        for (int w = 0; w < kEB / 64; w++) {
            before += w < wave ? s_ws[w] : 0ull;
            tot += s_ws[w];
        }
        if (i < m) offs[i] = before + x - v;
        __syncthreads();
        if (threadIdx.x == 0) s_carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) offs[m] = s_carry;
}

template <class Pred, class Emit>
__global__ __launch_bounds__(kEB) void compact_scatter(Pred pred, Emit emit, uint64_t n,
                                                       const unsigned long long* __restrict__ offs, uint64_t cap) {
    const uint64_t tile = blockIdx.x;
    __shared__ uint32_t s_ws[kEB / 64];
    unsigned long long base = offs[tile];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int k = 0; k < kCTile / kEB; k++) {
        const uint64_t i = tile * kCTile + uint64_t(k) * kEB + threadIdx.x;
        const bool f = i < n && pred(i);
        const unsigned long long bal = __ballot(f);
        const uint32_t below = uint32_t(__popcll(bal & ((1ull << lane) - 1ull)));
        if (lane == 0) s_ws[wave] = uint32_t(__popcll(bal));
        __syncthreads();
        uint32_t before = 0, tot = 0;
        for (int w = 0; w < kEB / 64; w++) {
            before += w < wave ? s_ws[w] : 0u;
            tot += s_ws[w];
        }
        const unsigned long long pos = base + before + below;
        if (f && pos < cap) emit(i, pos);
        base += tot;
        __syncthreads();
    }
}

template <typename E>
struct WiderThan {
    const E* v;
    unsigned W;
    __device__ bool operator()(uint64_t i) const {
        const uint64_t x = uint64_t(v[i]);
        return (x ? unsigned(64 - __clzll(x)) : 0u) > W;
    }
};
template <typename E>
struct EmitPatch {
    const E* v;
    uint64_t* idx;
    E* out;
    __device__ void operator()(uint64_t i, uint64_t pos) const {
        idx[pos] = i;
        out[pos] = v[i];
    }
};

// ------------------------------------------------------------------ ALP
template <typename F> struct AlpT;
template <> struct AlpT<double> {
    using I = int64_t;
    static constexpr int MAXE = 18;
    __device__ static double sweet() { return double(1ull << 52) + double(1ull << 51); }
    __device__ static double mul(double a, double b) { return __dmul_rn(a, b); }
    __device__ static double add(double a, double b) { return __dadd_rn(a, b); }
    __device__ static double sub(double a, double b) { return __dsub_rn(a, b); }
};
template <> struct AlpT<float> {
    using I = int32_t;
    static constexpr int MAXE = 10;
    __device__ static float sweet() { return float(1u << 23) + float(1u << 22); }
    __device__ static float mul(float a, float b) { return __fmul_rn(a, b); }
    __device__ static float add(float a, float b) { return __fadd_rn(a, b); }
    __device__ static float sub(float a, float b) { return __fsub_rn(a, b); }
};

// F10 / IF10 (alp/mod.rs:255-351, the engine's copies in capi.hip) by value
template <typename F> struct AlpTables { F f10[24]; F if10[24]; };

// Rust `as` float -> int: saturating, NaN -> 0
template <typename I, typename F>
__device__ __forceinline__ I sat_cast(F x) {
    if (x != x) return 0;
    if (x >= F(static_cast<double>(std::numeric_limits<I>::max()))) return std::numeric_limits<I>::max();
    if (x <= F(static_cast<double>(std::numeric_limits<I>::min()))) return std::numeric_limits<I>::min();
    return I(x);
}

// encode_single_unchecked: (v * F10[e] * IF10[f]).fast_round().as_int()  (alp/mod.rs:46-49, 165-170)
template <typename F>
__device__ __forceinline__ typename AlpT<F>::I alp_enc(F v, F f10e, F if10f) {
    F x = AlpT<F>::mul(AlpT<F>::mul(v, f10e), if10f);
    x = AlpT<F>::sub(AlpT<F>::add(x, AlpT<F>::sweet()), AlpT<F>::sweet());
    return sat_cast<typename AlpT<F>::I>(x);
}
// decode_single: (enc as F) * F10[f] * IF10[e]  (alp/mod.rs:161-163)
template <typename F>
__device__ __forceinline__ F alp_dec(typename AlpT<F>::I enc, F f10f, F if10e) {
    return AlpT<F>::mul(AlpT<F>::mul(F(enc), f10f), if10e);
}

// find_best_exponents (alp/mod.rs:51-86): thread p scores pair p of the reference's order (e
// descending, f < e ascending) on the sample: encode (+ the chunk's fill-forward, the sample is
// one encode chunk), estimate_encoded_size (:88-111).  The host picks the best in that order.
template <typename F>
__global__ __launch_bounds__(kEB) void alp_search_kernel(const F* __restrict__ sample, uint32_t ns, AlpTables<F> tb,
                                                         unsigned long long* __restrict__ sizes) {
    using I = typename AlpT<F>::I;
    constexpr int MAXE = AlpT<F>::MAXE;
    const int p = threadIdx.x;
    int e = -1, f = 0, k = 0;
    for (int ee = MAXE - 1; ee >= 0 && e < 0; ee--)
        for (int ff = 0; ff < ee; ff++, k++)
            if (k == p) { e = ee; f = ff; break; }
    if (e < 0) return;
    const F fe = tb.f10[e], iff = tb.if10[f], ff_ = tb.f10[f], ie = tb.if10[e];
    int first_ok = -1;
    uint32_t n_exc = 0;
    for (uint32_t i = 0; i < ns; i++) {
        const I x = alp_enc<F>(sample[i], fe, iff);
        const bool exc = alp_dec<F>(x, ff_, ie) != sample[i];
        n_exc += exc;
        if (!exc && first_ok < 0) first_ok = int(i);
    }
    const I fill = first_ok >= 0 ? alp_enc<F>(sample[first_ok], fe, iff) : I(0);
    I mn = 0, mx = 0;
    for (uint32_t i = 0; i < ns; i++) {
        I x = alp_enc<F>(sample[i], fe, iff);
        if (first_ok >= 0 && alp_dec<F>(x, ff_, ie) != sample[i]) x = fill;
        if (i == 0 || x < mn) mn = x;
        if (i == 0 || x > mx) mx = x;
    }
    unsigned bits;
    I range;
    if (ns == 0 || __builtin_sub_overflow(mx, mn, &range)) {
        bits = 8 * sizeof(I);
    } else {
        const uint64_t r = uint64_t(range);
        bits = r == 0 ? 0 : unsigned(64 - __clzll(r));
    }
    sizes[p] = (uint64_t(ns) * bits + 7) / 8 + uint64_t(n_exc) * (sizeof(F) + sizeof(uint16_t));
}

template <typename F>
__global__ __launch_bounds__(kEB) void alp_encode_kernel(const F* __restrict__ v, uint64_t n, F fe, F iff, F ff_,
                                                         F ie, typename AlpT<F>::I* __restrict__ enc,
                                                         unsigned long long* __restrict__ first_ok) {
    unsigned long long mine = ~0ull;
    const uint64_t stride = uint64_t(gridDim.x) * kEB;
    for (uint64_t i = uint64_t(blockIdx.x) * kEB + threadIdx.x; i < n; i += stride) {
        const typename AlpT<F>::I x = alp_enc<F>(v[i], fe, iff);
        enc[i] = x;
        if (alp_dec<F>(x, ff_, ie) == v[i] && i < mine) mine = i;
    }
    for (int d = 32; d > 0; d >>= 1) {
        const unsigned long long o = __shfl_xor(mine, d, 64);
        mine = o < mine ? o : mine;
    }
    if ((threadIdx.x & 63) == 0 && mine != ~0ull) atomicMin(first_ok, mine);
}

template <typename F>
struct AlpExc {
    const F* v;
    const typename AlpT<F>::I* enc;
    F ff_, ie;
    __device__ bool operator()(uint64_t i) const { return alp_dec<F>(enc[i], ff_, ie) != v[i]; }
};
template <typename F>
struct EmitIdxVal {
    const F* v;
    uint64_t* idx;
    F* out;
    __device__ void operator()(uint64_t i, uint64_t pos) const {
        idx[pos] = i;
        out[pos] = v[i];
    }
};
// the reference's fill-forward (alp/mod.rs:223-245): once a non-exception exists, every
// exception's encoded slot takes the first non-exception's encoded value
template <typename F>
__global__ __launch_bounds__(kEB) void alp_fill_kernel(AlpExc<F> exc, typename AlpT<F>::I* __restrict__ enc, uint64_t n,
                                                       const unsigned long long* __restrict__ first_ok) {
    const unsigned long long fo = *first_ok;
    if (fo == ~0ull) return;
    const typename AlpT<F>::I fill = enc[fo];
    const uint64_t stride = uint64_t(gridDim.x) * kEB;
    for (uint64_t i = uint64_t(blockIdx.x) * kEB + threadIdx.x; i < n; i += stride)
        if (exc(i)) enc[i] = fill;
}

}  // namespace

// ------------------------------------------------------------------ launchers
namespace {
struct Temps {
    hipStream_t s;
    std::vector<void*> ps;
    explicit Temps(hipStream_t st) : s(st) {}
    ~Temps() {
        for (void* p : ps) (void)hipFreeAsync(p, s);
    }
    vxg_status get(uint64_t bytes, void** p) {
        const vxg_status st = hip_check(hipMallocAsync(p, bytes ? bytes : 16, s), "hipMallocAsync (encoder)");
        if (st == VXG_OK) ps.push_back(*p);
        return st;
    }
};

template <class Pred, class Emit>
vxg_status compact(Pred pred, Emit emit, uint64_t n, uint64_t cap, uint64_t* count, Temps& tm, hipStream_t s) {
    const uint64_t tiles = (n + kCTile - 1) / kCTile;
    *count = 0;
    if (tiles == 0) return VXG_OK;
    if (tiles > 0x7FFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "array too long");
    void *cnt, *offs;
    VXG_TRY_E(tm.get(tiles * 4, &cnt));
    VXG_TRY_E(tm.get((tiles + 1) * 8, &offs));
    hipLaunchKernelGGL(compact_count<Pred>, dim3(unsigned(tiles)), dim3(kEB), 0, s, pred, n, static_cast<uint32_t*>(cnt));
    hipLaunchKernelGGL(compact_scan, dim3(1), dim3(kEB), 0, s, static_cast<const uint32_t*>(cnt), tiles,
                       static_cast<unsigned long long*>(offs));
    hipLaunchKernelGGL((compact_scatter<Pred, Emit>), dim3(unsigned(tiles)), dim3(kEB), 0, s, pred, emit, n,
                       static_cast<const unsigned long long*>(offs), cap);
    VXG_TRY_E(hip_check(hipGetLastError(), "compaction kernels"));
    VXG_TRY_E(hip_check(hipMemcpyAsync(count, static_cast<uint64_t*>(offs) + tiles, 8, hipMemcpyDeviceToHost, s),
                        "compaction count"));
    return hip_check(hipStreamSynchronize(s), "compaction sync");
}
}  // namespace

vxg_status launch_int_stats(int width, bool sgn, const void* v, uint64_t n, IntStats* out, hipStream_t s) {
    Temps tm(s);
    void* d;
    VXG_TRY_E(tm.get(sizeof(StatsDev), &d));
    StatsDev init{};
    init.min_key = ~0ull;
    VXG_TRY_E(hip_check(hipMemcpyAsync(d, &init, sizeof(init), hipMemcpyHostToDevice, s), "stats init"));
    StatsDev* sd = static_cast<StatsDev*>(d);
    const unsigned g = egrid(n);
#define VXG_STATS(E, SG) hipLaunchKernelGGL((int_stats_kernel<E, SG>), dim3(g), dim3(kEB), 0, s, static_cast<const E*>(v), n, sd)
    switch (width * (sgn ? -1 : 1)) {
    case 1: VXG_STATS(uint8_t, false); break;
    case 2: VXG_STATS(uint16_t, false); break;
    case 4: VXG_STATS(uint32_t, false); break;
    case 8: VXG_STATS(uint64_t, false); break;
    case -1: VXG_STATS(uint8_t, true); break;
    case -2: VXG_STATS(uint16_t, true); break;
    case -4: VXG_STATS(uint32_t, true); break;
    case -8: VXG_STATS(uint64_t, true); break;
    default: return set_error(VXG_ERR_INVALID_ARGUMENT, "stats: bad width");
    }
#undef VXG_STATS
    VXG_TRY_E(hip_check(hipGetLastError(), "int_stats_kernel"));
    StatsDev h;
    VXG_TRY_E(hip_check(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, s), "stats readback"));
    VXG_TRY_E(hip_check(hipStreamSynchronize(s), "stats sync"));
    const int T = 8 * width;
    const uint64_t sb = sgn ? (1ull << (T - 1)) : 0;
    out->n = n;
    out->min_bits = n ? (h.min_key ^ sb) : 0;
    out->max_bits = n ? (h.max_key ^ sb) : 0;
    out->trailing_zeros = h.or_bits ? unsigned(__builtin_ctzll(h.or_bits)) : unsigned(T);
    if (out->trailing_zeros > unsigned(T)) out->trailing_zeros = unsigned(T);
    for (int i = 0; i < 65; i++) out->bit_width_freq[i] = i <= T ? h.freq[i] : 0;
    return VXG_OK;
}

vxg_status launch_for_encode(int width, bool sgn, const void* v, uint64_t n, uint64_t ref, unsigned shift, void* out,
                             hipStream_t s) {
    const unsigned g = egrid(n);
#define VXG_FE(E, SG) hipLaunchKernelGGL((for_encode_kernel<E, SG>), dim3(g), dim3(kEB), 0, s, static_cast<const E*>(v), n, \
                                         E(ref), shift, static_cast<E*>(out))
    switch (width * (sgn ? -1 : 1)) {
    case 1: VXG_FE(uint8_t, false); break;
    case 2: VXG_FE(uint16_t, false); break;
    case 4: VXG_FE(uint32_t, false); break;
    case 8: VXG_FE(uint64_t, false); break;
    case -1: VXG_FE(uint8_t, true); break;
    case -2: VXG_FE(uint16_t, true); break;
    case -4: VXG_FE(uint32_t, true); break;
    case -8: VXG_FE(uint64_t, true); break;
    default: return set_error(VXG_ERR_INVALID_ARGUMENT, "for_encode: bad width");
    }
#undef VXG_FE
    return hip_check(hipGetLastError(), "for_encode_kernel");
}

vxg_status launch_gather_patches_gpu(int width, unsigned W, const void* v, uint64_t n, uint64_t* idx, void* vals,
                                     uint64_t cap, uint64_t* count, hipStream_t s) {
    Temps tm(s);
    switch (width) {
#define VXG_GP(E)                                                                                          \
    return compact(WiderThan<E>{static_cast<const E*>(v), W},                                               \
                   EmitPatch<E>{static_cast<const E*>(v), idx, static_cast<E*>(vals)}, n, cap, count, tm, s);
    case 1: VXG_GP(uint8_t)
    case 2: VXG_GP(uint16_t)
    case 4: VXG_GP(uint32_t)
    case 8: VXG_GP(uint64_t)
#undef VXG_GP
    default: return set_error(VXG_ERR_INVALID_ARGUMENT, "gather_patches: bad width");
    }
}

template <typename F>
static vxg_status alp_encode_t(const F* v, uint64_t n, const F* f10, const F* if10, uint8_t* e_out, uint8_t* f_out,
                               typename AlpT<F>::I* enc, uint64_t* idx, F* vals, uint64_t cap, uint64_t* count,
                               hipStream_t s) {
    constexpr int MAXE = AlpT<F>::MAXE;
    Temps tm(s);
    // the reference's sample: values.iter().step_by(len / SAMPLE_SIZE) when len > 32 (alp/mod.rs:55-62)
    const uint64_t step = n > 32 ? n / 32 : 1;
    const uint32_t ns = uint32_t(n > 32 ? (n + step - 1) / step : n);
    void *samp, *sizes, *fo;
    VXG_TRY_E(tm.get(uint64_t(ns) * sizeof(F), &samp));
    VXG_TRY_E(tm.get(256 * 8, &sizes));
    VXG_TRY_E(tm.get(8, &fo));
    if (ns) {
        VXG_TRY_E(hip_check(hipMemcpy2DAsync(samp, sizeof(F), v, step * sizeof(F), sizeof(F), ns,
                                             hipMemcpyDeviceToDevice, s), "alp sample"));
    }
    AlpTables<F> tb{};
    for (int i = 0; i < 24 && i < MAXE + 6; i++) {
        tb.f10[i] = f10[i];
        tb.if10[i] = if10[i];
    }
    hipLaunchKernelGGL(alp_search_kernel<F>, dim3(1), dim3(kEB), 0, s, static_cast<const F*>(samp), ns, tb,
                       static_cast<unsigned long long*>(sizes));
    VXG_TRY_E(hip_check(hipGetLastError(), "alp_search_kernel"));
    unsigned long long hs[256];
    VXG_TRY_E(hip_check(hipMemcpyAsync(hs, sizes, sizeof(hs), hipMemcpyDeviceToHost, s), "alp sizes"));
    VXG_TRY_E(hip_check(hipStreamSynchronize(s), "alp search sync"));
    int be = 0, bf = 0, k = 0;
    unsigned long long best = ~0ull;
    for (int e = MAXE - 1; e >= 0; e--)
        for (int f = 0; f < e; f++, k++) {
            if (hs[k] < best) { best = hs[k]; be = e; bf = f; }
            else if (hs[k] == best && e - f < be - bf) { be = e; bf = f; }
        }
    *e_out = uint8_t(be);
    *f_out = uint8_t(bf);
    const unsigned long long none = ~0ull;
    VXG_TRY_E(hip_check(hipMemcpyAsync(fo, &none, 8, hipMemcpyHostToDevice, s), "alp first_ok init"));
    const F fe = f10[be], iff = if10[bf], ff_ = f10[bf], ie = if10[be];
    hipLaunchKernelGGL(alp_encode_kernel<F>, dim3(egrid(n)), dim3(kEB), 0, s, v, n, fe, iff, ff_, ie, enc,
                       static_cast<unsigned long long*>(fo));
    VXG_TRY_E(hip_check(hipGetLastError(), "alp_encode_kernel"));
    const AlpExc<F> exc{v, enc, ff_, ie};
    VXG_TRY_E(compact(exc, EmitIdxVal<F>{v, idx, vals}, n, cap, count, tm, s));
    hipLaunchKernelGGL(alp_fill_kernel<F>, dim3(egrid(n)), dim3(kEB), 0, s, exc, enc, n,
                       static_cast<const unsigned long long*>(fo));
    VXG_TRY_E(hip_check(hipGetLastError(), "alp_fill_kernel"));
    return hip_check(hipStreamSynchronize(s), "alp encode sync");
}

vxg_status launch_alp_encode(int float_ptype, const void* v, uint64_t n, uint8_t* e, uint8_t* f, void* enc,
                             uint64_t* idx, void* vals, uint64_t cap, uint64_t* count, hipStream_t s) {
    if (float_ptype == VXG_F64)
        return alp_encode_t<double>(static_cast<const double*>(v), n, kF10d, kIF10d, e, f, static_cast<int64_t*>(enc), idx,
                                    static_cast<double*>(vals), cap, count, s);
    if (float_ptype == VXG_F32)
        return alp_encode_t<float>(static_cast<const float*>(v), n, kF10f, kIF10f, e, f, static_cast<int32_t*>(enc), idx,
                                   static_cast<float*>(vals), cap, count, s);
    return set_error(VXG_ERR_INVALID_ARGUMENT, "ALP encodes f32 and f64");
}

}  // namespace vxg
