// fsst_encode.hip — K17: FSST compress on the GPU.
//
// The reference compresses every string of a VarBin/VarBinView with a trained symbol table
// (encodings/fsst/src/compress.rs:83-129 fsst_compress_iter: codes pushed into a
// VarBinBuilder<i32>, nulls pushed as empty values with uncompressed length 0; the table from
// Compressor::train, which stays on the host here as in the reference).  The per-string
// compression over the table is the data-parallel part; it runs here with the code format of
// fsst-rs 0.4.3 (code < 255 = symbol, 255 = escape + literal byte) and the
// exact greedy choice of this engine's host compressor (csrc/encode.cpp vxe_fsst_compress:
// at each position the longest symbol of the candidates sharing the next two bytes, in
// (length desc, code asc) order, then the one-byte symbol, else an escape) -- so the GPU's
// codes, offsets and lengths are byte-equal to the host encoder's.
//
// Decomposition (MI355X-first):
//   * the symbol table is turned on the host into a 512-slot open-addressing hash over the
//     2-byte prefixes of the multi-byte symbols (each slot: a run of candidates sorted by
//     length), plus a 256-entry one-byte table: 6 KiB, staged into LDS by every workgroup;
//   * pass A (fsst_enc_len): a workgroup per tile of 1024 strings, 4 consecutive strings per
//     thread; each string is walked with an 8-byte window (two aligned 8-byte loads, funnel
//     shifted: every candidate test is one XOR + mask) and only its code length is kept;
//     per-string lengths and one total per tile;
//   * one workgroup scans the tile totals (u64);
//   * pass B (fsst_enc_write): the tile's lengths are scanned in the workgroup (wave prefix +
//     wave totals), the i32 code offsets and uncompressed lengths are written, and every string
//     is compressed again straight into its place in the code heap (the output is contiguous
//     in string order, so neighbouring threads write neighbouring bytes).
#include <algorithm>
#include <cstring>
#include <vector>

#include "encode_gpu.hpp"
#include "vxg_internal.hpp"

#define VXG_TRY_F(expr)              \
    do {                             \
        vxg_status _s = (expr);      \
        if (_s != VXG_OK) return _s; \
    } while (0)

namespace vxg {

namespace {

constexpr int kFB = 256;          // threads per workgroup
constexpr int kFPer = 4;          // consecutive strings per thread
constexpr int kFTile = kFB * kFPer;
constexpr int kSlots = 512;       // hash slots (>= 2x the <= 255 prefixes)

struct EncTab {
    uint64_t cand_sym[256];   // multi-byte symbols grouped by prefix, (len desc, code asc) in a group
    uint8_t cand_len[256];
    uint8_t cand_code[256];
    int16_t single[256];      // code of the one-byte symbol for a byte, -1 = none
    uint32_t slot_key[kSlots];  // 0 = empty, else 0x10000 | prefix
    uint16_t slot_val[kSlots];  // first candidate | count << 8
};

__host__ __device__ inline uint32_t prefix_slot(uint32_t prefix) { return (prefix * 2654435761u) >> 23; }

struct StrSrc {
    const void* offs;
    int offs_width;
    bool offs_signed;
    const uint8_t* bytes;
    uint64_t bytes_len;
    const uint8_t* validity;  // LSB bitmap or null
    uint64_t n;
    uint32_t* bad;            // set when offsets are not a <= b <= bytes_len
};

__device__ __forceinline__ int64_t load_off(const StrSrc& s, uint64_t i) {
    switch (s.offs_width) {
    case 1: return s.offs_signed ? int64_t(static_cast<const int8_t*>(s.offs)[i]) : int64_t(static_cast<const uint8_t*>(s.offs)[i]);
    case 2: return s.offs_signed ? int64_t(static_cast<const int16_t*>(s.offs)[i]) : int64_t(static_cast<const uint16_t*>(s.offs)[i]);
    case 4: return s.offs_signed ? int64_t(static_cast<const int32_t*>(s.offs)[i]) : int64_t(static_cast<const uint32_t*>(s.offs)[i]);
    default: return static_cast<const int64_t*>(s.offs)[i];
    }
}

// Bytes [p, p + 8) of the heap as a little-endian u64 (bytes at or past `end` are garbage; the
// caller masks by the string's remaining length).  Two aligned loads: the word holding p always
// holds a valid byte, the next one is read only when it starts before `end`, so no load touches
// an address outside the pages the heap occupies.
__device__ __forceinline__ uint64_t window8(const uint8_t* p, const uint8_t* end) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p) & ~uintptr_t(7);
    const uint32_t r = uint32_t(reinterpret_cast<uintptr_t>(p) & 7);
    const uint64_t lo = *reinterpret_cast<const uint64_t*>(a);
    if (r == 0) return lo;
    const uint64_t hi = (a + 8 < reinterpret_cast<uintptr_t>(end)) ? *reinterpret_cast<const uint64_t*>(a + 8) : 0ull;
    return (lo >> (8 * r)) | (hi << (64 - 8 * r));
}

// Compress one string; WRITE: emit the codes at `out`.  Returns the code length.
template <bool WRITE>
__device__ __forceinline__ uint32_t compress_one(const uint8_t* s, uint32_t L, const uint8_t* end, const EncTab& t,
                                                 uint8_t* __restrict__ out) {
    uint32_t i = 0, o = 0;
    while (i < L) {
        const uint64_t w = window8(s + i, end);
        const uint32_t rem = L - i;
        int code = -1;
        uint32_t clen = 1;
        if (rem >= 2) {
            const uint32_t prefix = uint32_t(w & 0xFFFFu);
            uint32_t slot = prefix_slot(prefix);
            for (;;) {
                const uint32_t key = t.slot_key[slot];
                if (key == 0) break;
                if (key == (0x10000u | prefix)) {
                    const uint32_t v = t.slot_val[slot], k0 = v & 0xFFu, k1 = k0 + (v >> 8);
                    for (uint32_t k = k0; k < k1; k++) {
                        const uint32_t sl = t.cand_len[k];
                        const uint64_t m = sl >= 8 ? ~0ull : ((1ull << (8 * sl)) - 1ull);
                        if (sl <= rem && ((w ^ t.cand_sym[k]) & m) == 0) {
                            code = t.cand_code[k];
                            clen = sl;
                            break;
                        }
                    }
                    break;
                }
                slot = (slot + 1) & (kSlots - 1);
            }
        }
        if (code < 0) code = t.single[w & 0xFFu];
        if (code < 0) {  // escape + literal
            if constexpr (WRITE) {
                out[o] = 255;
                out[o + 1] = uint8_t(w & 0xFFu);
            }
            o += 2;
            i += 1;
        } else {
            if constexpr (WRITE) out[o] = uint8_t(code);
            o += 1;
            i += clen;
        }
    }
    return o;
}

__device__ __forceinline__ void stage_tab(EncTab& s, const EncTab* g) {
    const uint32_t n4 = sizeof(EncTab) / 4;
    for (uint32_t q = threadIdx.x; q < n4; q += kFB) reinterpret_cast<uint32_t*>(&s)[q] = reinterpret_cast<const uint32_t*>(g)[q];
    __syncthreads();
}

__device__ __forceinline__ bool is_valid(const StrSrc& src, uint64_t i) {
    return !src.validity || ((src.validity[i >> 3] >> (i & 7)) & 1);
}

// pass A: per-string code lengths (u32) and one total per 1024-string tile (u64: a tile of
// all-escape strings can hold more than 4 GiB of codes, which must be rejected, not wrapped)
__global__ __launch_bounds__(kFB) void fsst_enc_len(StrSrc src, const EncTab* __restrict__ gtab,
                                                    uint32_t* __restrict__ clen,
                                                    unsigned long long* __restrict__ tile_tot) {
    __shared__ EncTab t;
    __shared__ unsigned long long s_w[kFB / 64];
    stage_tab(t, gtab);
    const uint64_t first = uint64_t(blockIdx.x) * kFTile + uint64_t(threadIdx.x) * kFPer;
    const uint8_t* end = src.bytes + src.bytes_len;
    unsigned long long sum = 0;
    for (int k = 0; k < kFPer; k++) {
        const uint64_t i = first + k;
        if (i >= src.n) break;
        uint32_t c = 0;
        if (is_valid(src, i)) {
            const int64_t a = load_off(src, i), b = load_off(src, i + 1);
            if (a < 0 || b < a || uint64_t(b) > src.bytes_len || b - a > INT32_MAX)
                __hip_atomic_fetch_or(src.bad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                c = compress_one<false>(src.bytes + a, uint32_t(b - a), end, t, nullptr);
        }
        clen[i] = c;
        sum += c;
    }
    for (int d = 32; d > 0; d >>= 1) sum += __shfl_xor(sum, d, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) tile_tot[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// exclusive scan of the tile totals into tile_off (u64), total at tile_off[m]; one workgroup
__global__ __launch_bounds__(kFB) void fsst_enc_scan(const unsigned long long* __restrict__ tot, uint64_t m,
                                                     unsigned long long* __restrict__ tile_off) {
    __shared__ unsigned long long s_ws[kFB / 64];
    __shared__ unsigned long long s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t base = 0; base < m; base += kFB) {
        const uint64_t i = base + threadIdx.x;
        const unsigned long long v = i < m ? tot[i] : 0ull;
        unsigned long long x = v;
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) s_ws[wave] = x;
        __syncthreads();
        unsigned long long before = s_carry, all = 0;
        for (int w = 0; w < kFB / 64; w++) {
            before += w < wave ? s_ws[w] : 0ull;
            all += s_ws[w];
        }
        if (i < m) tile_off[i] = before + x - v;
        __syncthreads();
        if (threadIdx.x == 0) s_carry += all;
        __syncthreads();
    }
    if (threadIdx.x == 0) tile_off[m] = s_carry;
}

// pass B: i32 code offsets + uncompressed lengths, and the codes themselves
__global__ __launch_bounds__(kFB) void fsst_enc_write(StrSrc src, const EncTab* __restrict__ gtab,
                                                      const uint32_t* __restrict__ clen,
                                                      const unsigned long long* __restrict__ tile_off,
                                                      uint8_t* __restrict__ codes, int32_t* __restrict__ code_offs,
                                                      int32_t* __restrict__ ulens) {
    __shared__ EncTab t;
    __shared__ unsigned long long s_w[kFB / 64];
    stage_tab(t, gtab);
    const uint64_t first = uint64_t(blockIdx.x) * kFTile + uint64_t(threadIdx.x) * kFPer;
    uint32_t c[kFPer];
    unsigned long long mine = 0;
    for (int k = 0; k < kFPer; k++) {
        c[k] = first + k < src.n ? clen[first + k] : 0u;
        mine += c[k];
    }
    // workgroup exclusive prefix of the per-thread sums
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long x = mine;
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    uint64_t o = tile_off[blockIdx.x] + (x - mine);
    for (int w = 0; w < wave; w++) o += s_w[w];
    const uint8_t* end = src.bytes + src.bytes_len;
    for (int k = 0; k < kFPer; k++) {
        const uint64_t i = first + k;
        if (i >= src.n) break;
        code_offs[i] = int32_t(o);
        int32_t ul = 0;
        if (is_valid(src, i)) {
            const int64_t a = load_off(src, i), b = load_off(src, i + 1);
            ul = int32_t(b - a);
            if (c[k]) compress_one<true>(src.bytes + a, uint32_t(b - a), end, t, codes + o);
        }
        ulens[i] = ul;
        o += c[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kFB - 1) code_offs[src.n] = int32_t(tile_off[gridDim.x]);
}

}  // namespace

// Host: the candidate hash of a trained table (the grouping of encode.cpp vxe_fsst_compress).
static vxg_status build_tab(const uint64_t* symbols, const uint8_t* lens, uint32_t n_symbols, EncTab& t) {
    if (n_symbols > 255) return set_error(VXG_ERR_INVALID_ARGUMENT, "FSST symbol table holds at most 255 symbols");
    std::memset(&t, 0, sizeof(t));
    std::fill(t.single, t.single + 256, int16_t(-1));
    std::vector<std::vector<uint32_t>> groups;
    std::vector<uint32_t> prefixes;
    for (uint32_t s = 0; s < n_symbols; s++) {
        if (lens[s] < 1 || lens[s] > 8) return set_error(VXG_ERR_INVALID_ARGUMENT, "FSST symbol length must be 1..8");
        if (lens[s] == 1) {
            if (t.single[symbols[s] & 0xFF] < 0) t.single[symbols[s] & 0xFF] = int16_t(s);
            continue;
        }
        const uint32_t p = uint32_t(symbols[s] & 0xFFFF);
        size_t g = std::find(prefixes.begin(), prefixes.end(), p) - prefixes.begin();
        if (g == prefixes.size()) {
            prefixes.push_back(p);
            groups.emplace_back();
        }
        groups[g].push_back(s);
    }
    uint32_t k = 0;
    for (size_t g = 0; g < groups.size(); g++) {
        auto& v = groups[g];
        std::stable_sort(v.begin(), v.end(), [&](uint32_t a, uint32_t b) { return lens[a] > lens[b]; });
        uint32_t slot = prefix_slot(prefixes[g]);
        while (t.slot_key[slot]) slot = (slot + 1) & (kSlots - 1);
        t.slot_key[slot] = 0x10000u | prefixes[g];
        t.slot_val[slot] = uint16_t(k | (uint32_t(v.size()) << 8));
        for (uint32_t s : v) {
            t.cand_sym[k] = symbols[s];
            t.cand_len[k] = lens[s];
            t.cand_code[k] = uint8_t(s);
            k++;
        }
    }
    return VXG_OK;
}

vxg_status launch_fsst_compress(const uint64_t* symbols, const uint8_t* sym_lens, uint32_t n_symbols, int offs_width,
                                bool offs_signed, const void* offsets, const uint8_t* bytes, uint64_t bytes_len,
                                const uint8_t* validity, uint64_t n, uint8_t* codes, uint64_t codes_cap,
                                int32_t* code_offsets, int32_t* ulens, uint64_t* codes_len, hipStream_t s) {
    EncTab host;
    VXG_TRY_F(build_tab(symbols, sym_lens, n_symbols, host));
    *codes_len = 0;
    if (offs_width != 1 && offs_width != 2 && offs_width != 4 && offs_width != 8)
        return set_error(VXG_ERR_INVALID_ARGUMENT, "VarBin offsets must be integers");
    const uint64_t tiles = (n + kFTile - 1) / kFTile;
    // scratch: table | per-string lengths | tile totals | tile offsets
    const uint64_t o_len = (sizeof(EncTab) + 255) & ~255ull;
    const uint64_t o_tot = o_len + ((n * 4 + 255) & ~255ull);
    const uint64_t o_off = o_tot + ((tiles * 8 + 255) & ~255ull);
    const uint64_t o_bad = o_off + (tiles + 1) * 8;
    const uint64_t scratch_bytes = o_bad + 8;
    void* scratch = nullptr;
    VXG_TRY_F(hip_check(hipMallocAsync(&scratch, scratch_bytes, s), "hipMallocAsync (fsst encode)"));
    uint8_t* sc = static_cast<uint8_t*>(scratch);
    auto done = [&](vxg_status st) {
        (void)hipFreeAsync(scratch, s);
        return st;
    };
    vxg_status st = hip_check(hipMemcpyAsync(sc, &host, sizeof(EncTab), hipMemcpyHostToDevice, s), "fsst table upload");
    if (st != VXG_OK) return done(st);
    uint32_t* bad = reinterpret_cast<uint32_t*>(sc + o_bad);
    st = hip_check(hipMemsetAsync(bad, 0, 4, s), "fsst encode flag");
    if (st != VXG_OK) return done(st);
    StrSrc src{offsets, offs_width, offs_signed, bytes, bytes_len, validity, n, bad};
    const EncTab* dt = reinterpret_cast<const EncTab*>(sc);
    uint32_t* clen = reinterpret_cast<uint32_t*>(sc + o_len);
    auto* tot = reinterpret_cast<unsigned long long*>(sc + o_tot);
    auto* toff = reinterpret_cast<unsigned long long*>(sc + o_off);
    if (tiles) hipLaunchKernelGGL(fsst_enc_len, dim3(unsigned(tiles)), dim3(kFB), 0, s, src, dt, clen, tot);
    hipLaunchKernelGGL(fsst_enc_scan, dim3(1), dim3(kFB), 0, s, tot, tiles, toff);
    st = hip_check(hipGetLastError(), "fsst_enc_len / scan");
    if (st != VXG_OK) return done(st);
    uint64_t total = 0;
    uint32_t hbad = 0;
    st = hip_check(hipMemcpyAsync(&total, toff + tiles, 8, hipMemcpyDeviceToHost, s), "fsst code total");
    if (st == VXG_OK) st = hip_check(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s), "fsst encode flag");
    if (st == VXG_OK) st = hip_check(hipStreamSynchronize(s), "fsst encode sync");
    if (st != VXG_OK) return done(st);
    if (hbad) return done(set_error(VXG_ERR_INVALID_ARGUMENT, "VarBin offsets out of range of the bytes"));
    if (total > uint64_t(INT32_MAX))
        return done(set_error(VXG_ERR_INVALID_ARGUMENT, "FSST codes exceed the i32 offsets of VarBinBuilder<i32>"));
    if (total > codes_cap)
        return done(set_error(VXG_ERR_INVALID_ARGUMENT, "codes buffer too small: need " + std::to_string(total) + " bytes"));
    if (tiles) {
        hipLaunchKernelGGL(fsst_enc_write, dim3(unsigned(tiles)), dim3(kFB), 0, s, src, dt, clen, toff, codes,
                           code_offsets, ulens);
    } else {
        const int32_t zero = 0;
        st = hip_check(hipMemcpyAsync(code_offsets, &zero, 4, hipMemcpyHostToDevice, s), "fsst empty offsets");
        if (st != VXG_OK) return done(st);
    }
    st = hip_check(hipGetLastError(), "fsst_enc_write");
    if (st == VXG_OK) st = hip_check(hipStreamSynchronize(s), "fsst encode sync");
    *codes_len = total;
    return done(st);
}

}  // namespace vxg
