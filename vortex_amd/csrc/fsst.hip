// fsst.hip — K6/K7: FSST -> canonical VarBinView on gfx950.
//
// Reference: encodings/fsst/src/canonical.rs:7-57 (bulk Decompressor::decompress of the whole
// code heap, i32 prefix sum of uncompressed_lengths, VarBin -> VarBinView via arrow-cast 53.2),
// fsst-rs 0.4.3 decode semantics, view layout (Appendix C).
//
// Design: per-string code slices never straddle an escape, so the bulk decode equals the
// concatenation of per-string decodes placed at the exclusive prefix sum of the lengths.
//   kernel 1 (tile_sums):   one 256-string tile per workgroup -> sum of its lengths
//   kernel 2 (scan_blocks): 1024 tiles per workgroup -> exclusive tile prefix inside the
//                           1024-tile block + one total per block (coalesced, fully parallel)
//   kernel 3 (decode):      per tile: (a) block prefix = sum of the preceding block totals
//                           (one wave, parallel loads), (b) block-scan of lengths -> offsets,
//                           (c) stage the tile's contiguous code bytes into LDS with coalesced
//                           loads, (d) thread-per-string decode from LDS into an LDS heap image
//                           with the symbol table in LDS, (e) coalesced copy-out of the image,
//                           (f) 16-byte views (inline <= 12 bytes) built with compile-time byte
//                           positions (no runtime-indexed register arrays -> no scratch).
//   Tiles whose codes or output do not fit the LDS images take a direct-to-HBM path.
#include "vxg_internal.hpp"

namespace vxg {

namespace {

constexpr int kTile = 256;            // strings per tile = threads per workgroup
// LDS images sized for short strings (TPC-H l_comment: 10-43 bytes, a 256-string tile is
// ~6.9 KB decoded / ~3 KB of codes).  ~18.8 KB of LDS per workgroup keeps 8 workgroups
// (32 waves) resident per CU; the kernel is latency-bound on its phase chain, so residency is
// what hides it (51 KB images gave 3 workgroups/CU and 3x the time).  Larger tiles take the
// direct path.
constexpr int kCodeLds = 6 * 1024;    // staged code bytes per tile
constexpr int kHeapLds = 10 * 1024;   // staged output bytes per tile
constexpr int kScanBlock = 1024;      // tiles per scan_blocks workgroup

// Integer load with compile-time width/signedness.  (A runtime width switch compiles to a
// branch nest that waits vmcnt(0) after every load: the decode prologue's 7 independent
// loads became 7 serialized HBM round trips, 730 us vs ~100 us on C4.)
template <int WIDTH, bool SGN>
__device__ __forceinline__ int64_t ld(const void* p, uint64_t i) {
    if constexpr (WIDTH == 1) return SGN ? int64_t(static_cast<const int8_t*>(p)[i]) : int64_t(static_cast<const uint8_t*>(p)[i]);
    else if constexpr (WIDTH == 2) return SGN ? int64_t(static_cast<const int16_t*>(p)[i]) : int64_t(static_cast<const uint16_t*>(p)[i]);
    else if constexpr (WIDTH == 4) return SGN ? int64_t(static_cast<const int32_t*>(p)[i]) : int64_t(static_cast<const uint32_t*>(p)[i]);
    else return static_cast<const int64_t*>(p)[i];
}

__device__ __forceinline__ int64_t wave_sum(int64_t x) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

// Block-wide exclusive scan of one int64 per thread (NW waves).
template <int NW>
__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t* wave_sums, int64_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wave_sums[wave] = x;
    __syncthreads();
    int64_t before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const int64_t s = wave_sums[w];
        before += w < wave ? s : 0;
        tot += s;
    }
    total = tot;
    __syncthreads();
    return before + x - v;
}

// arrow-array 53.2 make_view: len <= 12 -> [len][bytes, zero padded]; else
// [len][first 4 bytes][buffer_index = 0][offset].  `get(j)` returns byte j of the string (only
// called for j < 12 inline / j < 4 prefix, and masked by j < len).
template <typename Get>
__device__ __forceinline__ uint4 build_view(uint32_t len, uint32_t offset, Get get) {
    uint32_t w1 = 0, w2 = 0, w3 = 0;
    if (len <= 12) {
#pragma unroll
        for (int j = 0; j < 12; j++) {
            const uint32_t b = uint32_t(j) < len ? uint32_t(get(j)) : 0u;
            if (j < 4) w1 |= b << (8 * j);
            else if (j < 8) w2 |= b << (8 * (j - 4));
            else w3 |= b << (8 * (j - 8));
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) w1 |= uint32_t(get(j)) << (8 * j);
        w3 = offset;
    }
    return make_uint4(len, w1, w2, w3);
}

}  // namespace

template <int LW, bool LSG>
__global__ __launch_bounds__(kTile) void fsst_tile_sums(const void* lens, uint64_t n, int64_t* __restrict__ tile_sums) {
    __shared__ int64_t ws[kTile / 64];
    const uint64_t i = uint64_t(blockIdx.x) * kTile + threadIdx.x;
    const int64_t v = wave_sum(i < n ? ld<LW, LSG>(lens, i) : 0);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(kScanBlock) void fsst_scan_blocks(int64_t* __restrict__ tile_sums, uint64_t n_tiles,
                                                               int64_t* __restrict__ block_totals) {
    __shared__ int64_t ws[kScanBlock / 64];
    const uint64_t i = uint64_t(blockIdx.x) * kScanBlock + threadIdx.x;
    const int64_t v = i < n_tiles ? tile_sums[i] : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan<kScanBlock / 64>(v, ws, tot);
    if (i < n_tiles) tile_sums[i] = ex;
    if (threadIdx.x == 0) block_totals[blockIdx.x] = tot;
}

template <int OW, int LW, bool LSG>
__global__ __launch_bounds__(kTile) void fsst_decode(const uint64_t* __restrict__ symbols,
                                                     const uint8_t* __restrict__ sym_lens, unsigned n_symbols,
                                                     const uint8_t* __restrict__ codes, const void* code_offs,
                                                     const void* lens, uint64_t n,
                                                     const uint8_t* __restrict__ validity,
                                                     const int64_t* __restrict__ tile_prefix,
                                                     const int64_t* __restrict__ block_totals,
                                                     uint8_t* __restrict__ heap, uint4* __restrict__ views) {
    __shared__ uint64_t s_sym[256];
    __shared__ uint8_t s_len[256];
    __shared__ int64_t ws[kTile / 64];
    __shared__ int64_t s_block_prefix;
    __shared__ __attribute__((aligned(16))) uint8_t s_codes[kCodeLds + 32];
    __shared__ __attribute__((aligned(16))) uint8_t s_heap[kHeapLds + 32];

    const int tid = threadIdx.x;
    // Prologue: every global load below is unconditional (indices clamped, results selected
    // afterwards) so they issue back to back and retire under ONE wait.
    constexpr bool OSG = OW < 8;  // i32 offsets (VarBinBuilder<i32>, fsst/compress.rs:94)
    const uint64_t i = uint64_t(blockIdx.x) * kTile + tid;
    const bool live = i < n;
    const uint64_t ii = live ? i : n - 1;
    const uint64_t first = uint64_t(blockIdx.x) * kTile;
    const uint64_t last = first + kTile < n ? first + kTile : n;
    const uint64_t sk = uint32_t(tid) < n_symbols ? uint32_t(tid) : 0;
    const uint64_t sym_v = symbols[sk];
    const uint8_t slen_v = sym_lens[sk];
    const int64_t len_v = ld<LW, LSG>(lens, ii);
    const int64_t c_base = ld<OW, OSG>(code_offs, 0);
    const int64_t cf = ld<OW, OSG>(code_offs, first);
    const int64_t cl = ld<OW, OSG>(code_offs, last);
    const int64_t ci0 = ld<OW, OSG>(code_offs, ii);
    const int64_t ci1 = ld<OW, OSG>(code_offs, ii + 1);
    const int64_t tp = tile_prefix[blockIdx.x];
    const uint8_t vbyte = validity ? validity[ii >> 3] : uint8_t(0xFF);
    s_sym[tid] = uint32_t(tid) < n_symbols ? sym_v : 0;  // kTile == 256 symbol slots
    s_len[tid] = uint32_t(tid) < n_symbols ? slen_v : 0;
    if (tid < 64) {  // (a) prefix of the preceding 1024-tile blocks, one wave
        const uint64_t nb = blockIdx.x / kScanBlock;
        int64_t acc = 0;
        for (uint64_t b = tid; b < nb; b += 64) acc += block_totals[b];
        acc = wave_sum(acc);
        if (tid == 0) s_block_prefix = acc;
    }
    const int64_t my_len = live ? len_v : 0;
    int64_t tile_total;
    const int64_t my_rel = block_exclusive_scan<kTile / 64>(my_len, ws, tile_total);  // (b)
    const int64_t tile_out0 = tp + s_block_prefix;
    // code offsets are relative to code_offs[0] (sliced_bytes(), varbin/mod.rs:130-136)
    const int64_t c0 = cf - c_base;
    const int64_t c1 = cl - c_base;
    const int64_t my_c0 = live ? ci0 - c_base : 0;
    const int64_t my_c1 = live ? ci1 - c_base : 0;
    const uint8_t* gcodes = codes + c_base;
    const bool stage = (c1 - c0) <= kCodeLds && tile_total <= kHeapLds;
    // LDS images are placed at the same offset mod 16 as their global counterparts, so the
    // staging loads and the copy-out stores move whole aligned 16-byte chunks.
    const int64_t cabs0 = c_base + c0, cabs1 = c_base + c1;       // tile codes in `codes`
    const int cshift = int((reinterpret_cast<uintptr_t>(codes) + cabs0) & 15);  // s_codes[cshift] = codes[cabs0]
    const int hshift = int((reinterpret_cast<uintptr_t>(heap) + tile_out0) & 15);  // s_heap[hshift] = heap[tile_out0]

    if (stage && cabs1 > cabs0) {  // (c) aligned 16-byte loads (bytes at the ragged chunks)
        const int64_t a0 = cabs0 - cshift;
        const int64_t nchunk = (cabs1 - a0 + 15) / 16;
        for (int64_t q = tid; q < nchunk; q += kTile) {
            const int64_t g = a0 + 16 * q;
            if (g >= 0 && g + 16 <= cabs1) {
                *reinterpret_cast<uint4*>(s_codes + 16 * q) = *reinterpret_cast<const uint4*>(codes + g);
            } else {
                // ragged chunk: 16 unconditional byte loads at clamped in-range addresses,
                // issued together, then selected (no per-byte round trip)
                uint8_t bv[16];
#pragma unroll
                for (int b = 0; b < 16; b++) {
                    const int64_t a = g + b < cabs0 ? cabs0 : (g + b >= cabs1 ? cabs1 - 1 : g + b);
                    bv[b] = codes[a];
                }
#pragma unroll
                for (int b = 0; b < 16; b++)
                    if (g + b < cabs1 && g + b >= cabs0) s_codes[16 * q + b] = bv[b];
            }
        }
    }
    __syncthreads();

    const bool valid = live && ((vbyte >> (ii & 7)) & 1);
    const uint32_t vlen = valid ? uint32_t(my_len) : 0u;

    if (stage) {
        // (d) writes are clamped to this string's [my_rel, my_rel + my_len), so corrupt
        // lengths can never touch another string's bytes or leave the LDS image
        const uint8_t* sc = s_codes + cshift - c0;  // sc[k] = codes byte k (k relative to c_base)
        uint8_t* sh = s_heap + hshift;              // sh[r] = heap byte tile_out0 + r
        int64_t o = my_rel;
        const int64_t o_end = my_rel + my_len;
        for (int64_t k = my_c0; k < my_c1; k++) {
            const uint8_t c = sc[k];
            if (c == 255) {
                ++k;
                if (o < o_end) sh[o] = sc[k];
                o++;
            } else {
                const uint64_t sym = s_sym[c];
                const int L = s_len[c];
                for (int b = 0; b < L; b++)
                    if (o + b < o_end) sh[o + b] = uint8_t(sym >> (8 * b));
                o += L;
            }
        }
        __syncthreads();
        // (e) copy-out of [tile_out0, tile_out0 + tile_total): whole aligned 16-byte chunks via
        // ds_read_b128 + global_store_dwordx4; the ragged first/last chunk byte by byte (they
        // are shared with the neighbouring tiles)
        const int64_t g0 = tile_out0, g1 = tile_out0 + tile_total;
        const int64_t a0 = g0 - hshift;                      // aligned chunk containing g0
        const int64_t nchunk = (g1 - a0 + 15) / 16;
        for (int64_t q = tid; q < nchunk; q += kTile) {
            const int64_t g = a0 + 16 * q;
            if (g >= g0 && g + 16 <= g1) {
                *reinterpret_cast<uint4*>(heap + g) = *reinterpret_cast<const uint4*>(s_heap + 16 * q);
            } else {
                for (int b = 0; b < 16; b++)
                    if (g + b >= g0 && g + b < g1) heap[g + b] = s_heap[16 * q + b];
            }
        }
        // (f) views from the LDS image (reads past the string stay inside s_heap's slack)
        if (live) {
            const uint8_t* sp = sh + my_rel;
            views[i] = valid ? build_view(vlen, uint32_t(tile_out0 + my_rel), [&](int j) { return sp[j]; })
                             : make_uint4(0, 0, 0, 0);
        }
    } else {
        // direct path: decode straight into HBM
        int64_t o = tile_out0 + my_rel;
        const int64_t o_start = o, o_end = o + my_len;
        for (int64_t k = my_c0; k < my_c1; k++) {
            const uint8_t c = gcodes[k];
            if (c == 255) {
                ++k;
                if (o < o_end) heap[o] = gcodes[k];
                o++;
            } else {
                const uint64_t sym = s_sym[c];
                const int L = s_len[c];
                for (int b = 0; b < L; b++)
                    if (o + b < o_end) heap[o + b] = uint8_t(sym >> (8 * b));
                o += L;
            }
        }
        if (live) {
            const uint8_t* hp = heap + o_start;
            views[i] = valid ? build_view(vlen, uint32_t(o_start),
                                          [&](int j) { return uint32_t(j) < vlen ? hp[j] : uint8_t(0); })
                             : make_uint4(0, 0, 0, 0);
        }
    }
}

uint64_t fsst_scratch_bytes(uint64_t n) {
    const uint64_t n_tiles = (n + kTile - 1) / kTile;
    return (n_tiles + (n_tiles + kScanBlock - 1) / kScanBlock + 2) * sizeof(int64_t);
}

vxg_status launch_fsst(const uint64_t* symbols, const uint8_t* sym_lens, unsigned n_symbols,
                       const uint8_t* code_bytes, int offs_width, const void* code_offsets,
                       int lens_width, bool lens_signed, const void* lens, uint64_t n,
                       const uint8_t* validity, void* scratch, uint8_t* heap, uint8_t* views,
                       hipStream_t s) {
    if (n == 0) return VXG_OK;
    if (n_symbols > 255) return set_error(VXG_ERR_INVALID_ARGUMENT, "FSST symbol table > 255 entries");
    const uint64_t n_tiles = (n + kTile - 1) / kTile;
    const uint64_t n_blocks = (n_tiles + kScanBlock - 1) / kScanBlock;
    int64_t* tiles = static_cast<int64_t*>(scratch);
    int64_t* blocks = tiles + n_tiles;
    const bool lsg = lens_signed;
    auto run = [&](auto ow_c, auto lw_c, auto lsg_c) {
        constexpr int OW = decltype(ow_c)::value, LW = decltype(lw_c)::value;
        constexpr bool LSG = decltype(lsg_c)::value;
        hipLaunchKernelGGL((fsst_tile_sums<LW, LSG>), dim3(unsigned(n_tiles)), dim3(kTile), 0, s, lens, n, tiles);
        hipLaunchKernelGGL(fsst_scan_blocks, dim3(unsigned(n_blocks)), dim3(kScanBlock), 0, s, tiles, n_tiles,
                           blocks);
        hipLaunchKernelGGL((fsst_decode<OW, LW, LSG>), dim3(unsigned(n_tiles)), dim3(kTile), 0, s, symbols, sym_lens,
                           n_symbols, code_bytes, code_offsets, lens, n, validity, tiles, blocks, heap,
                           reinterpret_cast<uint4*>(views));
    };
    using I4 = std::integral_constant<int, 4>;
    using I8 = std::integral_constant<int, 8>;
    using I2 = std::integral_constant<int, 2>;
    using I1 = std::integral_constant<int, 1>;
    using T_ = std::true_type;
    using F_ = std::false_type;
    auto with_lens = [&](auto ow_c) -> vxg_status {
        switch (lens_width) {
        case 1: lsg ? run(ow_c, I1{}, T_{}) : run(ow_c, I1{}, F_{}); break;
        case 2: lsg ? run(ow_c, I2{}, T_{}) : run(ow_c, I2{}, F_{}); break;
        case 4: lsg ? run(ow_c, I4{}, T_{}) : run(ow_c, I4{}, F_{}); break;
        case 8: run(ow_c, I8{}, T_{}); break;
        default: return set_error(VXG_ERR_MISMATCHED_TYPES, "FSST lengths must be 1/2/4/8-byte integers");
        }
        return VXG_OK;
    };
    vxg_status st;
    switch (offs_width) {
    case 1: st = with_lens(I1{}); break;
    case 2: st = with_lens(I2{}); break;
    case 4: st = with_lens(I4{}); break;
    case 8: st = with_lens(I8{}); break;
    default: return set_error(VXG_ERR_MISMATCHED_TYPES, "FSST code offsets must be 1/2/4/8-byte integers");
    }
    if (st != VXG_OK) return st;
    return hip_check(hipGetLastError(), "fsst kernels");
}

}  // namespace vxg
