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
constexpr int kCodeLds = 16 * 1024;   // staged code bytes per tile
constexpr int kHeapLds = 32 * 1024;   // staged output bytes per tile
constexpr int kScanBlock = 1024;      // tiles per scan_blocks workgroup

__device__ __forceinline__ int64_t load_int(const void* p, int width, bool sgn, uint64_t i) {
    switch (width) {
    case 1: return sgn ? int64_t(static_cast<const int8_t*>(p)[i]) : int64_t(static_cast<const uint8_t*>(p)[i]);
    case 2: return sgn ? int64_t(static_cast<const int16_t*>(p)[i]) : int64_t(static_cast<const uint16_t*>(p)[i]);
    case 4: return sgn ? int64_t(static_cast<const int32_t*>(p)[i]) : int64_t(static_cast<const uint32_t*>(p)[i]);
    default: return static_cast<const int64_t*>(p)[i];
    }
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

__global__ __launch_bounds__(kTile) void fsst_tile_sums(const void* lens, int lens_width, int lens_signed,
                                                        uint64_t n, int64_t* __restrict__ tile_sums) {
    __shared__ int64_t ws[kTile / 64];
    const uint64_t i = uint64_t(blockIdx.x) * kTile + threadIdx.x;
    const int64_t v = wave_sum(i < n ? load_int(lens, lens_width, lens_signed != 0, i) : 0);
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

__global__ __launch_bounds__(kTile) void fsst_decode(const uint64_t* __restrict__ symbols,
                                                     const uint8_t* __restrict__ sym_lens, unsigned n_symbols,
                                                     const uint8_t* __restrict__ codes, const void* code_offs,
                                                     int offs_width, const void* lens, int lens_width,
                                                     int lens_signed, uint64_t n,
                                                     const uint8_t* __restrict__ validity,
                                                     const int64_t* __restrict__ tile_prefix,
                                                     const int64_t* __restrict__ block_totals,
                                                     uint8_t* __restrict__ heap, uint4* __restrict__ views) {
    __shared__ uint64_t s_sym[256];
    __shared__ uint8_t s_len[256];
    __shared__ int64_t ws[kTile / 64];
    __shared__ int64_t s_block_prefix;
    __shared__ __attribute__((aligned(16))) uint8_t s_codes[kCodeLds];
    __shared__ __attribute__((aligned(16))) uint8_t s_heap[kHeapLds + 16];

    const int tid = threadIdx.x;
    for (int k = tid; k < 256; k += kTile) {
        s_sym[k] = k < int(n_symbols) ? symbols[k] : 0;
        s_len[k] = k < int(n_symbols) ? sym_lens[k] : 0;
    }
    if (tid < 64) {  // (a) prefix of the preceding 1024-tile blocks, one wave
        const uint64_t nb = blockIdx.x / kScanBlock;
        int64_t acc = 0;
        for (uint64_t b = tid; b < nb; b += 64) acc += block_totals[b];
        acc = wave_sum(acc);
        if (tid == 0) s_block_prefix = acc;
    }
    const uint64_t i = uint64_t(blockIdx.x) * kTile + tid;
    const bool live = i < n;
    const int64_t my_len = live ? load_int(lens, lens_width, lens_signed != 0, i) : 0;
    int64_t tile_total;
    const int64_t my_rel = block_exclusive_scan<kTile / 64>(my_len, ws, tile_total);  // (b)
    const int64_t tile_out0 = tile_prefix[blockIdx.x] + s_block_prefix;
    const uint64_t first = uint64_t(blockIdx.x) * kTile;
    const uint64_t last = first + kTile < n ? first + kTile : n;
    // code offsets are relative to code_offs[0] (sliced_bytes(), varbin/mod.rs:130-136)
    const int64_t c_base = load_int(code_offs, offs_width, offs_width < 8, 0);
    const int64_t c0 = load_int(code_offs, offs_width, offs_width < 8, first) - c_base;
    const int64_t c1 = load_int(code_offs, offs_width, offs_width < 8, last) - c_base;
    const int64_t my_c0 = live ? load_int(code_offs, offs_width, offs_width < 8, i) - c_base : 0;
    const int64_t my_c1 = live ? load_int(code_offs, offs_width, offs_width < 8, i + 1) - c_base : 0;
    const uint8_t* gcodes = codes + c_base;
    const bool stage = (c1 - c0) <= kCodeLds && tile_total <= kHeapLds;

    if (stage) {  // (c)
        for (int64_t k = tid; k < c1 - c0; k += kTile) s_codes[k] = gcodes[c0 + k];
    }
    __syncthreads();

    bool valid = live;
    if (live && validity) valid = (validity[i >> 3] >> (i & 7)) & 1;
    const uint32_t vlen = valid ? uint32_t(my_len) : 0u;

    if (stage) {
        // (d) writes are clamped to this string's [my_rel, my_rel + my_len), so corrupt
        // lengths can never touch another string's bytes or leave the LDS image
        int64_t o = my_rel;
        const int64_t o_end = my_rel + my_len;
        for (int64_t k = my_c0 - c0; k < my_c1 - c0; k++) {
            const uint8_t c = s_codes[k];
            if (c == 255) {
                ++k;
                if (o < o_end) s_heap[o] = s_codes[k];
                o++;
            } else {
                const uint64_t sym = s_sym[c];
                const int L = s_len[c];
                for (int b = 0; b < L; b++)
                    if (o + b < o_end) s_heap[o + b] = uint8_t(sym >> (8 * b));
                o += L;
            }
        }
        __syncthreads();
        // (e) coalesced copy-out of [tile_out0, tile_out0 + tile_total)
        uint8_t* dst = heap + tile_out0;
        const int64_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
        const int64_t h = head < tile_total ? head : tile_total;
        for (int64_t k = tid; k < h; k += kTile) dst[k] = s_heap[k];
        const int64_t body = (tile_total - h) / 16;
        for (int64_t k = tid; k < body; k += kTile) {
            const uint8_t* src = s_heap + h + 16 * k;
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; q++)
                w[q] = uint32_t(src[4 * q]) | (uint32_t(src[4 * q + 1]) << 8) |
                       (uint32_t(src[4 * q + 2]) << 16) | (uint32_t(src[4 * q + 3]) << 24);
            reinterpret_cast<uint4*>(dst + h)[k] = make_uint4(w[0], w[1], w[2], w[3]);
        }
        for (int64_t k = h + body * 16 + tid; k < tile_total; k += kTile) dst[k] = s_heap[k];
        // (f) views from the LDS image (reads past the string stay inside s_heap's slack)
        if (live) {
            const uint8_t* sp = s_heap + my_rel;
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
    hipLaunchKernelGGL(fsst_tile_sums, dim3(unsigned(n_tiles)), dim3(kTile), 0, s, lens, lens_width,
                       int(lens_signed), n, tiles);
    hipLaunchKernelGGL(fsst_scan_blocks, dim3(unsigned(n_blocks)), dim3(kScanBlock), 0, s, tiles, n_tiles, blocks);
    hipLaunchKernelGGL(fsst_decode, dim3(unsigned(n_tiles)), dim3(kTile), 0, s, symbols, sym_lens,
                       n_symbols, code_bytes, code_offsets, offs_width, lens, lens_width,
                       int(lens_signed), n, validity, tiles, blocks, heap, reinterpret_cast<uint4*>(views));
    return hip_check(hipGetLastError(), "fsst kernels");
}

}  // namespace vxg
