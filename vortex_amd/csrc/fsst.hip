// fsst.hip — K6/K7: FSST -> canonical VarBinView on gfx950.
//
// Reference: encodings/fsst/src/canonical.rs:7-57 (bulk Decompressor::decompress of the whole
// code heap, i32 prefix sum of uncompressed_lengths, VarBin -> VarBinView via arrow-cast 53.2),
// fsst-rs 0.4.3 decode semantics, view layout (Appendix C).
//
// Design: per-string code slices never straddle an escape, so the bulk decode equals the
// concatenation of per-string decodes placed at the exclusive prefix sum of the lengths.
//   kernel 1 (tile_sums):   one 256-string tile per workgroup -> sum of lengths
//   kernel 2 (scan_tiles):  single workgroup exclusive scan of the tile sums (chunked loop)
//   kernel 3 (decode):      per tile: (a) block-scan lengths -> output offsets, (b) stage the
//                           tile's contiguous code bytes into LDS with coalesced loads,
//                           (c) thread-per-string decode from LDS into an LDS heap image using
//                           the symbol table held in LDS, (d) coalesced copy of the heap image
//                           to HBM, (e) 16-byte views written coalesced (inline <= 12 bytes).
//   Tiles whose codes or output do not fit the LDS images take a direct-to-HBM path.
#include "vxg_internal.hpp"

namespace vxg {

namespace {

constexpr int kTile = 256;            // strings per tile = threads per workgroup
constexpr int kCodeLds = 16 * 1024;   // staged code bytes per tile
constexpr int kHeapLds = 32 * 1024;   // staged output bytes per tile

__device__ __forceinline__ int64_t load_int(const void* p, int width, bool sgn, uint64_t i) {
    switch (width) {
    case 1: return sgn ? int64_t(static_cast<const int8_t*>(p)[i]) : int64_t(static_cast<const uint8_t*>(p)[i]);
    case 2: return sgn ? int64_t(static_cast<const int16_t*>(p)[i]) : int64_t(static_cast<const uint16_t*>(p)[i]);
    case 4: return sgn ? int64_t(static_cast<const int32_t*>(p)[i]) : int64_t(static_cast<const uint32_t*>(p)[i]);
    default: return static_cast<const int64_t*>(p)[i];
    }
}

// Block-wide exclusive scan of one int64 per thread (256 threads = 4 waves).
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
    int64_t before = 0;
    for (int w = 0; w < wave; w++) before += wave_sums[w];
    total = wave_sums[0] + wave_sums[1] + wave_sums[2] + wave_sums[3];
    __syncthreads();
    return before + x - v;
}

}  // namespace

__global__ __launch_bounds__(kTile) void fsst_tile_sums(const void* lens, int lens_width, int lens_signed,
                                                        uint64_t n, int64_t* __restrict__ tile_sums) {
    __shared__ int64_t ws[4];
    const uint64_t i = uint64_t(blockIdx.x) * kTile + threadIdx.x;
    const int64_t v = i < n ? load_int(lens, lens_width, lens_signed != 0, i) : 0;
    int64_t tot;
    (void)block_exclusive_scan(v, ws, tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

// Exclusive scan of the tile sums by ONE 1024-thread workgroup: thread k sums a contiguous
// run of ceil(n_tiles/1024) tiles, the 1024 partials are block-scanned (16 waves), then each
// thread rewrites its run.  Two passes over n_tiles (~23 K for C4) instead of a serial
// 256-wide loop (70 us -> a few us).
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void fsst_scan_tiles(int64_t* __restrict__ tile_sums, uint64_t n_tiles) {
    __shared__ int64_t wsum[kScanThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t per = (n_tiles + kScanThreads - 1) / kScanThreads;
    const uint64_t lo = uint64_t(tid) * per;
    const uint64_t hi = lo + per < n_tiles ? lo + per : n_tiles;
    int64_t s = 0;
    for (uint64_t i = lo; i < hi; i++) s += tile_sums[i];
    int64_t x = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int64_t before = 0;
    for (int w = 0; w < wave; w++) before += wsum[w];
    int64_t run = before + x - s;  // exclusive prefix of this thread's run
    for (uint64_t i = lo; i < hi; i++) {
        const int64_t v = tile_sums[i];
        tile_sums[i] = run;
        run += v;
    }
}

__global__ __launch_bounds__(kTile) void fsst_decode(const uint64_t* __restrict__ symbols,
                                                     const uint8_t* __restrict__ sym_lens, unsigned n_symbols,
                                                     const uint8_t* __restrict__ codes, const void* code_offs,
                                                     int offs_width, const void* lens, int lens_width,
                                                     int lens_signed, uint64_t n,
                                                     const uint8_t* __restrict__ validity,
                                                     const int64_t* __restrict__ tile_prefix,
                                                     uint8_t* __restrict__ heap, uint4* __restrict__ views) {
    __shared__ uint64_t s_sym[256];
    __shared__ uint8_t s_len[256];
    __shared__ int64_t ws[4];
    __shared__ __attribute__((aligned(16))) uint8_t s_codes[kCodeLds];
    __shared__ __attribute__((aligned(16))) uint8_t s_heap[kHeapLds + 16];

    const int tid = threadIdx.x;
    for (int k = tid; k < 256; k += kTile) {
        s_sym[k] = k < int(n_symbols) ? symbols[k] : 0;
        s_len[k] = k < int(n_symbols) ? sym_lens[k] : 0;
    }
    const uint64_t i = uint64_t(blockIdx.x) * kTile + tid;
    const bool live = i < n;
    const int64_t my_len = live ? load_int(lens, lens_width, lens_signed != 0, i) : 0;
    int64_t tile_total;
    const int64_t my_rel = block_exclusive_scan(my_len, ws, tile_total);   // offset inside tile
    const int64_t tile_out0 = tile_prefix[blockIdx.x];
    const uint64_t last = (uint64_t(blockIdx.x) + 1) * kTile < n ? (uint64_t(blockIdx.x) + 1) * kTile : n;
    const uint64_t first = uint64_t(blockIdx.x) * kTile;
    // code offsets are relative to code_offs[0] (sliced_bytes(), varbin/mod.rs:130-136)
    const int64_t c_base = load_int(code_offs, offs_width, offs_width < 8, 0);
    const int64_t c0 = load_int(code_offs, offs_width, offs_width < 8, first) - c_base;
    const int64_t c1 = load_int(code_offs, offs_width, offs_width < 8, last) - c_base;
    const int64_t my_c0 = live ? load_int(code_offs, offs_width, offs_width < 8, i) - c_base : 0;
    const int64_t my_c1 = live ? load_int(code_offs, offs_width, offs_width < 8, i + 1) - c_base : 0;
    const uint8_t* gcodes = codes + c_base;
    const bool stage = (c1 - c0) <= kCodeLds && tile_total <= kHeapLds;

    if (stage) {
        for (int64_t k = tid; k < c1 - c0; k += kTile) s_codes[k] = gcodes[c0 + k];
    }
    __syncthreads();

    bool valid = live;
    if (live && validity) valid = (validity[i >> 3] >> (i & 7)) & 1;

    if (stage) {
        // decode from LDS codes into the LDS heap image
        // writes are clamped to this string's [my_rel, my_rel + my_len) so corrupt lengths
        // can never touch another string's bytes or leave the LDS image
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
        // coalesced copy-out of [tile_out0, tile_out0 + tile_total)
        uint8_t* dst = heap + tile_out0;
        const int64_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
        const int64_t h = head < tile_total ? head : tile_total;
        for (int64_t k = tid; k < h; k += kTile) dst[k] = s_heap[k];
        const int64_t body = (tile_total - h) / 16;
        for (int64_t k = tid; k < body; k += kTile) {
            uint32_t w[4];
            const uint8_t* src = s_heap + h + 16 * k;
#pragma unroll
            for (int q = 0; q < 4; q++)
                w[q] = uint32_t(src[4 * q]) | (uint32_t(src[4 * q + 1]) << 8) |
                       (uint32_t(src[4 * q + 2]) << 16) | (uint32_t(src[4 * q + 3]) << 24);
            // plain stores: these 16-B chunks do not cover whole 128-B lines per instruction,
            // and non-temporal stores made this kernel 10x slower (660 vs 66 us on C4, r01)
            reinterpret_cast<uint4*>(dst + h)[k] = make_uint4(w[0], w[1], w[2], w[3]);
        }
        for (int64_t k = h + body * 16 + tid; k < tile_total; k += kTile) dst[k] = s_heap[k];
        // views from the LDS image
        if (live) {
            uint8_t b[16];
#pragma unroll
            for (int k = 0; k < 16; k++) b[k] = 0;
            if (valid) {
                const uint32_t len = uint32_t(my_len);
                __builtin_memcpy(b, &len, 4);
                if (len <= 12) {
                    for (uint32_t k = 0; k < len; k++) b[4 + k] = s_heap[my_rel + k];
                } else {
#pragma unroll
                    for (int k = 0; k < 4; k++) b[4 + k] = s_heap[my_rel + k];
                    const uint32_t off = uint32_t(tile_out0 + my_rel);
                    __builtin_memcpy(b + 12, &off, 4);
                }
            }
            uint4 q;
            __builtin_memcpy(&q, b, 16);
            views[i] = q;
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
            uint8_t b[16];
#pragma unroll
            for (int k = 0; k < 16; k++) b[k] = 0;
            if (valid) {
                const uint32_t len = uint32_t(my_len);
                __builtin_memcpy(b, &len, 4);
                if (len <= 12) {
                    for (uint32_t k = 0; k < len; k++) b[4 + k] = heap[o_start + k];
                } else {
#pragma unroll
                    for (int k = 0; k < 4; k++) b[4 + k] = heap[o_start + k];
                    const uint32_t off = uint32_t(o_start);
                    __builtin_memcpy(b + 12, &off, 4);
                }
            }
            uint4 q;
            __builtin_memcpy(&q, b, 16);
            views[i] = q;
        }
    }
}

uint64_t fsst_scratch_bytes(uint64_t n) { return ((n + kTile - 1) / kTile + 1) * sizeof(int64_t); }

vxg_status launch_fsst(const uint64_t* symbols, const uint8_t* sym_lens, unsigned n_symbols,
                       const uint8_t* code_bytes, int offs_width, const void* code_offsets,
                       int lens_width, bool lens_signed, const void* lens, uint64_t n,
                       const uint8_t* validity, void* scratch, uint8_t* heap, uint8_t* views,
                       hipStream_t s) {
    if (n == 0) return VXG_OK;
    if (n_symbols > 255) return set_error(VXG_ERR_INVALID_ARGUMENT, "FSST symbol table > 255 entries");
    const uint64_t n_tiles = (n + kTile - 1) / kTile;
    int64_t* tiles = static_cast<int64_t*>(scratch);
    hipLaunchKernelGGL(fsst_tile_sums, dim3(unsigned(n_tiles)), dim3(kTile), 0, s, lens, lens_width,
                       int(lens_signed), n, tiles);
    hipLaunchKernelGGL(fsst_scan_tiles, dim3(1), dim3(kScanThreads), 0, s, tiles, n_tiles);
    hipLaunchKernelGGL(fsst_decode, dim3(unsigned(n_tiles)), dim3(kTile), 0, s, symbols, sym_lens,
                       n_symbols, code_bytes, code_offsets, offs_width, lens, lens_width,
                       int(lens_signed), n, validity, tiles, heap, reinterpret_cast<uint4*>(views));
    return hip_check(hipGetLastError(), "fsst kernels");
}

}  // namespace vxg
