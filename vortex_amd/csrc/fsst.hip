// fsst.hip — K6/K7: FSST -> canonical VarBinView on gfx950.
//
// Reference: encodings/fsst/src/canonical.rs:7-57 (bulk Decompressor::decompress of the whole
// code heap, i32 prefix sum of uncompressed_lengths, VarBin -> VarBinView via arrow-cast 53.2),
// fsst-rs 0.4.3 decode semantics, view layout (Appendix C).
//
// The reference decodes the whole code heap as ONE stream and slices string i at the prefix sum
// of the uncompressed lengths.  Every tile of 256 strings owns a contiguous code range that
// starts at a code boundary, so the decoded bytes of a tile land at [prefix(tile), prefix(tile)
// + sum of its lengths) — tiles are independent once the tile prefix is known.
//   kernel 1 (tile_sums):   sum of the lengths of each 256-string tile (16 tiles per workgroup)
//   kernel 2 (scan_blocks): exclusive tile prefix inside 1024-tile blocks + one total per block
//   kernel 3 (decode):      per tile, in LDS:
//     (a) block prefix (one wave) + block scan of the lengths -> each string's offset;
//     (b) the tile's code bytes staged with aligned 16-byte loads;
//     (c) CODE-parallel decode: thread t takes 16-byte-aligned segments of the code bytes
//         (not one string: per-string loops ran as long as the longest of 64 strings and were
//         VALU-issue bound).  Pass 1 sums the decoded length of the codes starting in the
//         segment, a block scan places every segment, pass 2 ORs each code's <= 8 bytes into a
//         zeroed LDS image (ds_or_b32 into <= 3 dwords).  An escape (255) emits the next byte;
//         a segment that starts inside a run of 255s finds its parity by counting back;
//     (d) aligned 16-byte copy-out of the image, 16-byte views read from the image with
//         aligned dword reads + v_alignbyte.
//   A tile whose codes do not decode to exactly the sum of its lengths raises an error (the
//   reference would slice a shifted stream); tiles too large for the LDS images take a
//   per-string direct-to-HBM path that checks every string.
#include "intcol.hpp"

namespace vxg {

namespace {

constexpr int kTile = 256;            // strings per tile = threads per workgroup
// LDS images sized for short strings (TPC-H l_comment: 10-43 bytes, a 256-string tile is
// ~6.9 KB decoded / ~2.3 KB of codes).  ~18.9 KB of LDS per workgroup keeps 8 workgroups
// resident per CU.  Larger tiles take the direct path.
constexpr int kCodeLds = 6 * 1024;    // staged code bytes per tile
constexpr int kHeapLds = 10 * 1024;   // staged output bytes per tile
constexpr int kScanBlock = 1024;      // tiles per scan_blocks workgroup
constexpr int kSumTiles = 16;         // tiles per tile_sums workgroup

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

// The same view from an LDS byte image: four aligned dword reads and byte funnel shifts.
__device__ __forceinline__ uint4 lds_view(const uint32_t* h32, int a, uint32_t len, uint32_t offset) {
    const int w = a >> 2;
    const uint32_t sh = uint32_t(a & 3);
    const uint32_t d0 = h32[w], d1 = h32[w + 1], d2 = h32[w + 2], d3 = h32[w + 3];
    uint32_t w1 = __builtin_amdgcn_alignbyte(d1, d0, sh);
    if (len > 12) return make_uint4(len, w1, 0u, offset);
    uint32_t w2 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    uint32_t w3 = __builtin_amdgcn_alignbyte(d3, d2, sh);
    auto keep = [&](int base) -> uint32_t {
        const int k = int(len) - base;
        return k >= 4 ? 0xFFFFFFFFu : (k <= 0 ? 0u : (1u << (8 * k)) - 1u);
    };
    return make_uint4(len, w1 & keep(0), w2 & keep(4), w3 & keep(8));
}

__device__ __forceinline__ uint32_t byte_of(const uint4& v, int j) {
    const uint32_t w = j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w;
    return (w >> (8 * (j & 3))) & 0xFFu;
}

}  // namespace

template <class LenAcc>
__global__ __launch_bounds__(kTile) void fsst_tile_sums(LenAcc lens, uint64_t n, uint64_t n_tiles,
                                                        int64_t* __restrict__ tile_sums) {
    // 16 tiles per workgroup; in round r wave w sums tile 4r + w: each lane adds 4 consecutive
    // lengths (64 lanes x 4 = one 256-string tile), then ONE wave reduction per tile.
    const uint64_t t0 = uint64_t(blockIdx.x) * kSumTiles;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t v[kSumTiles / 4];
#pragma unroll
    for (int r = 0; r < kSumTiles / 4; r++) {  // 16 independent loads in flight per lane
        const uint64_t base = (t0 + 4 * r + wave) * kTile + 4 * lane;
        int64_t acc = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const uint64_t i = base + e;
            const int64_t x = lens(i < n ? i : n - 1);
            acc += i < n ? x : 0;
        }
        v[r] = acc;
    }
#pragma unroll
    for (int r = 0; r < kSumTiles / 4; r++) {
        const int64_t s = wave_sum(v[r]);
        const uint64_t t = t0 + 4 * r + wave;
        if (lane == 0 && t < n_tiles) tile_sums[t] = s;
    }
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

template <class OffAcc, class LenAcc>
__global__ __launch_bounds__(kTile) void fsst_decode(const uint64_t* __restrict__ symbols,
                                                     const uint8_t* __restrict__ sym_lens, unsigned n_symbols,
                                                     const uint8_t* __restrict__ codes, OffAcc code_offs,
                                                     LenAcc lens, uint64_t n,
                                                     const uint8_t* __restrict__ validity,
                                                     const int64_t* __restrict__ tile_prefix,
                                                     const int64_t* __restrict__ block_totals,
                                                     uint8_t* __restrict__ heap, uint4* __restrict__ views,
                                                     uint32_t* __restrict__ err) {
    __shared__ uint64_t s_sym[256];
    __shared__ uint8_t s_len[256];
    __shared__ int64_t ws[kTile / 64];
    __shared__ int64_t s_block_prefix;
    __shared__ int64_t s_coff[3];  // code_offs[0], code_offs[first], code_offs[last]
    __shared__ __attribute__((aligned(16))) uint8_t s_codes[kCodeLds + 48];
    __shared__ __attribute__((aligned(16))) uint32_t s_heap32[(kHeapLds + 48) / 4];
    uint8_t* const s_heap = reinterpret_cast<uint8_t*>(s_heap32);

    const int tid = threadIdx.x;
    // Prologue: every global load below is unconditional (indices clamped, results selected
    // afterwards) so they issue back to back and retire under ONE wait.
    const uint64_t i = uint64_t(blockIdx.x) * kTile + tid;
    const bool live = i < n;
    const uint64_t ii = live ? i : n - 1;
    const uint64_t first = uint64_t(blockIdx.x) * kTile;
    const uint64_t last = first + kTile < n ? first + kTile : n;
    const uint64_t sk = uint32_t(tid) < n_symbols ? uint32_t(tid) : 0;
    const uint64_t sym_v = symbols[sk];
    const uint8_t slen_v = sym_lens[sk];
    const int64_t len_v = lens(ii);
    if (tid < 3) s_coff[tid] = code_offs(tid == 0 ? 0 : (tid == 1 ? first : last));  // read after the scan's barrier
    const int64_t tp = tile_prefix[blockIdx.x];
    const uint8_t vbyte = validity ? validity[ii >> 3] : uint8_t(0xFF);
    // symbol slot 255 is the escape: length 1, its byte comes from the code stream
    // (kTile == 256 symbol slots.)  Symbols are stored zero-padded past their length, so a
    // code can OR all 8 bytes; a length > 8 is corrupt input.
    {
        const bool has = uint32_t(tid) < n_symbols;
        const uint32_t sl = slen_v;
        if (has && sl > 8) __hip_atomic_fetch_or(err, kErrFsst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_sym[tid] = has ? (sl >= 8 ? sym_v : sym_v & ((1ull << (8 * sl)) - 1)) : 0;
        s_len[tid] = has ? uint8_t(min(sl, 8u)) : uint8_t(tid == 255 ? 1 : 0);
    }
    if (tid < 64) {  // (a) prefix of the preceding 1024-tile blocks, one wave
        const uint64_t nb = blockIdx.x / kScanBlock;
        int64_t acc = 0;
        for (uint64_t b = tid; b < nb; b += 64) acc += block_totals[b];
        acc = wave_sum(acc);
        if (tid == 0) s_block_prefix = acc;
    }
    const int64_t my_len = live ? len_v : 0;
    int64_t tile_total;
    const int64_t my_rel = block_exclusive_scan<kTile / 64>(my_len, ws, tile_total);
    const int64_t tile_out0 = tp + s_block_prefix;
    const int64_t c_base = s_coff[0], cf = s_coff[1], cl = s_coff[2];
    // code offsets are relative to code_offs[0] (sliced_bytes(), varbin/mod.rs:130-136)
    const int64_t c0 = cf - c_base;
    const int64_t c1 = cl - c_base;
    const bool valid = live && ((vbyte >> (ii & 7)) & 1);
    const uint32_t vlen = valid ? uint32_t(my_len) : 0u;
    const bool stage = (c1 - c0) <= kCodeLds && tile_total <= kHeapLds && tile_total >= 0 && c1 >= c0;

    if (stage) {
        // LDS images sit at the same offset mod 16 as their global counterparts, so staging
        // loads and copy-out stores move whole aligned 16-byte chunks.
        const int64_t cabs0 = c_base + c0, cabs1 = c_base + c1;  // tile codes in `codes`
        const int cshift = int((reinterpret_cast<uintptr_t>(codes) + cabs0) & 15);
        const int hshift = int((reinterpret_cast<uintptr_t>(heap) + tile_out0) & 15);
        const int ncode = int(cabs1 - cabs0);
        const int span = cshift + ncode;  // tile codes at s_codes[cshift, span)
        {   // (b) an aligned 16-byte chunk holding at least one tile byte never crosses a page
            // boundary, so it is read whole; bytes outside the tile are ignored below.
            const uint8_t* a0 = codes + (cabs0 - cshift);
            const int nchunk = (span + 15) >> 4;
            for (int q = tid; q < nchunk; q += kTile)
                *reinterpret_cast<uint4*>(s_codes + 16 * q) = *reinterpret_cast<const uint4*>(a0 + 16 * q);
            const int nz = (hshift + int(tile_total) + 16 + 15) >> 4;  // zero the image (+16 slack)
            for (int q = tid; q < nz; q += kTile) reinterpret_cast<uint4*>(s_heap32)[q] = make_uint4(0, 0, 0, 0);
        }
        __syncthreads();

        // (c) code-parallel decode.  Segment = `seg` bytes (multiple of 16, at most two 16-byte
        // chunks) of s_codes per thread.
        static_assert(((kCodeLds + 15 + kTile - 1) / kTile + 15) / 16 <= 2, "segment > 2 chunks");
        const int seg = (((span + kTile - 1) / kTile) + 15) & ~15;
        const int s0 = tid * seg;
        const int nch = s0 < span ? (min(s0 + seg, span) - s0 + 15) >> 4 : 0;
        bool skip0 = false;  // is s_codes[s0] the literal byte of an escape?
        if (s0 > cshift && s0 < span) {
            int r = 0;
            for (int p = s0 - 1; p >= cshift && s_codes[p] == 255; --p) ++r;
            skip0 = r & 1;
        }
        // pass 1: decoded length of every code byte (0 for literals and bytes outside the
        // tile), packed as 4-bit fields, and their sum
        uint64_t lp[2] = {0, 0};
        int sum = 0;
        {
            bool skp = skip0;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                if (h < nch) {
                    const int q = s0 + 16 * h;
                    const uint4 ch = *reinterpret_cast<const uint4*>(s_codes + q);
                    const int lo = cshift - q, hi = span - q;  // in-tile bytes j: lo <= j < hi
                    uint32_t ls[16];
#pragma unroll
                    for (int j = 0; j < 16; j++) ls[j] = s_len[byte_of(ch, j)];  // 16 reads in flight
                    uint64_t pk = 0;
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        const uint32_t c = byte_of(ch, j);
                        const bool emit = j >= lo && j < hi && !skp;
                        skp = emit && c == 255;
                        const uint32_t L = emit ? ls[j] : 0u;
                        pk |= uint64_t(L) << (4 * j);
                        sum += int(L);
                    }
                    lp[h] = pk;
                }
            }
        }
        int64_t dec_total;
        const int64_t seg_rel = block_exclusive_scan<kTile / 64>(sum, ws, dec_total);
        if (tid == 0 && dec_total != tile_total)
            __hip_atomic_fetch_or(err, kErrFsst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // pass 2: every code ORs its (zero-padded) bytes into <= 3 dwords of the image.  All 16
        // symbol reads of a chunk are issued before its first ds_or; the ORs are unconditional
        // (zero for literals / outside the tile) so the chunk runs without branches.  Offsets
        // are clamped to the tile's end (only corrupt input, already flagged, reaches it).
        {
            int o = hshift + int(seg_rel);
            const int o_end = hshift + int(tile_total);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                if (h < nch) {
                    const int q = s0 + 16 * h;
                    const uint4 ch = *reinterpret_cast<const uint4*>(s_codes + q);
                    const uint32_t after = s_codes[q + 16];  // literal of an escape in byte 15
                    uint64_t sy[16];
#pragma unroll
                    for (int j = 0; j < 16; j++) sy[j] = s_sym[byte_of(ch, j)];
                    const uint64_t pk = lp[h];
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        const uint32_t c = byte_of(ch, j);
                        const int L = int((pk >> (4 * j)) & 15u);
                        const uint64_t lit = j < 15 ? byte_of(ch, j + 1) : after;
                        uint64_t m = c == 255 ? lit : sy[j];
                        m = (L > 0 && o < o_end) ? m : 0ull;
                        const int oc = min(o, o_end);
                        const uint32_t sh = 8u * uint32_t(oc & 3);
                        const int w = oc >> 2;
                        const uint64_t lo64 = m << sh;
                        const uint32_t hi32 = sh ? uint32_t(m >> (64u - sh)) : 0u;
                        __hip_atomic_fetch_or(&s_heap32[w], uint32_t(lo64), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_or(&s_heap32[w + 1], uint32_t(lo64 >> 32), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_or(&s_heap32[w + 2], hi32, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                        o += L;
                    }
                }
            }
        }
        __syncthreads();
        // (d) copy-out of [tile_out0, tile_out0 + tile_total): whole aligned 16-byte chunks via
        // ds_read_b128 + global_store_dwordx4; the ragged first/last chunk byte by byte (they
        // are shared with the neighbouring tiles)
        const int64_t g0 = tile_out0, g1 = tile_out0 + tile_total;
        const int64_t a0 = g0 - hshift;  // aligned chunk containing g0
        const int nchunk = int((g1 - a0 + 15) / 16);
        for (int q = tid; q < nchunk; q += kTile) {
            const int64_t g = a0 + 16 * q;
            if (g >= g0 && g + 16 <= g1) {
                *reinterpret_cast<uint4*>(heap + g) = *reinterpret_cast<const uint4*>(s_heap + 16 * q);
            } else {
                for (int b = 0; b < 16; b++)
                    if (g + b >= g0 && g + b < g1) heap[g + b] = s_heap[16 * q + b];
            }
        }
        if (live)
            views[i] = valid ? lds_view(s_heap32, hshift + int(my_rel), vlen, uint32_t(tile_out0 + my_rel))
                             : make_uint4(0, 0, 0, 0);
    } else {
        // direct path: per-string decode straight into HBM (codes of string i are
        // [offs[i], offs[i+1]); each must decode to exactly lengths[i] bytes)
        const int64_t my_c0 = live ? code_offs(ii) - c_base : 0;
        const int64_t my_c1 = live ? code_offs(ii + 1) - c_base : 0;
        const uint8_t* gcodes = codes + c_base;
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
        if (o != o_end) __hip_atomic_fetch_or(err, kErrFsst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
                       const uint8_t* code_bytes, const IntCol& offs, const IntCol& lens, uint64_t n,
                       const uint8_t* validity, void* scratch, uint8_t* heap, uint8_t* views,
                       uint32_t* err, hipStream_t s) {
    if (n == 0) return VXG_OK;
    if (n_symbols > 255) return set_error(VXG_ERR_INVALID_ARGUMENT, "FSST symbol table > 255 entries");
    const uint64_t n_tiles = (n + kTile - 1) / kTile;
    const uint64_t n_blocks = (n_tiles + kScanBlock - 1) / kScanBlock;
    const uint64_t n_sum_wgs = (n_tiles + kSumTiles - 1) / kSumTiles;
    int64_t* tiles = static_cast<int64_t*>(scratch);
    int64_t* blocks = tiles + n_tiles;
    auto run = [&](auto off_acc, auto len_acc) {
        using OA = decltype(off_acc);
        using LA = decltype(len_acc);
        hipLaunchKernelGGL((fsst_tile_sums<LA>), dim3(unsigned(n_sum_wgs)), dim3(kTile), 0, s, len_acc, n, n_tiles,
                           tiles);
        hipLaunchKernelGGL(fsst_scan_blocks, dim3(unsigned(n_blocks)), dim3(kScanBlock), 0, s, tiles, n_tiles,
                           blocks);
        hipLaunchKernelGGL((fsst_decode<OA, LA>), dim3(unsigned(n_tiles)), dim3(kTile), 0, s, symbols, sym_lens,
                           n_symbols, code_bytes, off_acc, len_acc, n, validity, tiles, blocks, heap,
                           reinterpret_cast<uint4*>(views), err);
    };
    // accessor = plain width 1/2/4/8 or packed T = 32/64
    auto with = [](const IntCol& c, auto&& f) -> bool {
        if (c.packed) {
            if (c.width == 4) return f(PackedCol<32>(c)), true;
            if (c.width == 8) return f(PackedCol<64>(c)), true;
            return false;
        }
        switch (c.width) {
        case 1: return f(PlainCol<1>(c)), true;
        case 2: return f(PlainCol<2>(c)), true;
        case 4: return f(PlainCol<4>(c)), true;
        case 8: return f(PlainCol<8>(c)), true;
        default: return false;
        }
    };
    bool ok = true;
    const bool ok_off = with(offs, [&](auto oa) { ok = with(lens, [&](auto la) { run(oa, la); }); });
    if (!ok_off || !ok)
        return set_error(VXG_ERR_MISMATCHED_TYPES, "FSST offsets/lengths must be 1/2/4/8-byte integers "
                                                    "(packed: 32/64-bit)");
    return hip_check(hipGetLastError(), "fsst kernels");
}

}  // namespace vxg
