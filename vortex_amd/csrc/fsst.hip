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
//     (c) CODE-parallel decode: thread t takes a segment of ND dwords of the code bytes (not
//         one string: per-string loops ran as long as the longest of 64 strings and were
//         VALU-issue bound; ND per tile, the segment code templated on it, branch-free).
//         Pass 1 sums the decoded length of the codes starting in the segment, a block scan
//         places every segment, pass 2 ORs each code's <= 8 bytes into a zeroed LDS image
//         (ds_or_b32 into <= 3 dwords).  An escape (255) emits the next byte; a segment that
//         starts inside a run of 255s finds its parity by counting back;
//     (d) aligned 16-byte copy-out of the image, 16-byte views read from the image with
//         aligned dword reads + v_alignbyte.
//   A tile whose codes do not decode to exactly the sum of its lengths raises an error (the
//   reference would slice a shifted stream); tiles too large for the LDS images take a
//   per-string direct-to-HBM path that checks every string.
#include <algorithm>
#include <tuple>

#include "fl_unpack_impl.hpp"
#include "intcol.hpp"
#include "k1g_impl.hpp"

namespace vxg {


namespace {

constexpr int kTile = 256;            // threads per workgroup = strings per tile
// (Two strings per thread -- twice the work per tile, 27 KiB of LDS -- measured 112 us on C4
// against 109 us for one: profiles/r03_fsst_spt.md.)
constexpr int kTS = kTile;            // strings per tile
// LDS images sized for short strings (TPC-H l_comment: 10-43 bytes, a 256-string tile is
// ~6.8 KB decoded / ~2.2 KB of codes).  Larger tiles take the direct path.
constexpr int kCodeLds = 6 * 1024;    // staged code bytes per tile
constexpr int kHeapLds = 10 * 1024;   // staged output bytes per tile
constexpr int kTPB = 1024 / kTS;      // tiles per FastLanes block of lengths
constexpr int kScanTiles = 32 * kTPB; // tiles per pre-pass workgroup (= 32 FastLanes blocks)

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
// [len][first 4 bytes][buffer_index][offset].  `get(j)` returns byte j of the string (only
// called for j < 12 inline / j < 4 prefix, and masked by j < len).
template <typename Get>
__device__ __forceinline__ uint4 build_view(uint32_t len, uint32_t offset, uint32_t bidx, Get get) {
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
        w2 = bidx;
        w3 = offset;
    }
    return make_uint4(len, w1, w2, w3);
}

// The same view from an LDS byte image: four aligned dword reads and byte funnel shifts; the
// inline bytes past the string are masked with hi32(0xFFFFFFFF << 8 k), k = clamp(len - base, 0, 4).
__device__ __forceinline__ uint4 lds_view(const uint32_t* h32, int a, uint32_t len, uint32_t offset, uint32_t bidx) {
    const int w = a >> 2;
    const uint32_t sh = uint32_t(a & 3);
    const uint32_t d0 = h32[w], d1 = h32[w + 1], d2 = h32[w + 2], d3 = h32[w + 3];
    uint32_t w1 = __builtin_amdgcn_alignbyte(d1, d0, sh);
    if (len > 12) return make_uint4(len, w1, bidx, offset);
    uint32_t w2 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    uint32_t w3 = __builtin_amdgcn_alignbyte(d3, d2, sh);
    auto keep = [&](int base) -> uint32_t {
        const int k = min(max(int(len) - base, 0), 4);
        return uint32_t((0xFFFFFFFFull << (8 * k)) >> 32);
    };
    return make_uint4(len, w1 & keep(0), w2 & keep(4), w3 & keep(8));
}

// Bytes [sh, sh + 16) of the 32-byte concatenation x:y (little endian), sh in [0, 16).
__device__ __forceinline__ uint4 funnel16(const uint4 x, const uint4 y, int sh) {
    const uint32_t z[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
    const uint32_t b = uint32_t(sh & 3);
    auto ab = [b](uint32_t hi, uint32_t lo) { return __builtin_amdgcn_alignbyte(hi, lo, b); };
    switch (sh >> 2) {  // uniform per tile
    case 0: return make_uint4(ab(z[1], z[0]), ab(z[2], z[1]), ab(z[3], z[2]), ab(z[4], z[3]));
    case 1: return make_uint4(ab(z[2], z[1]), ab(z[3], z[2]), ab(z[4], z[3]), ab(z[5], z[4]));
    case 2: return make_uint4(ab(z[3], z[2]), ab(z[4], z[3]), ab(z[5], z[4]), ab(z[6], z[5]));
    default: return make_uint4(ab(z[4], z[3]), ab(z[5], z[4]), ab(z[6], z[5]), ab(z[7], z[6]));
    }
}

__device__ __forceinline__ uint32_t byte_of(const uint4& v, int j) {
    const uint32_t w = j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w;
    return (w >> (8 * (j & 3))) & 0xFFu;
}

}  // namespace

// Inclusive scan of one int32 per lane across the wave: DPP row shifts inside 16-lane rows,
// then row broadcasts (no LDS round trips).
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Exact wave-wide total of one int64 per lane, uniform (SGPR) result, without LDS: three DPP
// inclusive scans of 32-bit parts (16 + 16 bits of the low word: each sum < 2^22; the high word
// modulo 2^32, which is all the 64-bit total needs), read from lane 63.  Replaces a 64-bit
// __shfl_xor tree (6 rounds of two ds_bpermute + ~7 VALU).
__device__ __forceinline__ int64_t wave_total64(int64_t v) {
    const uint64_t u = uint64_t(v);
    const int a = wave_incl_scan(int(uint32_t(u) & 0xFFFFu));
    const int b = wave_incl_scan(int(uint32_t(u) >> 16));
    const int c = wave_incl_scan(int(uint32_t(u >> 32)));
    const uint32_t A = uint32_t(__builtin_amdgcn_readlane(a, 63));
    const uint32_t B = uint32_t(__builtin_amdgcn_readlane(b, 63));
    const uint32_t C = uint32_t(__builtin_amdgcn_readlane(c, 63));
    return int64_t(uint64_t(A) + (uint64_t(B) << 16) + (uint64_t(C) << 32));
}

// Exclusive block scan of one int32 per thread (kTile/64 waves); `ws` must not be reused
// before the next barrier.
__device__ __forceinline__ int block_excl_scan32(int v, int* ws, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = wave_incl_scan(v);
    if (lane == 63) ws[wave] = x;
    __syncthreads();
    int before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kTile / 64; w++) {
        const int s = ws[w];
        before += w < wave ? s : 0;
        tot += s;
    }
    total = tot;
    return before + x - v;
}

// Pre-pass: per workgroup of 128 tiles, the tile length sums, their exclusive scan
// (tile_prefix) and the workgroup total (block_totals).  The decode adds the totals of the
// preceding workgroups (<= a few hundred) itself.
// The absolute code offset at which each tile's codes end (code_offs[min(256 (t + 1), n)]): the
// decode reads its tile's code range from these (with the tile prefix, one L2 round trip) and
// issues the code loads together with its other prologue loads.  One element per thread of the
// first kScanTiles threads, read before the pre-pass's barrier.
__device__ __forceinline__ int64_t tile_code_end(const FsstChunk& c, uint64_t sb) {
    const uint64_t tt = sb * kScanTiles + threadIdx.x;
    const uint64_t n_tiles = (c.n + kTS - 1) / kTS;
    if (threadIdx.x >= kScanTiles || tt >= n_tiles) return 0;
    const uint64_t e = (tt + 1) * kTS < c.n ? (tt + 1) * kTS : c.n;
    return intcol_get(c.offs, e);
}

__device__ __forceinline__ void scan_tile_sums(const int64_t* s_ts, int64_t* ws, uint64_t n_tiles, uint64_t sb,
                                               int64_t* __restrict__ tile_prefix, int64_t* __restrict__ block_totals,
                                               int64_t* __restrict__ tile_code, int64_t code_end) {
    // sb = scan block within the chunk; tile_prefix / block_totals / tile_code point at the
    // chunk's slices
    const int tid = threadIdx.x;
    int64_t tot;
    const int64_t ex = block_exclusive_scan<kTile / 64>(tid < kScanTiles ? s_ts[tid] : 0, ws, tot);
    const uint64_t tt = sb * kScanTiles + tid;
    if (tid < kScanTiles && tt < n_tiles) {
        tile_prefix[tt] = ex;
        tile_code[tt] = code_end;
    }
    if (tid == 0) block_totals[sb] = tot;
}

// Chunk of workgroup g in a launch: workgroup-uniform binary search on the kernarg table's
// first_*, or (EXT: a recorded plan's device table of any length) the wave-wide count.  EXT is
// a template parameter so the kernarg path keeps its scalar-load code unchanged.
template <bool SCAN, bool EXT>
__device__ __forceinline__ const FsstChunk& fsst_chunk_of(const FsstTable& tab, uint64_t g) {
    if constexpr (EXT) {
        return tab.ext[ext_chunk_index(tab.ext, tab.n, g,
                                       [](const FsstChunk& d) { return SCAN ? d.first_scan : d.first_tile; })];
    } else {
        uint32_t lo = 0, hi = tab.n;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((SCAN ? tab.c[mid].first_scan : tab.c[mid].first_tile) <= g) lo = mid; else hi = mid;
        }
        return tab.c[lo];
    }
}

// Any length column: wave w sums tile 4r + w in round r (kTS / 64 consecutive lengths per lane).
template <class LenAcc, bool EXT>
__global__ __launch_bounds__(kTile) void fsst_tile_scan(FsstTable tab, int64_t* __restrict__ tile_prefix_all,
                                                        int64_t* __restrict__ block_totals_all,
                                                        int64_t* __restrict__ tile_code_all) {
    __shared__ int64_t s_ts[kScanTiles];
    __shared__ int64_t ws[kTile / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const FsstChunk& c = fsst_chunk_of<true, EXT>(tab, blockIdx.x);
    const LenAcc lens(c.lens);
    const uint64_t n = c.n, n_tiles = (n + kTS - 1) / kTS, sb = blockIdx.x - c.first_scan;
    int64_t* const tile_prefix = tile_prefix_all + c.first_tile;
    int64_t* const block_totals = block_totals_all + c.first_scan;
    const int64_t code_end = tile_code_end(c, sb);
    const uint64_t t0 = sb * kScanTiles;
    constexpr int PL = kTS / 64;  // lengths per lane per tile
    for (int r0 = 0; r0 < kScanTiles / 4; r0 += 8) {
        int64_t v[8];
#pragma unroll
        for (int r = 0; r < 8; r++) {  // 32 independent loads in flight per lane
            const uint64_t base = (t0 + 4 * (r0 + r) + wave) * kTS + PL * lane;
            int64_t acc = 0;
#pragma unroll
            for (int e = 0; e < PL; e++) {
                const uint64_t i = base + e;
                const int64_t x = lens(i < n ? i : n - 1);
                acc += i < n ? x : 0;
            }
            v[r] = acc;
        }
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const int64_t sum = wave_total64(v[r]);
            if (lane == 0) s_ts[4 * (r0 + r) + wave] = sum;
        }
    }
    __syncthreads();
    scan_tile_sums(s_ts, ws, n_tiles, sb, tile_prefix, block_totals, tile_code_all + c.first_tile, code_end);
}

// Patch-free FoR(BitPacked u32/i32) lengths with offset 0 (the reference cascade): one thread
// per (FastLanes block, 32-bit lane) -- 1024 threads = the scan block's 32 blocks -- reads its
// lane's W words (the 32 lanes of a block: 128 contiguous bytes per word) and extracts the
// lane's 32 rows with immediate shifts.  Row R of a block holds strings (R % 8) * 128 + ..., i.e.
// tile (R % 8) * 128 / kTS of the block, so each thread keeps kTPB tile partial sums, reduced
// across the block's 32 lanes.  (Round 4 used 8 threads per block with 16-byte slices: 183
// workgroups of 4 waves for C4, ~1,000 VALU per wave on one serial chain per SIMD; round 5
// spreads the same work over 4x the waves.)
// A: int64 (any lengths) or uint32 (every length of the column < 2^23 and non-negative, so
// 256 of them sum below 2^31: the common case, half the adds and no 64-bit selects).
constexpr int kScanThreads = 32 * 32;  // 32 blocks x 32 lanes
static_assert(kScanTiles == 32 * kTPB, "a scan block is 32 FastLanes blocks of lengths");

template <int W, class A, int... Rs>
__device__ __forceinline__ void fl32_lane_rows(const uint32_t* p, int lane, uint32_t left, uint32_t for_shift,
                                               uint32_t reference, bool sgn, A* acc,
                                               std::integer_sequence<int, Rs...>) {
    auto row = [&](auto rc) {
        constexpr int R = decltype(rc)::value;
        uint32_t v = 0;
        if constexpr (W > 0) {
            constexpr int start = R * W, word = start / 32, sh = start % 32;
            constexpr uint32_t m = W >= 32 ? 0xFFFFFFFFu : ((1u << W) - 1u);
            if constexpr (sh + W <= 32) v = (p[word] >> sh) & m;
            else v = __builtin_amdgcn_alignbit(p[word + 1], p[word], uint32_t(sh)) & m;
        }
        const uint32_t u = uint32_t(v << for_shift) + reference;
        A x;
        if constexpr (sizeof(A) == 8) x = sgn ? A(int32_t(u)) : A(u);
        else x = u;
        acc[(R % 8) * 128 / kTS] += uint32_t(fl_index(R, lane)) < left ? x : A(0);
    };
    (row(std::integral_constant<int, Rs>{}), ...);
}

template <int W, bool EXT>
__global__ __launch_bounds__(kScanThreads) void fsst_tile_scan_fl32(FsstTable tab, int64_t* __restrict__ tile_prefix_all,
                                                                    int64_t* __restrict__ block_totals_all,
                                                                    int64_t* __restrict__ tile_code_all) {
    __shared__ int64_t s_ts[kScanTiles];
    __shared__ int64_t ws[2];
    const int tid = threadIdx.x, lane = tid & 31, lane64 = tid & 63, wave = tid >> 6;
    const FsstChunk& c = fsst_chunk_of<true, EXT>(tab, blockIdx.x);
    const uint8_t* __restrict__ packed = static_cast<const uint8_t*>(c.lens.p);
    const uint32_t for_shift = c.lens.shift, reference = uint32_t(c.lens.reference);
    const bool sgn = c.lens.sgn;
    const uint64_t n = c.n, n_tiles = (n + kTS - 1) / kTS, sb = blockIdx.x - c.first_scan;
    int64_t* const tile_prefix = tile_prefix_all + c.first_tile;
    int64_t* const block_totals = block_totals_all + c.first_scan;
    const uint64_t blk = sb * 32 + (tid >> 5);
    const int64_t code_end = tile_code_end(c, sb);
    // every value of the column below 2^23 (uniform): 32-bit sums are exact
    const uint64_t vmax = ((W >= 32 ? 0xFFFFFFFFull : ((1ull << W) - 1)) << for_shift) + reference;
    const bool small = vmax < (1ull << 23) && !(sgn && int32_t(reference) < 0);
    auto run = [&](auto* tag) {
        using A = std::remove_pointer_t<decltype(tag)>;
        A acc[kTPB];
#pragma unroll
        for (int k = 0; k < kTPB; k++) acc[k] = 0;
        if (blk * 1024 < n) {
            uint32_t p[W > 0 ? W : 1];
            if constexpr (W > 0) {
                const uint32_t* __restrict__ base = reinterpret_cast<const uint32_t*>(packed + blk * (128 * W)) + lane;
#pragma unroll
                for (int w = 0; w < W; w++) p[w] = gload(base + 32 * w);
            }
            const uint32_t left = blk * 1024 + 1024 <= n ? 1024u : uint32_t(n - blk * 1024);
            fl32_lane_rows<W>(p, lane, left, for_shift, reference, sgn, acc, std::make_integer_sequence<int, 32>{});
        }
#pragma unroll
        for (int k = 0; k < kTPB; k++) {
#pragma unroll
            for (int d = 1; d < 32; d <<= 1) acc[k] += __shfl_xor(acc[k], d, 64);
        }
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < kTPB; k++) s_ts[(tid >> 5) * kTPB + k] = int64_t(acc[k]);
        }
    };
    if (small) run(static_cast<uint32_t*>(nullptr));
    else run(static_cast<int64_t*>(nullptr));
    __syncthreads();
    // exclusive scan of the 128 tile sums by waves 0-1
    const int64_t v = tid < kScanTiles ? s_ts[tid] : 0;
    int64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(x, d, 64);
        if (lane64 >= d) x += y;
    }
    if (lane64 == 63 && wave < 2) ws[wave] = x;
    __syncthreads();
    const uint64_t tt = sb * kScanTiles + tid;
    if (tid < kScanTiles && tt < n_tiles) {
        tile_prefix[tt] = x - v + (wave == 1 ? ws[0] : 0);
        tile_code_all[c.first_tile + tt] = code_end;
    }
    if (tid == 0) block_totals[sb] = ws[0] + ws[1];
}

// ----- In-grid pre-pass records (the fused plan launch, round 6) -----
// A batched plan's fused launch runs its FSST group's length pre-pass as its FIRST workgroups
// (one per kFusedScanTiles tiles) instead of as a kernel of its own before it: on an 8-GPU C5
// shard that kernel was ~24 workgroups of 1,024 threads alone on the chip, latency-bound, plus a
// launch boundary.  The records are published with the launch's tag in their top 16 bits (value:
// low 48 bits, two's complement) by single-copy-atomic 8-byte device-scope stores, so a tile
// reads a record and its validity in ONE load: in the common case (the pre-pass workgroups,
// dispatched first, finished long before) the tile's prologue keeps its two round trips; a record
// with another tag (the previous launch's) is re-read until it carries this one.  Workgroups are
// dispatched in grid order, so every pre-pass workgroup is resident or done before any tile that
// waits for it: the wait always ends.  (A bound on it reports kErrPlanSync instead of hanging
// should two replays of one plan ever overlap.)  The tag (1-65535, never 0, the zero-initialised
// records' tag) is a kernel argument that vxg_plan_launch advances before every launch.  (A
// device-side epoch advanced by the launch's last workgroup -- one same-address device-scope
// atomic per workgroup -- serialised to ~75 ns per workgroup: the 8-GPU C5 shard's fused launch
// took 448 us instead of ~38.)
constexpr int kFusedScanTiles = 32;  // tiles per in-grid pre-pass workgroup = 8 FastLanes length blocks
static_assert(kFusedScanTiles * kTS == 8 * 1024, "an in-grid scan block is 8 FastLanes blocks of lengths");

__device__ __forceinline__ int64_t rec_load(const int64_t* p) {
    return __hip_atomic_load((gptr<const int64_t>)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void rec_store(int64_t* p, int64_t v) {
    __hip_atomic_store((gptr<int64_t>)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t rec_tag(int64_t r) { return uint32_t(uint64_t(r) >> 48); }
__device__ __forceinline__ int64_t rec_val(int64_t r) { return int64_t(uint64_t(r) << 16) >> 16; }
// (a value outside [-2^47, 2^47) -- only corrupt lengths or offsets give one -- is reported)
__device__ __forceinline__ int64_t rec_make(int64_t v, uint32_t tag, uint32_t* err) {
    if (v != rec_val(v)) __hip_atomic_fetch_or(err, kErrFsst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return int64_t((uint64_t(v) & ((1ull << 48) - 1)) | (uint64_t(tag) << 48));
}
// The record at p once it carries `tag` (r: the value already loaded from p).
__device__ __forceinline__ int64_t rec_wait(const int64_t* p, int64_t r, uint32_t tag, uint32_t* err) {
    for (uint32_t k = 0; rec_tag(r) != tag; k++) {
        if (k == (1u << 18)) {  // ~0.3 s: never in a well-formed replay
            __hip_atomic_fetch_or(err, kErrPlanSync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
        r = rec_load(p);
    }
    return rec_val(r);
}
__device__ __forceinline__ int64_t uni64(int64_t x) {
    const uint64_t u = uint64_t(x);
    return int64_t(uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(u))))) |
                   (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(u >> 32))))) << 32));
}

// One in-grid pre-pass workgroup: scan block sb (kFusedScanTiles tiles) of chunk c -- the tile
// length sums, their exclusive scan, the block total and each tile's code end, tagged.  Patch-free
// FoR(BitPacked u32) lengths at offset 0 (the file reader's cascade) are staged 4 FastLanes blocks
// at a time (<= 16 KiB) and extracted one lane's 16 rows per thread (runtime width: rows R W of
// the lane's words, funnel-shifted from LDS); any other length column is read element-wise.
template <class LenAcc>
__device__ __forceinline__ void fsst_prepass_ingrid(const FsstChunk& c, uint64_t sb, int64_t* __restrict__ tp_all,
                                                    int64_t* __restrict__ bt_all, int64_t* __restrict__ tc_all,
                                                    uint32_t tag, uint8_t* lds, uint32_t* err) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int64_t* const s_ts = reinterpret_cast<int64_t*>(lds);  // kFusedScanTiles tile sums
    uint32_t* const stage = reinterpret_cast<uint32_t*>(lds + 256);
    const uint64_t n = c.n, n_tiles = (n + kTS - 1) / kTS, t0 = sb * kFusedScanTiles;
    const uint64_t tt = t0 + uint64_t(tid);
    int64_t code_end = 0;  // (issued first; used last)
    if (tid < kFusedScanTiles && tt < n_tiles) code_end = intcol_get(c.offs, (tt + 1) * kTS < n ? (tt + 1) * kTS : n);
    const IntCol& L = c.lens;
    if (L.packed && L.width == 4 && L.offset == 0 && L.W <= 32) {  // uniform
        const uint32_t W = L.W, shift = L.shift, ref = uint32_t(L.reference);
        const uint32_t mask = W >= 32 ? 0xFFFFFFFFu : ((1u << W) - 1u);
        const uint64_t nblk = (n + 1023) / 1024;
        const int l32 = lane & 31, half = lane >> 5;
        for (int pass = 0; pass < 2; pass++) {
            const uint64_t blk0 = sb * 8 + uint64_t(pass) * 4;
            const uint64_t have = blk0 < nblk ? (nblk - blk0 < 4 ? nblk - blk0 : 4) : 0;
            const uint4* src = reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(L.p) + blk0 * (128ull * W));
            for (uint32_t q = tid; q < uint32_t(have) * 8u * W; q += kTile)
                reinterpret_cast<uint4*>(stage)[q] = gload(src + q);
            __syncthreads();
            // wave w: block blk0 + w; lanes 0-31 rows 0-15 of lane l32, lanes 32-63 rows 16-31
            int64_t acc[kTPB] = {0, 0, 0, 0};
            const uint64_t blk = blk0 + uint64_t(wave);
            if (blk < nblk) {
                const uint32_t left = blk * 1024 + 1024 <= n ? 1024u : uint32_t(n - blk * 1024);
                const uint32_t* words = stage + 32u * W * uint32_t(wave);
#pragma unroll 4  // (fully unrolled: 152 B/lane of scratch in the fused kernel)
                for (int r = 0; r < 16; r++) {
                    const uint32_t R = uint32_t(16 * half + r);
                    uint32_t v = 0;
                    if (W) {
                        const uint32_t start = R * W, w0 = start >> 5, w1 = w0 + 1 < W ? w0 + 1 : w0;
                        v = __builtin_amdgcn_alignbit(words[32 * w1 + l32], words[32 * w0 + l32], start & 31) & mask;
                    }
                    const uint32_t u = uint32_t(v << shift) + ref;
                    const int64_t x = L.sgn ? int64_t(int32_t(u)) : int64_t(u);
                    acc[(R % 8) * 128 / kTS] += uint32_t(fl_index(int(R), l32)) < left ? x : 0;
                }
            }
#pragma unroll
            for (int k = 0; k < kTPB; k++) {
                const int64_t s = wave_total64(acc[k]);
                if (lane == 0) s_ts[(pass * 4 + wave) * kTPB + k] = s;
            }
            __syncthreads();  // (the stage is refilled by the next pass; s_ts published)
        }
    } else {
        // wave w sums tiles t0 + w + 4 r (r < 8), kTS / 64 consecutive lengths per lane, four tiles'
        // loads in flight at a time (the fused kernel's 64-VGPR budget)
        const LenAcc lens(L);
        constexpr int PL = kTS / 64, RB = 4;
#pragma unroll 1
        for (int r0 = 0; r0 < kFusedScanTiles / 4; r0 += RB) {
            int64_t v[RB];
#pragma unroll
            for (int r = 0; r < RB; r++) {
                const uint64_t base = (t0 + 4 * (r0 + r) + wave) * kTS + PL * lane;
                int64_t a = 0;
#pragma unroll
                for (int e = 0; e < PL; e++) {
                    const uint64_t i = base + e;
                    const int64_t x = lens(i < n ? i : n - 1);
                    a += i < n ? x : 0;
                }
                v[r] = a;
            }
#pragma unroll
            for (int r = 0; r < RB; r++) {
                const int64_t s = wave_total64(v[r]);
                if (lane == 0) s_ts[4 * (r0 + r) + wave] = s;
            }
        }
        __syncthreads();
    }
    if (wave == 0) {  // exclusive scan of the block's tile sums, tagged records
        const int64_t x0 = lane < kFusedScanTiles ? s_ts[lane] : 0;
        int64_t x = x0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane < kFusedScanTiles && t0 + uint64_t(lane) < n_tiles) {
            rec_store(tp_all + c.first_tile + t0 + lane, rec_make(x - x0, tag, err));
            rec_store(tc_all + c.first_tile + t0 + lane, rec_make(code_end, tag, err));
        }
        if (lane == kFusedScanTiles - 1) rec_store(bt_all + c.first_scan + sb, rec_make(x, tag, err));
    }
}

// Length of string first + k of a tile (k clamped by the caller), in two steps so the load can
// be issued together with the prologue's other loads and used after all of them: issue() starts
// the load(s), value() finishes.  A packed (FastLanes) length column's tile lies in at most two
// blocks: the block base is uniform and the in-block index 32-bit (unpack_single arithmetic of
// intcol.hpp fl_word_pair, whose two words are combined only in value()).
template <class LenAcc>
struct TileLen {
    int64_t x;
    __device__ __forceinline__ void issue(const LenAcc& a, uint64_t first, uint32_t k) { x = a(first + k); }
    __device__ __forceinline__ int64_t value(const LenAcc&) const { return x; }
};
template <int T>
struct TileLen<PackedCol<T>> {
    using E = std::conditional_t<T == 32, uint32_t, uint64_t>;
    E lo, hi;
    uint32_t sh;
    __device__ __forceinline__ void issue(const PackedCol<T>& a, uint64_t first, uint32_t k) {
        // raw buffer loads over the tile's (at most) two blocks: no branch for W = 0 (the
        // resource then has no records and the loads return 0 without touching memory)
        constexpr uint32_t LANES = 1024 / T;
        const uint64_t g0 = first + a.offset;  // uniform
        const uint8_t* base = static_cast<const uint8_t*>(a.p) + (g0 >> 10) * (128ull * a.W);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), short(0), int(256 * a.W), 0x00020000);
        const uint32_t local = uint32_t(g0 & 1023) + k;
        const uint32_t idx = local & 1023, lane = idx % LANES, s = idx >> 7;
        const uint32_t fl = ((idx & 127) - lane) >> 4;
        const uint32_t row = (((fl & 1) << 2) | (fl & 2) | (fl >> 2)) * 8 + s;  // FL_ORDER[fl]*8 + s
        const uint32_t start = __umul24(row, a.W), word = start / T;
        const uint32_t word2 = word + 1 < a.W ? word + 1 : word;
        const uint32_t bo = (local >> 10) ? 128 * a.W : 0u;
        sh = start % T;
        if constexpr (T == 32) {
            lo = __builtin_amdgcn_raw_buffer_load_b32(rs, bo + 4 * (LANES * word + lane), 0, 0);
            hi = __builtin_amdgcn_raw_buffer_load_b32(rs, bo + 4 * (LANES * word2 + lane), 0, 0);
        } else {
            const auto l2 = __builtin_amdgcn_raw_buffer_load_b64(rs, bo + 8 * (LANES * word + lane), 0, 0);
            const auto h2 = __builtin_amdgcn_raw_buffer_load_b64(rs, bo + 8 * (LANES * word2 + lane), 0, 0);
            lo = uint64_t(uint32_t(l2[0])) | (uint64_t(uint32_t(l2[1])) << 32);
            hi = uint64_t(uint32_t(h2[0])) | (uint64_t(uint32_t(h2[1])) << 32);
        }
    }
    __device__ __forceinline__ int64_t value(const PackedCol<T>& a) const {
        const E mask = a.W >= uint32_t(T) ? E(~E(0)) : E((E(1) << a.W) - 1);
        E v;
        if constexpr (T == 32) v = __builtin_amdgcn_alignbit(hi, lo, sh) & mask;
        else v = (sh ? (lo >> sh) | (hi << (64 - sh)) : lo) & mask;
        const E r = E(E(v << a.shift) + E(a.reference));
        if constexpr (T == 64) return int64_t(r);
        else return a.sgn ? int64_t(int32_t(r)) : int64_t(r);
    }
};

template <class V4>
__device__ __forceinline__ uint4 as_uint4(const V4& v) {
    return make_uint4(uint32_t(v[0]), uint32_t(v[1]), uint32_t(v[2]), uint32_t(v[3]));
}

// (c) CODE-parallel decode of a staged tile: thread t takes code bytes [4 ND t, 4 ND (t + 1)) of
// the tile (ND dwords; ND uniform per tile = ceil(span / 1 KiB)).  Pass 1 packs each code's
// decoded length x 8 into one byte lane per dword (v_sad_u8 sums them), a block scan places every
// segment, pass 2 ORs each code's zero-padded symbol into <= 3 dwords of the zeroed LDS image.
// Pass 1 first assumes no escape: code 255 reads the sentinel length 16 (x 8 = bit 7 of its byte
// lane, real lengths are <= 8), and a tile in which any thread saw it (flag through the scan's
// barrier) redoes pass 1 in the general form and scans again -- an escape (255) emits the next
// byte; a segment that starts inside a run of 255s finds its parity by counting back; bytes past
// the tile do not count.  Threads whose segment starts past the tile do nothing (their ORs
// would all hit one address); the one thread whose segment straddles the tile end masks it.
template <int ND>
__device__ __forceinline__ void fsst_segments(const uint8_t* __restrict__ s_codes, int span,
                                              const uint64_t* __restrict__ s_sym, const uint8_t* __restrict__ s_len,
                                              uint32_t* __restrict__ s_heap32, int hshift, int ttot, int* ws_b,
                                              unsigned* ws_esc, uint32_t* __restrict__ err) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int s0 = tid * 4 * ND;
    const bool act = s0 < span;
    const uint32_t* __restrict__ c32 = reinterpret_cast<const uint32_t*>(s_codes);
    uint32_t pk[ND];  // (the code dwords are re-read in pass 2: fewer registers live across the scan)
    uint32_t sum8 = 0;
    bool esc = false;
#pragma unroll
    for (int d = 0; d < ND; d++) pk[d] = 0;
    if (act) {
        uint32_t wd[ND];
#pragma unroll
        for (int d = 0; d < ND; d++) wd[d] = c32[(s0 >> 2) + d];
#pragma unroll
        for (int d = 0; d < ND; d++) {
            const uint32_t x = wd[d];
            uint32_t ls[4];
#pragma unroll
            for (int j = 0; j < 4; j++) ls[j] = s_len[(x >> (8 * j)) & 0xFFu];
            uint32_t k = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) k |= ls[j] << (8 * j + 3);
            pk[d] = k;
        }
        if (s0 + 4 * ND > span) {  // bytes past the tile have no length
#pragma unroll
            for (int d = 0; d < ND; d++) {
                const int vb = span - (s0 + 4 * d);
                pk[d] &= vb >= 4 ? 0xFFFFFFFFu : (vb <= 0 ? 0u : (1u << (8 * vb)) - 1u);
            }
        }
        uint32_t any = 0;
#pragma unroll
        for (int d = 0; d < ND; d++) {
            any |= pk[d];
            sum8 = __builtin_amdgcn_sad_u8(pk[d], 0u, sum8);
        }
        esc = (any & 0x80808080u) != 0;
    }
    const unsigned long long eb = __ballot(esc);
    if (lane == 0) ws_esc[wave] = eb != 0;
    int dec_total;
    int seg_rel = block_excl_scan32(int(sum8 >> 3), ws_b, dec_total);
    const bool fast = (ws_esc[0] | ws_esc[1] | ws_esc[2] | ws_esc[3]) == 0;  // tile-uniform
    if (!fast) {
        sum8 = 0;
        if (act) {
            bool skp = false;  // is the current byte the literal of an escape?
            if (s0 > 0 && s_codes[s0 - 1] == 255) {
                int r = 0;
                for (int p = s0 - 1; p >= 0 && s_codes[p] == 255; --p) ++r;
                skp = r & 1;
            }
#pragma unroll
            for (int d = 0; d < ND; d++) {
                const uint32_t x = c32[(s0 >> 2) + d];
                uint32_t k = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t c = (x >> (8 * j)) & 0xFFu;
                    const bool emit = s0 + 4 * d + j < span && !skp;
                    skp = emit && c == 255;
                    const uint32_t L = emit ? (c == 255 ? 1u : uint32_t(s_len[c])) : 0u;
                    k |= L << (8 * j + 3);
                }
                pk[d] = k;
                sum8 = __builtin_amdgcn_sad_u8(k, 0u, sum8);
            }
        }
        __syncthreads();  // every thread has read the first scan's wave totals
        seg_rel = block_excl_scan32(int(sum8 >> 3), ws_b, dec_total);
    }
    if (tid == 0 && dec_total != ttot) __hip_atomic_fetch_or(err, kErrFsst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // a tile whose codes do not decode to its length sum (corrupt input, flagged above) is not written
    if (!act || dec_total != ttot) return;
    uint32_t o8 = uint32_t(hshift + seg_rel) << 3;  // bit position in the image
    auto put = [&](uint64_t m, uint32_t L8) {
        // (w1:w0) = sym << 8(o & 3), w2 = the bytes shifted past them
        const uint32_t sh = o8 & 24u;
        const uint32_t w = o8 >> 5;
        const uint64_t lo64 = m << sh;
        const uint32_t hi32 = uint32_t((m >> 32) << sh >> 32);
        __hip_atomic_fetch_or(&s_heap32[w], uint32_t(lo64), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_or(&s_heap32[w + 1], uint32_t(lo64 >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_or(&s_heap32[w + 2], hi32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        o8 += L8;
    };
    if (fast) {
        // the next code dword is requested before this dword's ORs: waiting for it then does not
        // also wait for the ORs (LDS requests complete in order)
        uint32_t xn = c32[s0 >> 2];
#pragma unroll
        for (int d = 0; d < ND; d++) {
            const uint32_t x = xn;
            uint64_t sy[4];
#pragma unroll
            for (int j = 0; j < 4; j++) sy[j] = s_sym[(x >> (8 * j)) & 0xFFu];
            if (d + 1 < ND) xn = c32[(s0 >> 2) + d + 1];
#pragma unroll
            for (int j = 0; j < 4; j++) put(sy[j], (pk[d] >> (8 * j)) & 0xFFu);
        }
    } else {
#pragma unroll
        for (int d = 0; d < ND; d++) {
            const uint32_t x = c32[(s0 >> 2) + d];
            const uint32_t after = s_codes[s0 + 4 * d + 4];  // literal of an escape in byte 3
            uint64_t sy[4];
#pragma unroll
            for (int j = 0; j < 4; j++) sy[j] = s_sym[(x >> (8 * j)) & 0xFFu];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t c = (x >> (8 * j)) & 0xFFu;
                const uint32_t L8 = (pk[d] >> (8 * j)) & 0xFFu;
                const uint64_t lit = j < 3 ? ((x >> (8 * j + 8)) & 0xFFu) : after;
                const uint64_t m = c == 255 ? lit : sy[j];
                put(L8 ? m : 0ull, L8);
            }
        }
    }
}


// The decode's LDS (declared by the kernel, handed to the tile functions).
struct DecLds {
    uint64_t* s_sym;
    uint8_t* s_len;
    int* ws_a;
    int* ws_b;
    unsigned* ws_bad;
    unsigned* ws_esc;
    int64_t* ws64;
    int64_t* s_block_prefix;
    uint8_t* s_codes;
    uint32_t* s_heap32;
};

// Everything a tile's decode reads from memory before it can start, requested together (no
// result used before all are issued): the pre-pass records (scalar), the thread's length word(s),
// its validity byte and two 16-byte chunks of the tile's code range.
template <class LenAcc>
struct TileIn {
    uint32_t tile;  // within the chunk
    int64_t tp, cl, cf;
    TileLen<LenAcc> tl;
    uint8_t vbyte;
    uint4 cx, cy;
};

// TAG (the fused launch's in-grid pre-pass): the records are tagged (rec_*), read with device-
// scope loads and waited for after the tile's other prologue loads are issued.
template <class OffAcc, class LenAcc, bool TAG = false>
__device__ __forceinline__ void tile_issue(const FsstChunk& ch, uint64_t g, const int64_t* __restrict__ tile_prefix_all,
                                           const int64_t* __restrict__ tile_code_all, TileIn<LenAcc>& in,
                                           uint32_t tag = 0, uint32_t* err = nullptr) {
    const int tid = threadIdx.x;
    const OffAcc code_offs(ch.offs);
    const LenAcc lens(ch.lens);
    const uint64_t n = ch.n;
    const uint32_t tile = uint32_t(g - ch.first_tile);  // within the chunk
    in.tile = tile;
    // the tile's code range [cf, cl) (absolute offsets into `codes`) comes from the pre-pass
    // records, so the code bytes are requested in the same round trip as the other loads.  The
    // records are indexed by the launch-global tile g (= first_tile + tile): their loads do not
    // wait for the chunk's fields
    const int64_t* const pp = tile_code_all + (g > 0 ? g - 1 : 0);
    int64_t prev;
    if constexpr (TAG) {
        // (waited for before the length and validity loads are issued: the record values are
        // uniform from then on, and those loads are needed only after the code round trip)
        const int64_t rtp = rec_load(tile_prefix_all + g), rcl = rec_load(tile_code_all + g), rpv = rec_load(pp);
        in.tp = uni64(rec_wait(tile_prefix_all + g, rtp, tag, err));
        in.cl = uni64(rec_wait(tile_code_all + g, rcl, tag, err));
        prev = tile > 0 ? uni64(rec_wait(pp, rpv, tag, err)) : 0;
    } else {
        in.tp = tile_prefix_all[g];
        in.cl = tile_code_all[g];
        prev = *pp;
    }
    const uint64_t first = uint64_t(tile) * kTile;
    const bool live = first + uint64_t(tid) < n;
    const uint32_t kc = live ? uint32_t(tid) : uint32_t(n - 1 - first);  // clamped index in the tile
    in.tl.issue(lens, first, kc);
    in.vbyte = ch.validity ? gload(ch.validity + ((first + kc) >> 3)) : uint8_t(0xFF);
    in.cf = tile > 0 ? prev : code_offs(0);
    const int cshift = int((reinterpret_cast<uintptr_t>(ch.codes) + uintptr_t(in.cf)) & 15);
    const int64_t span64 = in.cl - in.cf;
    const int span = span64 >= 0 && span64 <= kCodeLds ? int(span64) : 0;
    const uint4* const a0 = reinterpret_cast<const uint4*>(ch.codes + (in.cf - cshift));
    // chunks tid and tid + 1 of the tile's aligned code range (funnel-shifted when staged), as
    // bounds-checked buffer loads: no branch (a chunk past the range reads as zeros without a
    // memory access), so they retire under one wait
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint4*>(a0), short(0), span ? int((cshift + span + 15) & ~15) : 0, 0x00020000);
    in.cx = as_uint4(__builtin_amdgcn_raw_buffer_load_b128(crs, 16 * tid, 0, 0));
    in.cy = as_uint4(__builtin_amdgcn_raw_buffer_load_b128(crs, 16 * tid + 16, 0, 0));
}

// The chunk's symbol table: loads (symbol_load) and its LDS image (symbol_store).  Symbols are
// stored zero-padded past their length, so a code can OR all 8 bytes; a length > 8 is corrupt
// input (reported).  Slot 255 (the escape, never a symbol) has no bytes and the sentinel length
// 16 (pass 1's escape detector); escapes are decoded explicitly.
__device__ __forceinline__ void symbol_load(const FsstChunk& ch, uint64_t& sym_v, uint32_t& sl) {
    sym_v = 0;
    sl = 0;
    if (ch.n_symbols) {  // (an empty table -- e.g. trained on null strings only -- may have null buffers)
        const uint32_t sk = uint32_t(threadIdx.x) < ch.n_symbols ? uint32_t(threadIdx.x) : 0u;
        sym_v = gload(ch.symbols + sk);
        sl = gload(ch.sym_lens + sk);
    }
}
__device__ __forceinline__ void symbol_store(const FsstChunk& ch, const DecLds& L, uint64_t sym_v, uint32_t sl,
                                             uint32_t* __restrict__ err) {
    const int tid = threadIdx.x;
    const bool has = uint32_t(tid) < ch.n_symbols;
    L.s_sym[tid] = has ? (sl >= 8 ? sym_v : sym_v & ((1ull << (8 * sl)) - 1)) : 0;
    L.s_len[tid] = has ? uint8_t(min(sl, 8u)) : uint8_t(tid == 255 ? 16 : 0);
    if (has && sl > 8) __hip_atomic_fetch_or(err, kErrFsst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Prefix of the scan blocks before the tile's (<= a few hundred totals), by wave 0 into
// s_block_prefix: four loads per lane in flight per round (clamped index, no per-element
// branch), so a tile deep in a large chunk pays one memory round trip here, not one per 64 blocks.
template <int SCAN_TILES = kScanTiles, bool TAG = false>
__device__ __forceinline__ void block_prefix(const FsstChunk& ch, uint32_t tile, const int64_t* __restrict__ block_totals_all,
                                             const DecLds& L, uint32_t tag = 0, uint32_t* err = nullptr) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nb = tile / SCAN_TILES;
    if (wave != 0) return;
    if (nb == 0) {
        if (lane == 0) *L.s_block_prefix = 0;
        return;
    }
    const int64_t* __restrict__ block_totals = block_totals_all + ch.first_scan;
    int64_t acc = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
        int64_t v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t b = b0 + 64 * k + lane;
            v[k] = TAG ? rec_load(block_totals + (b < nb ? b : nb - 1)) : block_totals[b < nb ? b : nb - 1];
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t b = b0 + 64 * k + lane;
            if constexpr (TAG) v[k] = b < nb ? rec_wait(block_totals + b, v[k], tag, err) : 0;
            acc += b < nb ? v[k] : 0;
        }
    }
    acc = wave_total64(acc);
    if (lane == 0) *L.s_block_prefix = acc;
}

// Ablation mask (diagnostics only, VXG_FSST_ABL read once by the host; outputs are then WRONG):
// 1 skips the segment passes, 2 the copy-out, 4 the views, 8 everything after the prologue.
__constant__ uint32_t g_fsst_abl = 0;

// One tile's decode once its loads are in flight and its symbol table and s_block_prefix have been
// written (the length scan's barrier publishes them): length scan, staging, segments, copy-out,
// views -- or the per-string direct path.
template <class OffAcc, class LenAcc>
__device__ __forceinline__ void tile_run(const FsstChunk& ch, const TileIn<LenAcc>& in, const DecLds& L,
                                         uint32_t* __restrict__ err) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint8_t* __restrict__ codes = ch.codes;
    const OffAcc code_offs(ch.offs);
    const LenAcc lens(ch.lens);
    const uint64_t n = ch.n;
    uint8_t* __restrict__ heap = ch.heap;
    uint4* __restrict__ views = reinterpret_cast<uint4*>(ch.views);
    const uint32_t bidx = ch.bidx;
    const uint64_t first = uint64_t(in.tile) * kTile;
    const bool live = first + uint64_t(tid) < n;
    const uint8_t vbyte = in.vbyte;
    const int cshift = int((reinterpret_cast<uintptr_t>(codes) + uintptr_t(in.cf)) & 15);
    const int64_t span64 = in.cl - in.cf;
    const bool span_ok = span64 >= 0 && span64 <= kCodeLds;
    const int span = span_ok ? int(span64) : 0;  // tile codes at s_codes[0, span) once staged
    const uint4* const a0 = reinterpret_cast<const uint4*>(codes + (in.cf - cshift));  // (pointer arithmetic: global loads)
    const int nchunk = (span + 15) >> 4;
    uint8_t* const s_codes = L.s_codes;
    uint32_t* const s_heap32 = L.s_heap32;
    uint8_t* const s_heap = reinterpret_cast<uint8_t*>(s_heap32);
    const int64_t my_len = live ? in.tl.value(lens) : 0;
    const bool bad = my_len < 0 || my_len > kHeapLds;

    // (a) length scan: int32 with DPP when every length is in [0, kHeapLds] (then a staged
    // tile is possible), int64 otherwise (direct path).
    const unsigned long long bm = __ballot(bad);
    if (lane == 0) L.ws_bad[wave] = bm != 0;
    int t32;
    const int rel32 = block_excl_scan32(bad ? 0 : int(my_len), L.ws_a, t32);
    const bool any_bad = (L.ws_bad[0] | L.ws_bad[1] | L.ws_bad[2] | L.ws_bad[3]) != 0;
    int64_t my_rel = rel32, tile_total = t32;
    if (any_bad) my_rel = block_exclusive_scan<kTile / 64>(my_len, L.ws64, tile_total);  // uniform branch
    const int64_t tile_out0 = in.tp + *L.s_block_prefix;
    const bool stage = !any_bad && span_ok && tile_total <= kHeapLds;

    const uint32_t abl = g_fsst_abl;
    if (abl & 8) return;
    if (stage) {
        // (b) stage the tile's code bytes into LDS shifted so that the tile's first code is
        // s_codes[0] (chunk tid was loaded with the prologue; larger tiles load the rest here),
        // and zero the image.  (Doing this before the length scan, so that one barrier publishes
        // both, measured the same: profiles/r04_fsst_decode.md.)
        const int hshift = int((reinterpret_cast<uintptr_t>(heap) + tile_out0) & 15);  // image byte hshift = heap[tile_out0]
        const int ttot = int(tile_total);
        if (tid < nchunk) *reinterpret_cast<uint4*>(s_codes + 16 * tid) = funnel16(in.cx, in.cy, cshift);
        for (int q = tid + kTile; q < nchunk; q += kTile) {  // tiles of > 4 KiB of codes
            const uint4 x = gload(a0 + q);
            uint4 y = make_uint4(0, 0, 0, 0);
            if (cshift != 0 && 16 * (q + 1) - cshift < span) y = gload(a0 + q + 1);
            *reinterpret_cast<uint4*>(s_codes + 16 * q) = funnel16(x, y, cshift);
        }
        const int nz = (hshift + ttot + 16 + 15) >> 4;
        for (int q = tid; q < nz; q += kTile) reinterpret_cast<uint4*>(s_heap32)[q] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        if (!(abl & 1)) switch ((span + 4 * kTile - 1) / (4 * kTile)) {  // dwords per thread, tile-uniform
        case 0:
        case 1: fsst_segments<1>(s_codes, span, L.s_sym, L.s_len, s_heap32, hshift, ttot, L.ws_b, L.ws_esc, err); break;
        case 2: fsst_segments<2>(s_codes, span, L.s_sym, L.s_len, s_heap32, hshift, ttot, L.ws_b, L.ws_esc, err); break;
        case 3: fsst_segments<3>(s_codes, span, L.s_sym, L.s_len, s_heap32, hshift, ttot, L.ws_b, L.ws_esc, err); break;
        case 4: fsst_segments<4>(s_codes, span, L.s_sym, L.s_len, s_heap32, hshift, ttot, L.ws_b, L.ws_esc, err); break;
        case 5: fsst_segments<5>(s_codes, span, L.s_sym, L.s_len, s_heap32, hshift, ttot, L.ws_b, L.ws_esc, err); break;
        default: fsst_segments<6>(s_codes, span, L.s_sym, L.s_len, s_heap32, hshift, ttot, L.ws_b, L.ws_esc, err); break;
        }
        static_assert(kCodeLds <= 6 * 4 * kTile, "six dwords per thread cover the staged codes");
        __syncthreads();
        // (d) copy-out of [tile_out0, tile_out0 + ttot): the image sits at the same offset mod 16
        // as its destination, so whole aligned chunks [qa, qb) move as ds_read_b128 + 16-byte
        // stores; the <= 15 + 15 bytes of the ragged first/last chunk (shared with the
        // neighbouring tiles) are one byte store per lane of wave 0 (lanes 0-15 the head, 16-31
        // the tail) instead of a per-thread loop of byte/short/dword stores.
        if (!(abl & 2)) {
            uint8_t* const gbase = heap + (tile_out0 - hshift);
            const int end = hshift + ttot;
            const int qa = (hshift + 15) >> 4, qb = end >> 4;
            for (int q = qa + tid; q < qb; q += kTile)
                nt_store(reinterpret_cast<uint4*>(gbase + 16 * q), *reinterpret_cast<const uint4*>(s_heap + 16 * q));
            if (tid < 32) {
                const int a = tid < 16 ? tid : 16 * qb + (tid - 16);
                const bool inr = tid < 16 ? (a >= hshift && a < min(16 * qa, end)) : (a >= max(16 * qb, 16 * qa) && a < end);
                if (inr) gstore(gbase + a, s_heap[a]);
            }
        }
        if (live && !(abl & 4)) {
            const bool valid = (vbyte >> (tid & 7)) & 1;
            // non-temporal like the heap copy-out: the views are written once and not re-read
            nt_store(views + first + tid, valid ? lds_view(s_heap32, hshift + int(my_rel), uint32_t(my_len),
                                                          uint32_t(tile_out0 + my_rel), bidx)
                                                : make_uint4(0, 0, 0, 0));
        }
    } else {
        // direct path: per-string decode straight into HBM (codes of string i are
        // [offs[i], offs[i+1]); each must decode to exactly lengths[i] bytes)
        const uint64_t i = first + tid;
        const int64_t my_c0 = live ? code_offs(i) : 0;
        const int64_t my_c1 = live ? code_offs(i + 1) : 0;
        int64_t o = tile_out0 + my_rel;
        const int64_t o_start = o, o_end = o + my_len;
        for (int64_t k = my_c0; k < my_c1; k++) {
            const uint8_t c = gload(codes + k);
            if (c == 255) {
                ++k;
                if (o < o_end) gstore(heap + o, gload(codes + k));
                o++;
            } else {
                const uint64_t sym = L.s_sym[c];
                const int Ln = L.s_len[c];
                for (int b = 0; b < Ln; b++)
                    if (o + b < o_end) gstore(heap + o + b, uint8_t(sym >> (8 * b)));
                o += Ln;
            }
        }
        if (o != o_end) __hip_atomic_fetch_or(err, kErrFsst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (live) {
            const bool valid = (vbyte >> (i & 7)) & 1;
            const uint32_t vlen = valid ? uint32_t(my_len) : 0u;
            const uint8_t* hp = heap + o_start;
            // (non-temporal like the staged path's view store: the compiler merges the two stores
            // after the branch and keeps the hint only if both carry it)
            nt_store(views + i, valid ? build_view(vlen, uint32_t(o_start), bidx,
                                                   [&](int b) { return uint32_t(b) < vlen ? gload(hp + b) : uint8_t(0); })
                                      : make_uint4(0, 0, 0, 0));
        }
    }
}

// The decode's LDS carved from one buffer (the plan launch that runs decode tiles beside K1g
// jobs has only dynamic LDS): image, codes, symbols, scan scratch -- kDecLdsBytes in all.
constexpr uint32_t kDecHeapBytes = kHeapLds + 96;  // + slack: view reads past a string, and ORs
                                                   // of the (<= 3) dwords past the tile
constexpr uint32_t kDecCodesBytes = kCodeLds + 48; // + slack: the straddling segment's dwords
                                                   // past the tile (masked in pass 1)
constexpr uint32_t kDecLdsBytes = kDecHeapBytes + kDecCodesBytes + 8 * 256 + 8 * (kTile / 64) + 8 +
                                  4 * 4 * (kTile / 64) + 256;
static_assert(kDecHeapBytes % 16 == 0 && kDecCodesBytes % 16 == 0, "16-byte aligned stages");
__device__ __forceinline__ DecLds dec_lds(uint8_t* p) {
    DecLds L;
    L.s_heap32 = reinterpret_cast<uint32_t*>(p);
    p += kDecHeapBytes;
    L.s_codes = p;
    p += kDecCodesBytes;
    L.s_sym = reinterpret_cast<uint64_t*>(p);
    p += 8 * 256;
    L.ws64 = reinterpret_cast<int64_t*>(p);
    p += 8 * (kTile / 64);
    L.s_block_prefix = reinterpret_cast<int64_t*>(p);
    p += 8;
    L.ws_a = reinterpret_cast<int*>(p);
    L.ws_b = L.ws_a + kTile / 64;
    L.ws_bad = reinterpret_cast<unsigned*>(L.ws_b + kTile / 64);
    L.ws_esc = L.ws_bad + kTile / 64;
    L.s_len = reinterpret_cast<uint8_t*>(L.ws_esc + kTile / 64);
    return L;
}

// One tile per workgroup: the tile's loads (tile_issue) are all in flight before the symbol
// table and the scan-block prefix are loaded.  (Two consecutive tiles per workgroup with both
// tiles' loads issued in the prologue was measured 10 % slower on C4 -- 6 instead of 8 waves per
// SIMD; profiles/r04_fsst_decode.md.)
template <class OffAcc, class LenAcc, bool TAG = false>
__device__ __forceinline__ void fsst_decode_tile(const FsstChunk& ch, uint64_t g, const int64_t* __restrict__ tile_prefix_all,
                                                 const int64_t* __restrict__ block_totals_all,
                                                 const int64_t* __restrict__ tile_code_all, uint32_t* __restrict__ err,
                                                 const DecLds& L, uint32_t tag = 0) {
    TileIn<LenAcc> in;
    uint64_t sym_v;
    uint32_t sl;
    tile_issue<OffAcc, LenAcc, TAG>(ch, g, tile_prefix_all, tile_code_all, in, tag, err);
    symbol_load(ch, sym_v, sl);
    block_prefix<TAG ? kFusedScanTiles : kScanTiles, TAG>(ch, in.tile, block_totals_all, L, tag, err);
    symbol_store(ch, L, sym_v, sl, err);
    tile_run<OffAcc, LenAcc>(ch, in, L, err);
}

template <class OffAcc, class LenAcc, bool EXT>
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8, 8))) void fsst_decode(
    FsstTable tab, const int64_t* __restrict__ tile_prefix_all, const int64_t* __restrict__ block_totals_all,
    const int64_t* __restrict__ tile_code_all, uint32_t* __restrict__ err, const uint32_t* __restrict__ wg_chunk) {
    __shared__ __attribute__((aligned(16))) uint8_t s_lds[kDecLdsBytes];
    const DecLds L = dec_lds(s_lds);
    // the tile's chunk: a recorded plan's device table through the plan's per-tile map (one
    // scalar load; the chunk's entry is then shared by its ~255 tiles' workgroups in the scalar
    // cache -- a per-tile copy of the entry, which saves that dependent load but always misses,
    // measured 1-2 % slower on C5: profiles/r04_fsst_decode.md), else the workgroup-uniform
    // search of the kernel-argument table (a chunk INDEX, not a pointer: a pointer into the
    // kernel-argument table would force the table into scratch)
    const uint64_t g = blockIdx.x;
    uint32_t ci;
    if constexpr (EXT) {
        ci = wg_chunk[g];
    } else {
        uint32_t lo = 0, hi = tab.n;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tab.c[mid].first_tile <= g) lo = mid; else hi = mid;
        }
        ci = lo;
    }
    fsst_decode_tile<OffAcc, LenAcc>(EXT ? tab.ext[ci] : tab.c[ci], g, tile_prefix_all, block_totals_all, tile_code_all,
                                     err, L);
}

// The plan launch of a batched plan (FsstFused): one recorded group's decode tiles and the
// plan's K1g jobs (k1g_impl.hpp) in ONE grid, so that the decode's latency-bound tiles (two
// dependent memory round trips and two barriers per 256 strings) run beside the K1g jobs' store
// streams instead of alone.  Grid: [fa.prepass in-grid pre-pass workgroups] then the K1g and
// decode workgroups; after `delay` K1g workgroups the decode tiles are spread evenly over the next
// `mix` workgroups (the rest are K1g jobs): workgroup b < mix of that range is tile floor(b T /
// mix) when that floor steps at b.  Every workgroup has the decode's LDS (8 per CU, the wave
// limit anyway).
template <class OffAcc, class LenAcc>
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8, 8))) void fsst_k1g_kernel(
    FsstFusedArgs fa, const GenChunk* __restrict__ gtab, uint32_t gn, uint32_t dict_off, bool dict_lds,
    uint32_t* __restrict__ err, uint64_t gpe) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint64_t P = fa.prepass, T = fa.tiles, M = fa.mix, D = fa.delay;
    const uint32_t tag = fa.tag;
    const uint64_t b = blockIdx.x;
    if (b < P) {
        fsst_prepass_ingrid<LenAcc>(fa.ext[fa.scan_chunk[b]], b - fa.ext[fa.scan_chunk[b]].first_scan,
                                    const_cast<int64_t*>(fa.tp), const_cast<int64_t*>(fa.bt), const_cast<int64_t*>(fa.tc),
                                    tag, lds, err);
    } else {
        const uint64_t bb = b - P;
        uint64_t gg = ~0ull;  // K1g workgroup, or a decode tile
        if (bb < D) {
            gg = bb;
        } else if (bb - D < M) {
            const uint64_t c = bb - D, d0 = c * T / M, d1 = (c + 1) * T / M;
            if (d1 > d0) {
                const FsstChunk& ch = fa.ext[fa.wg_chunk[d0]];
                if (P) fsst_decode_tile<OffAcc, LenAcc, true>(ch, d0, fa.tp, fa.bt, fa.tc, err, dec_lds(lds), tag);
                else fsst_decode_tile<OffAcc, LenAcc>(ch, d0, fa.tp, fa.bt, fa.tc, err, dec_lds(lds));
            } else {
                gg = D + c - d1;
            }
        } else {
            gg = bb - T;
        }
        if (gg != ~0ull) {
            const GenChunk& gc = gtab[ext_chunk_index_gpe(gtab, gn, gg, gpe, [](const GenChunk& d) { return d.d.first_group; })];
            gen_dispatch(int(gc.kind), gc, gg, lds, dict_off, dict_lds, err);
        }
    }
}

bool is_fsst_fused_kernel(const void* func) {
    return func == reinterpret_cast<const void*>(&fsst_k1g_kernel<PackedCol<32>, PackedCol<32>>) ||
           func == reinterpret_cast<const void*>(&fsst_k1g_kernel<PlainCol<4>, PlainCol<4>>);
}

uint64_t fsst_scratch_bytes(uint64_t n) {
    // tile prefixes + scan-block totals + tile code ends
    const uint64_t n_tiles = (n + kTS - 1) / kTS;
    return (2 * n_tiles + (n_tiles + kScanTiles - 1) / kScanTiles + 2) * sizeof(int64_t);
}

uint64_t fsst_batch_scratch_bytes(const FsstChunk* chunks, size_t n_chunks) {
    uint64_t b = 16;
    for (size_t i = 0; i < n_chunks; i++) b += fsst_scratch_bytes(chunks[i].n);
    return b;
}

namespace {

// Kernel key of a chunk: accessor kind of offsets and lengths (plain width 1/2/4/8 or packed
// T = 32/64) and, for the FastLanes lengths pre-pass, the lengths' bit width.
int acc_kind(const IntCol& c) { return c.packed ? (c.width == 4 ? 32 : 64) : c.width; }
bool fl32_lens(const IntCol& c) { return c.packed && c.width == 4 && c.offset == 0 && c.W <= 32; }
std::tuple<int, int, int> fsst_key(const FsstChunk& c) {
    return {acc_kind(c.offs), acc_kind(c.lens), fl32_lens(c.lens) ? int(c.lens.W) : -1};
}

template <int... Ws>
void launch_tile_scan_fl32(int W, dim3 grid, hipStream_t s, const FsstTable& t, int64_t* tiles, int64_t* blocks,
                           int64_t* codes, std::integer_sequence<int, Ws...>) {
    using Fn = void (*)(FsstTable, int64_t*, int64_t*, int64_t*);
    static constexpr Fn table[] = {&fsst_tile_scan_fl32<Ws, false>...};
    static constexpr Fn table_ext[] = {&fsst_tile_scan_fl32<Ws, true>...};
    hipLaunchKernelGGL((t.ext ? table_ext : table)[W], grid, dim3(kScanThreads), 0, s, t, tiles, blocks, codes);
}

// accessor = plain width 1/2/4/8 or packed T = 32/64
template <class F>
bool with_acc(int kind, F&& f) {
    switch (kind) {
    case 1: f(static_cast<PlainCol<1>*>(nullptr)); return true;
    case 2: f(static_cast<PlainCol<2>*>(nullptr)); return true;
    case 4: f(static_cast<PlainCol<4>*>(nullptr)); return true;
    case 8: f(static_cast<PlainCol<8>*>(nullptr)); return true;
    case 32: f(static_cast<PackedCol<32>*>(nullptr)); return true;
    case 64: f(static_cast<PackedCol<64>*>(nullptr)); return true;
    default: return false;
    }
}

}  // namespace

// Extra (unused) dynamic LDS per decode workgroup, VXG_FSST_PAD_LDS bytes (diagnostics: the
// occupancy sensitivity of the decode -- 16 KiB more leaves 4 instead of 8 workgroups per CU).
static size_t fsst_pad_lds() {
    static const size_t v = [] {
        const char* e = std::getenv("VXG_FSST_PAD_LDS");
        const long x = e ? std::strtol(e, nullptr, 10) : 0;
        return size_t(x > 0 && x <= 65536 ? x : 0);
    }();
    return v;
}

// Called by every vxg_open after its device is selected: the mask is parsed once per process,
// copied to each context's device (g_fsst_abl is per device).
hipError_t fsst_diag_init() {
    static const uint32_t m = [] {
        const char* e = std::getenv("VXG_FSST_ABL");
        return e ? uint32_t(std::strtoul(e, nullptr, 10)) : 0u;
    }();
    return m ? hipMemcpyToSymbol(HIP_SYMBOL(g_fsst_abl), &m, sizeof m) : hipSuccess;
}

// Accessor pairs the fused plan launch is instantiated for (the file reader's FastLanes-packed
// u32 offsets and lengths; plain u32 for arrays built in memory): each is one more copy of K1g's
// 43 job bodies.
static bool fused_acc(int oa, int la) { return (oa == 32 && la == 32) || (oa == 4 && la == 4); }

// Percentage of the K1g workgroups interleaved with the decode tiles (VXG_FUSED_MIX, 0-100,
// read once; default 100: the tiles spread over the whole grid).
static uint64_t fused_mix_pct() {
    static const uint64_t v = [] {
        const char* e = std::getenv("VXG_FUSED_MIX");
        const long x = e ? std::strtol(e, nullptr, 10) : 100;
        return uint64_t(x >= 0 && x <= 100 ? x : 100);
    }();
    return v;
}

// In-grid pre-pass of the fused launch for groups of at most VXG_FUSED_PREPASS_MAX_TILES decode
// tiles (read at every plan recording; default 8,192; 0: always the separate pre-pass kernel), and
// the K1g workgroups placed before the first decode tile (VXG_FUSED_DELAY, read once; default:
// all of them with the in-grid pre-pass -- the tiles then find their records published --, none
// without).  C5, same box, ms per step (session r06g): 8-GPU shard (2,930 tiles) 0.0434 separate
// pre-pass -> 0.0392 in-grid with the tiles last (0.0422 spread from the start); 4-GPU (5,860)
// 0.0745 -> 0.0735 (0.0803); 2-GPU (11,720) 0.1454 -> 0.1475; 1 GPU (23,443) 0.272 -> 0.280-0.288
// (not because of the device-scope record loads: plain first reads of parity-alternated record
// buffers measured the same, profiles/r06_fsst_decode.md).
static uint64_t fused_prepass_max_tiles() {
    const char* e = std::getenv("VXG_FUSED_PREPASS_MAX_TILES");
    return e ? uint64_t(std::strtoull(e, nullptr, 10)) : uint64_t(8192);
}
static int64_t fused_delay() {
    static const int64_t v = [] {
        const char* e = std::getenv("VXG_FUSED_DELAY");
        return e ? int64_t(std::strtoull(e, nullptr, 10)) : int64_t(-1);
    }();
    return v;
}

vxg_status launch_fsst_k1g(const FsstFused& fuse, const GenChunk* ext, uint32_t n, uint64_t groups, uint32_t dict_off,
                           bool dict_lds, size_t shm, uint32_t* err, hipStream_t s, uint64_t gpe) {
    if (!fuse.valid || !fused_acc(fuse.oa, fuse.la)) return set_error(VXG_ERR_INVALID_ARGUMENT, "internal: fused FSST group");
    if (n == 0) groups = 0;
    FsstFusedArgs a = fuse.a;
    a.delay = fused_delay() >= 0 ? std::min(uint64_t(fused_delay()), groups) : (a.prepass ? groups : 0);
    a.mix = a.tiles + (groups - a.delay) * fused_mix_pct() / 100;
    const uint64_t grid = a.prepass + a.tiles + groups;
    if (grid == 0) return VXG_OK;
    if (grid > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "array too long for one launch");
    shm = std::max<size_t>(shm, kDecLdsBytes + fsst_pad_lds());
    if (fuse.oa == 32)
        hipLaunchKernelGGL((fsst_k1g_kernel<PackedCol<32>, PackedCol<32>>), dim3(unsigned(grid)), dim3(kTile), shm, s, a,
                           ext, n, dict_off, dict_lds, err, gpe);
    else
        hipLaunchKernelGGL((fsst_k1g_kernel<PlainCol<4>, PlainCol<4>>), dim3(unsigned(grid)), dim3(kTile), shm, s, a, ext,
                           n, dict_off, dict_lds, err, gpe);
    return hip_check(hipGetLastError(), "fsst_k1g_kernel launch");
}

vxg_status launch_fsst_batch(std::vector<FsstChunk>& chunks, void* scratch, uint32_t* err, hipStream_t s,
                             DevTables* dt, FsstFused* fuse) {
    if (fuse) fuse->valid = false;
    for (const FsstChunk& c : chunks) {
        if (c.n_symbols > 255) return set_error(VXG_ERR_INVALID_ARGUMENT, "FSST symbol table > 255 entries");
        if ((c.n + kTS - 1) / kTS > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "FSST array too long");
        if (acc_kind(c.offs) == 0 || acc_kind(c.lens) == 0 || (c.offs.packed && c.offs.width != 4 && c.offs.width != 8) ||
            (c.lens.packed && c.lens.width != 4 && c.lens.width != 8))
            return set_error(VXG_ERR_MISMATCHED_TYPES, "FSST offsets/lengths must be 1/2/4/8-byte integers "
                                                        "(packed: 32/64-bit)");
    }
    std::stable_sort(chunks.begin(), chunks.end(),
                     [](const FsstChunk& a, const FsstChunk& b) { return fsst_key(a) < fsst_key(b); });
    int64_t* tiles_all = static_cast<int64_t*>(scratch);
    size_t i = 0;
    while (i < chunks.size()) {
        FsstTable tab{};
        uint64_t tiles = 0, scans = 0;
        // one launch pair per kernarg table of kFsstArgChunks, or (recording a plan) per
        // accessor group over a device table
        size_t j = i, live = 0;
        while (j < chunks.size() && (dt || j - i < size_t(kFsstArgChunks)) && fsst_key(chunks[j]) == fsst_key(chunks[i]))
            live += chunks[j++].n != 0;
        // the first group the fused launch covers (a device table: the fused kernel reads no kernarg table)
        const bool fusing = fuse && dt && !fuse->valid && live &&
                            fused_acc(std::get<0>(fsst_key(chunks[i])), std::get<1>(fsst_key(chunks[i])));
        uint64_t group_tiles = 0;
        for (size_t k = i; k < j; k++) group_tiles += (chunks[k].n + kTS - 1) / kTS;
        const bool ingrid = fusing && group_tiles <= fused_prepass_max_tiles();
        const uint64_t scan_tiles = ingrid ? uint64_t(kFusedScanTiles) : uint64_t(kScanTiles);
        FsstChunk* cs = tab.c;
        if (live > size_t(kFsstArgChunks) || fusing) {
            FsstChunk* host;
            const vxg_status st = dt->table(live, &host, &tab.ext);
            if (st != VXG_OK) return st;
            cs = host;
        }
        for (size_t k = i; k < j; k++) {
            if (chunks[k].n == 0) continue;
            FsstChunk& c = cs[tab.n++];
            c = chunks[k];
            const uint64_t nt = (c.n + kTS - 1) / kTS;
            c.first_tile = tiles;
            c.first_scan = scans;
            tiles += nt;
            scans += (nt + scan_tiles - 1) / scan_tiles;
        }
        if (tab.n) {
            const uint32_t* wg_chunk = nullptr;  // device table launches: chunk of every decode workgroup
            if (tab.ext) {
                uint32_t* host_map;
                const vxg_status st = dt->table(tiles, &host_map, &wg_chunk);
                if (st != VXG_OK) return st;
                for (uint32_t k = 0; k < tab.n; k++) {
                    const FsstChunk& c = cs[k];
                    const uint64_t nt = (c.n + kTS - 1) / kTS;
                    for (uint64_t t = 0; t < nt; t++) host_map[c.first_tile + t] = k;
                }
            }
            const auto key = fsst_key(cs[0]);
            if (ingrid) {  // records zeroed once (tag 0), written by the fused launch's first workgroups
                int64_t* rec_host;
                const int64_t* rec;
                uint32_t* scan_host;
                const uint32_t* scan_chunk;
                vxg_status st = dt->table(2 * tiles + scans, &rec_host, &rec);
                if (st == VXG_OK) st = dt->table(scans, &scan_host, &scan_chunk);
                if (st != VXG_OK) return st;
                for (uint32_t k = 0; k < tab.n; k++) {
                    const FsstChunk& c = cs[k];
                    const uint64_t ns = ((c.n + kTS - 1) / kTS + kFusedScanTiles - 1) / kFusedScanTiles;
                    for (uint64_t b = 0; b < ns; b++) scan_host[c.first_scan + b] = k;
                }
                int64_t* r = const_cast<int64_t*>(rec);
                fuse->valid = true;
                fuse->oa = std::get<0>(key);
                fuse->la = std::get<1>(key);
                fuse->a = FsstFusedArgs{tab.ext, r, r + tiles, r + tiles + scans, wg_chunk, tiles, tiles,
                                        scans, 0, scan_chunk, 1};
                i = j;
                continue;
            }
            int64_t* tp = tiles_all;
            int64_t* bt = tiles_all + tiles;
            int64_t* tc = bt + scans;
            tiles_all += 2 * tiles + scans;
            if (std::get<2>(key) >= 0)
                launch_tile_scan_fl32(std::get<2>(key), dim3(unsigned(scans)), s, tab, tp, bt, tc,
                                      std::make_integer_sequence<int, 33>{});
            if (fusing) {  // its pre-pass now, its decode inside the K1g launch
                if (std::get<2>(key) < 0) {
                    bool ok = with_acc(std::get<1>(key), [&](auto* la) {
                        using LA = std::remove_pointer_t<decltype(la)>;
                        hipLaunchKernelGGL((fsst_tile_scan<LA, true>), dim3(unsigned(scans)), dim3(kTile), 0, s, tab, tp,
                                           bt, tc);
                    });
                    if (!ok) return set_error(VXG_ERR_MISMATCHED_TYPES, "FSST accessor");
                }
                fuse->valid = true;
                fuse->oa = std::get<0>(key);
                fuse->la = std::get<1>(key);
                fuse->a = FsstFusedArgs{tab.ext, tp, bt, tc, wg_chunk, tiles, tiles, 0, 0, nullptr, 0};
                const vxg_status st = hip_check(hipGetLastError(), "fsst pre-pass");
                if (st != VXG_OK) return st;
                i = j;
                continue;
            }
            bool ok = true;
            with_acc(std::get<0>(key), [&](auto* oa) {
                ok = with_acc(std::get<1>(key), [&](auto* la) {
                    using OA = std::remove_pointer_t<decltype(oa)>;
                    using LA = std::remove_pointer_t<decltype(la)>;
                    auto go = [&](auto ext) {
                        constexpr bool X = decltype(ext)::value;
                        if (std::get<2>(key) < 0)
                            hipLaunchKernelGGL((fsst_tile_scan<LA, X>), dim3(unsigned(scans)), dim3(kTile), 0, s, tab,
                                               tp, bt, tc);
                        hipLaunchKernelGGL((fsst_decode<OA, LA, X>), dim3(unsigned(tiles)), dim3(kTile), fsst_pad_lds(), s,
                                           tab, tp, bt, tc, err, wg_chunk);
                    };
                    if (tab.ext) go(std::true_type{});
                    else go(std::false_type{});
                });
            });
            if (!ok) return set_error(VXG_ERR_MISMATCHED_TYPES, "FSST accessor");
            const vxg_status st = hip_check(hipGetLastError(), "fsst kernels");
            if (st != VXG_OK) return st;
        }
        i = j;
    }
    return VXG_OK;
}

}  // namespace vxg
