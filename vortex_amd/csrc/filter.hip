// filter.hip — compute::filter (compute next to the canonicalize path).
//
// Reference: vortex-array/src/compute/filter.rs:23-52 dispatches to the encoding's FilterFn;
// PrimitiveArray (primitive/compute/filter.rs:15-50), BoolArray (bool/compute/filter.rs:15-60)
// and VarBinArray (varbin/compute/filter.rs:19-200) keep the rows whose predicate bit is set, in
// order, and filter the validity the same way (validity.rs filter); FSSTArray filters its codes
// and lengths (fsst/compute.rs:147-160), so its canonical is a VarBinView over a heap of only
// the selected strings.  Encodings without a FilterFn canonicalize and filter (filter.rs:41-49).
// Whatever route the reference takes, the result is the selected rows in order; the GPU does
// it as one stream compaction:
//   1. filter_count: one wavefront per 4096-row tile (64 predicate words) -> tile true counts;
//   2. scan_tiles:   one workgroup scans the tile counts (exclusive, total at the end);
//   3. filter_values / filter_bits: each wavefront re-derives its words' output bases with a
//      wave scan, then walks its 64 words: lane l of word w moves row 64w + l to
//      base(w) + popcount(word & lanes_below(l)) — coalesced reads, contiguous writes.  Bits
//      (Bool values, validity) are packed per word with a wave OR-reduction and ORed in.
// Strings additionally rebuild the heap: lengths from the compacted views, a tile scan of them,
// then each thread copies its strings and rewrites their views (buffer 0, new offset) — the
// layout arrow-cast gives the filtered VarBin (varbin/flatten.rs:10-17, Appendix C).
#include "filter.hpp"

namespace vxg {

namespace {

constexpr int kWave = 64;
constexpr int kFilterBlock = 256;  // 4 wavefronts = 4 tiles
constexpr int kScanBlock = 1024;
constexpr int kHeapRowsPerThread = 16;  // heap kernels: 256 threads x 16 rows = one 4096-row tile

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(v), lane);
    const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(v >> 32), lane);
    return (uint64_t(hi) << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint64_t o = __shfl_up(v, d, kWave);
        if (lane >= d) v += o;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_or(uint64_t v) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) v |= __shfl_xor(v, d, kWave);
    return v;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) v += __shfl_xor(v, d, kWave);
    return v;
}

__device__ __forceinline__ uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__global__ __launch_bounds__(kFilterBlock) void filter_count_kernel(const uint64_t* __restrict__ mask, uint64_t n,
                                                                    uint64_t* __restrict__ tile_off, uint64_t tiles) {
    const int lane = threadIdx.x % kWave;
    const uint64_t t = uint64_t(blockIdx.x) * (kFilterBlock / kWave) + threadIdx.x / kWave;
    if (t >= tiles) return;
    const uint64_t nw = (n + 63) / 64, wi = t * 64 + lane;
    const uint64_t c = wi < nw ? uint64_t(__popcll(mask[wi])) : 0;
    const uint64_t sum = wave_sum(c);
    if (lane == 0) tile_off[t] = sum;
}

// Exclusive scan of a[0..n) in place, a[n] = total (one workgroup).
__global__ __launch_bounds__(kScanBlock) void scan_tiles_kernel(uint64_t* __restrict__ a, uint64_t n) {
    __shared__ uint64_t part[kScanBlock / kWave];
    const int tid = threadIdx.x, lane = tid % kWave, wv = tid / kWave;
    const uint64_t per = (n + kScanBlock - 1) / kScanBlock;
    const uint64_t lo = min(n, uint64_t(tid) * per), hi = min(n, lo + per);
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += a[i];
    const uint64_t incl = wave_incl_scan(s, lane);
    if (lane == kWave - 1) part[wv] = incl;
    __syncthreads();
    if (wv == 0) {
        const uint64_t p = lane < kScanBlock / kWave ? part[lane] : 0;
        const uint64_t pi = wave_incl_scan(p, lane);
        if (lane < kScanBlock / kWave) part[lane] = pi - p;
        if (lane == kScanBlock / kWave - 1) a[n] = pi;
    }
    __syncthreads();
    uint64_t run = part[wv] + incl - s;
    for (uint64_t i = lo; i < hi; ++i) {
        const uint64_t v = a[i];
        a[i] = run;
        run += v;
    }
}

template <int W>
struct Cell;
template <> struct Cell<1> { using T = uint8_t; };
template <> struct Cell<2> { using T = uint16_t; };
template <> struct Cell<4> { using T = uint32_t; };
template <> struct Cell<8> { using T = uint64_t; };
template <> struct Cell<16> { using T = uint4; };

// Per wavefront: the mask word of this lane and the output base of its first selected row.
struct TileWords {
    uint64_t m, base;
};

__device__ __forceinline__ TileWords tile_words(const uint64_t* __restrict__ mask, uint64_t n,
                                                const uint64_t* __restrict__ tile_off, uint64_t t, int lane) {
    const uint64_t nw = (n + 63) / 64, wi = t * 64 + lane;
    TileWords r;
    r.m = wi < nw ? mask[wi] : 0;
    const uint64_t c = uint64_t(__popcll(r.m));
    r.base = tile_off[t] + wave_incl_scan(c, lane) - c;
    return r;
}

template <int W>
__global__ __launch_bounds__(kFilterBlock) void filter_values_kernel(const uint64_t* __restrict__ mask, uint64_t n,
                                                                     const uint64_t* __restrict__ tile_off,
                                                                     const void* __restrict__ in_,
                                                                     void* __restrict__ out_, uint64_t tiles) {
    using C = typename Cell<W>::T;
    const C* __restrict__ in = static_cast<const C*>(in_);
    C* __restrict__ out = static_cast<C*>(out_);
    const int lane = threadIdx.x % kWave;
    const uint64_t t = uint64_t(blockIdx.x) * (kFilterBlock / kWave) + threadIdx.x / kWave;
    if (t >= tiles) return;
    const TileWords tw = tile_words(mask, n, tile_off, t, lane);
    const uint64_t below = lanes_below(lane);
    const uint64_t row0 = t * kFilterTileRows + uint64_t(lane);
    for (int w = 0; w < 64; ++w) {
        const uint64_t mw = readlane64(tw.m, w);
        if (mw == 0) continue;
        const uint64_t bw = readlane64(tw.base, w);
        if ((mw >> lane) & 1ull) out[bw + uint64_t(__popcll(mw & below))] = in[row0 + uint64_t(w) * 64];
    }
}

__global__ __launch_bounds__(kFilterBlock) void filter_bits_kernel(const uint64_t* __restrict__ mask, uint64_t n,
                                                                   const uint64_t* __restrict__ tile_off,
                                                                   const uint8_t* __restrict__ src,
                                                                   uint32_t* __restrict__ dst, uint64_t tiles) {
    const int lane = threadIdx.x % kWave;
    const uint64_t t = uint64_t(blockIdx.x) * (kFilterBlock / kWave) + threadIdx.x / kWave;
    if (t >= tiles) return;
    const TileWords tw = tile_words(mask, n, tile_off, t, lane);
    const uint64_t below = lanes_below(lane);
    const uint64_t row0 = t * kFilterTileRows + uint64_t(lane);
    for (int w = 0; w < 64; ++w) {
        const uint64_t mw = readlane64(tw.m, w);
        if (mw == 0) continue;
        const uint64_t bw = readlane64(tw.base, w);
        uint64_t v = 0;
        if ((mw >> lane) & 1ull) {
            const uint64_t row = row0 + uint64_t(w) * 64;
            if ((src[row >> 3] >> (row & 7)) & 1u) v = 1ull << __popcll(mw & below);
        }
        v = wave_or(v);
        if (lane == 0 && v) {
            const unsigned sh = unsigned(bw & 31);
            uint32_t* d = dst + (bw >> 5);
            const uint32_t p0 = uint32_t(v << sh);
            const uint32_t p1 = uint32_t(v >> (32 - sh));
            const uint32_t p2 = sh ? uint32_t(v >> (64 - sh)) : 0u;
            if (p0) atomicOr(d, p0);
            if (p1) atomicOr(d + 1, p1);
            if (p2) atomicOr(d + 2, p2);
        }
    }
}

// Length of view i; a null row (validity bit clear) keeps no bytes: VarBin's filter appends
// nulls as empty values (varbin/compute/filter.rs:153-200), so its view is all zeros.
__device__ __forceinline__ uint32_t view_len(const uint8_t* views, const uint8_t* valid, uint64_t i) {
    if (valid && !((valid[i >> 3] >> (i & 7)) & 1u)) return 0;
    return *reinterpret_cast<const uint32_t*>(views + 16 * i);
}

__global__ __launch_bounds__(kFilterBlock) void heap_sizes_kernel(const uint8_t* __restrict__ views, uint64_t n,
                                                                  const uint8_t* __restrict__ valid,
                                                                  uint64_t* __restrict__ heap_off) {
    __shared__ uint64_t part[kFilterBlock / kWave];
    const int tid = threadIdx.x, lane = tid % kWave;
    const uint64_t r0 = uint64_t(blockIdx.x) * kFilterTileRows + uint64_t(tid) * kHeapRowsPerThread;
    uint64_t s = 0;
    for (int k = 0; k < kHeapRowsPerThread; ++k)
        if (r0 + k < n) s += view_len(views, valid, r0 + k);
    s = wave_sum(s);
    if (lane == 0) part[tid / kWave] = s;
    __syncthreads();
    if (tid == 0) {
        uint64_t tot = 0;
        for (int i = 0; i < kFilterBlock / kWave; ++i) tot += part[i];
        heap_off[blockIdx.x] = tot;
    }
}

__global__ __launch_bounds__(kFilterBlock) void heap_build_kernel(uint8_t* __restrict__ views, uint64_t n,
                                                                  const uint8_t* __restrict__ valid,
                                                                  const uint64_t* __restrict__ heap_off,
                                                                  const uint8_t* const* __restrict__ bufs,
                                                                  uint32_t n_bufs, uint8_t* __restrict__ heap,
                                                                  uint32_t* __restrict__ err) {
    __shared__ uint64_t part[kFilterBlock / kWave];
    const int tid = threadIdx.x, lane = tid % kWave, wv = tid / kWave;
    const uint64_t r0 = uint64_t(blockIdx.x) * kFilterTileRows + uint64_t(tid) * kHeapRowsPerThread;
    uint64_t s = 0;
    for (int k = 0; k < kHeapRowsPerThread; ++k)
        if (r0 + k < n) s += view_len(views, valid, r0 + k);
    const uint64_t incl = wave_incl_scan(s, lane);
    if (lane == kWave - 1) part[wv] = incl;
    __syncthreads();
    uint64_t off = heap_off[blockIdx.x] + incl - s;
    for (int i = 0; i < wv; ++i) off += part[i];
    bool bad = false;
    for (int k = 0; k < kHeapRowsPerThread; ++k) {
        const uint64_t r = r0 + k;
        if (r >= n) break;
        uint32_t* v = reinterpret_cast<uint32_t*>(views + 16 * r);
        const uint32_t len = view_len(views, valid, r);
        if (len == 0) {
            v[0] = v[1] = v[2] = v[3] = 0u;
        } else if (len <= 12) {
            const uint8_t* b = reinterpret_cast<const uint8_t*>(v) + 4;
            for (uint32_t j = 0; j < len; ++j) heap[off + j] = b[j];
        } else {
            const uint32_t bi = v[2];
            if (bi >= n_bufs) {
                bad = true;
            } else {
                const uint8_t* b = bufs[bi] + v[3];
                for (uint32_t j = 0; j < len; ++j) heap[off + j] = b[j];
            }
            v[2] = 0;
            v[3] = uint32_t(off);
        }
        off += len;
    }
    if (bad) __hip_atomic_fetch_or(err, kErrTakeOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

unsigned grid_for_tiles(uint64_t tiles) { return unsigned((tiles + 3) / 4); }

}  // namespace

vxg_status launch_filter_count(const uint64_t* mask, uint64_t n, uint64_t* tile_off, hipStream_t s) {
    const uint64_t tiles = filter_tiles(n);
    if (tiles) {
        if (grid_for_tiles(tiles) > 0x7FFFFFFFu) return set_error(VXG_ERR_INVALID_ARGUMENT, "filter: array too long");
        hipLaunchKernelGGL(filter_count_kernel, dim3(grid_for_tiles(tiles)), dim3(kFilterBlock), 0, s, mask, n,
                           tile_off, tiles);
        if (vxg_status st = hip_check(hipGetLastError(), "filter_count_kernel"); st != VXG_OK) return st;
    }
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(kScanBlock), 0, s, tile_off, tiles);
    return hip_check(hipGetLastError(), "scan_tiles_kernel");
}

vxg_status launch_filter_values(const uint64_t* mask, uint64_t n, const uint64_t* tile_off, const void* in, int width,
                                void* out, hipStream_t s) {
    const uint64_t tiles = filter_tiles(n);
    if (!tiles) return VXG_OK;
    const dim3 g(grid_for_tiles(tiles)), b(kFilterBlock);
    switch (width) {
    case 1: hipLaunchKernelGGL(filter_values_kernel<1>, g, b, 0, s, mask, n, tile_off, in, out, tiles); break;
    case 2: hipLaunchKernelGGL(filter_values_kernel<2>, g, b, 0, s, mask, n, tile_off, in, out, tiles); break;
    case 4: hipLaunchKernelGGL(filter_values_kernel<4>, g, b, 0, s, mask, n, tile_off, in, out, tiles); break;
    case 8: hipLaunchKernelGGL(filter_values_kernel<8>, g, b, 0, s, mask, n, tile_off, in, out, tiles); break;
    case 16: hipLaunchKernelGGL(filter_values_kernel<16>, g, b, 0, s, mask, n, tile_off, in, out, tiles); break;
    default: return set_error(VXG_ERR_INVALID_ARGUMENT, "filter: unsupported value width");
    }
    return hip_check(hipGetLastError(), "filter_values_kernel");
}

vxg_status launch_filter_bits(const uint64_t* mask, uint64_t n, const uint64_t* tile_off, const uint8_t* src,
                              void* dst, hipStream_t s) {
    const uint64_t tiles = filter_tiles(n);
    if (!tiles) return VXG_OK;
    hipLaunchKernelGGL(filter_bits_kernel, dim3(grid_for_tiles(tiles)), dim3(kFilterBlock), 0, s, mask, n, tile_off,
                       src, static_cast<uint32_t*>(dst), tiles);
    return hip_check(hipGetLastError(), "filter_bits_kernel");
}

vxg_status launch_view_heap_sizes(const uint8_t* views, uint64_t n, const uint8_t* valid, uint64_t* heap_off,
                                  hipStream_t s) {
    const uint64_t tiles = filter_tiles(n);
    if (tiles) {
        if (tiles > 0x7FFFFFFFu) return set_error(VXG_ERR_INVALID_ARGUMENT, "filter: array too long");
        hipLaunchKernelGGL(heap_sizes_kernel, dim3(unsigned(tiles)), dim3(kFilterBlock), 0, s, views, n, valid, heap_off);
        if (vxg_status st = hip_check(hipGetLastError(), "heap_sizes_kernel"); st != VXG_OK) return st;
    }
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(kScanBlock), 0, s, heap_off, tiles);
    return hip_check(hipGetLastError(), "scan_tiles_kernel");
}

vxg_status launch_view_heap_build(uint8_t* views, uint64_t n, const uint8_t* valid, const uint64_t* heap_off,
                                  const uint8_t* const* bufs,
                                  uint32_t n_bufs, uint8_t* heap, uint32_t* err, hipStream_t s) {
    const uint64_t tiles = filter_tiles(n);
    if (!tiles) return VXG_OK;
    hipLaunchKernelGGL(heap_build_kernel, dim3(unsigned(tiles)), dim3(kFilterBlock), 0, s, views, n, valid, heap_off, bufs,
                       n_bufs, heap, err);
    return hip_check(hipGetLastError(), "heap_build_kernel");
}

}  // namespace vxg
