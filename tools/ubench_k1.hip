// ubench_k1.hip — A/B variants of the FastLanes unpack kernel on the C1 shape
// (u32, W=7, 64 Mi values), timed interleaved in one process (cdna_hip_programming.md §5.4
// rule 24).  Inputs rotate over 8 copies (470 MB > the 256 MiB Infinity Cache) so every launch
// reads HBM; `./ubench_k1 flush` also writes a 512 MiB buffer between timed launches.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/ubench_k1.hip -o tools/ubench_k1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../vortex_amd/csrc/fl_unpack_impl.hpp"

namespace vxg {
vxg_status set_error(vxg_status s, const std::string&) { return s; }
vxg_status hip_check(hipError_t e, const char*) { return e == hipSuccess ? VXG_OK : VXG_ERR_HIP; }
}  // namespace vxg

using namespace vxg;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int T = 32, W = 7;

// the engine's K1 path today: 32 blocks per 256-thread workgroup, one block per 8 threads
template <int NT>
__global__ __launch_bounds__(256) void k_base(const uint8_t* __restrict__ packed, uint32_t* __restrict__ out,
                                              uint64_t n_blocks) {
    const uint64_t gid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t blk = gid >> 3;
    if (blk >= n_blocks) return;
    EpiParams ep{};
    unpack_block<T, W, Epi::Plain, 0, NT>(packed + blk * (128 * W), int(gid & 7), out, int64_t(blk * 1024), true,
                                          n_blocks * 1024, ep);
}

// persistent + software-pipelined: each 8-thread group walks blocks g, g+G, ...; the next
// block's packed words are loaded BEFORE the current block's 32 stores are issued, so every
// wave keeps HBM reads in flight while it writes.
template <int NT>
__global__ __launch_bounds__(256) void k_pipe(const uint8_t* __restrict__ packed, uint32_t* __restrict__ out,
                                              uint64_t n_blocks) {
    const int t = int(threadIdx.x & 7);
    const uint64_t ngrp = uint64_t(gridDim.x) * 32;
    uint64_t blk = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 3;
    if (blk >= n_blocks) return;
    Vec16<T> cur[W], nxt[W];
#pragma unroll
    for (int w = 0; w < W; w++) cur[w] = load16<T>(packed + blk * (128 * W) + 128 * w + 16 * t);
    EpiParams ep{};
    bool oob = false;
    for (;;) {
        const uint64_t nb = blk + ngrp;
        const bool more = nb < n_blocks;
        if (more) {
#pragma unroll
            for (int w = 0; w < W; w++) nxt[w] = load16<T>(packed + nb * (128 * W) + 128 * w + 16 * t);
        }
        process_rows<T, W, Epi::Plain, 0, NT, true>(cur, t * 4, out, int64_t(blk * 1024), n_blocks * 1024, ep, oob,
                                                    std::make_integer_sequence<int, T>{});
        if (!more) break;
#pragma unroll
        for (int w = 0; w < W; w++) cur[w] = nxt[w];
        blk = nb;
    }
}

// row split S=2: 16 threads per block, each takes half of the rows (only the word rows those
// rows read are loaded) -> 2x the waves, half the stores per wave
template <int NT, int S>
__global__ __launch_bounds__(256) void k_split(const uint8_t* __restrict__ packed, uint32_t* __restrict__ out,
                                               uint64_t n_blocks) {
    constexpr int BPG = 32 / S;
    const uint64_t blk = uint64_t(blockIdx.x) * BPG + ((threadIdx.x >> 3) % BPG);
    const int t = int(threadIdx.x & 7);
    if (blk >= n_blocks) return;
    EpiParams ep{};
    const uint8_t* bp = packed + blk * (128 * W);
    if constexpr (S == 2) {
        if ((threadIdx.x >> 7) == 0) unpack_block_part<T, W, Epi::Plain, 0, NT, 2, 0>(bp, t, out, int64_t(blk * 1024), true, n_blocks * 1024, ep);
        else unpack_block_part<T, W, Epi::Plain, 0, NT, 2, 1>(bp, t, out, int64_t(blk * 1024), true, n_blocks * 1024, ep);
    } else {
        switch (threadIdx.x >> 6) {
        case 0: unpack_block_part<T, W, Epi::Plain, 0, NT, 4, 0>(bp, t, out, int64_t(blk * 1024), true, n_blocks * 1024, ep); break;
        case 1: unpack_block_part<T, W, Epi::Plain, 0, NT, 4, 1>(bp, t, out, int64_t(blk * 1024), true, n_blocks * 1024, ep); break;
        case 2: unpack_block_part<T, W, Epi::Plain, 0, NT, 4, 2>(bp, t, out, int64_t(blk * 1024), true, n_blocks * 1024, ep); break;
        default: unpack_block_part<T, W, Epi::Plain, 0, NT, 4, 3>(bp, t, out, int64_t(blk * 1024), true, n_blocks * 1024, ep); break;
        }
    }
}


// transposed stores: each lane group decodes its block's rows phase by phase (a phase = the
// 8 rows that make up 1 KiB of the block), parks them in LDS, and the wave then writes every
// block's 1 KiB with ONE fully contiguous 1 KiB store instruction (64 lanes x 16 B).
template <int NT, int P, int R>
__device__ __forceinline__ void tr_row(const Vec16<T>* p, int t, uint8_t* lds_j) {
    constexpr int off = fl_index(R, 0) * 4;
    if constexpr (off / 1024 == P) {
        const Vec16<T> v = extract_row<T, W, R>(p);
        uint4 q;
        __builtin_memcpy(&q, v.w, 16);
        *reinterpret_cast<uint4*>(lds_j + (off - 1024 * P) + 16 * t) = q;
    }
}
template <int NT, int P, int... Rs>
__device__ __forceinline__ void tr_phase(const Vec16<T>* p, int t, uint8_t* lds_w, int j, int lane,
                                         uint8_t* out_w, std::integer_sequence<int, Rs...>) {
    (tr_row<NT, P, Rs>(p, t, lds_w + j * 1024), ...);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int m = 0; m < 8; m++) {
        uint4 q = *reinterpret_cast<const uint4*>(lds_w + m * 1024 + 16 * lane);
        store_bytes<16, NT>(out_w + size_t(m) * 4096 + 1024 * P + 16 * lane, &q);
    }
    __builtin_amdgcn_wave_barrier();
}
template <int NT>
__global__ __launch_bounds__(256) void k_tr(const uint8_t* __restrict__ packed, uint32_t* __restrict__ out,
                                            uint64_t n_blocks) {
    __shared__ __attribute__((aligned(16))) uint8_t s_tr[4 * 8 * 1024];
    const uint64_t gid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t blk = gid >> 3;
    const int t = int(gid & 7), lane = int(threadIdx.x & 63), j = lane >> 3;
    if (blk >= n_blocks) return;
    Vec16<T> p[W];
#pragma unroll
    for (int w = 0; w < W; w++) p[w] = load16<T>(packed + blk * (128 * W) + 128 * w + 16 * t);
    uint8_t* lds_w = s_tr + (threadIdx.x >> 6) * 8192;
    uint8_t* out_w = reinterpret_cast<uint8_t*>(out) + (gid >> 6) * 8 * 4096;
    tr_phase<NT, 0>(p, t, lds_w, j, lane, out_w, std::make_integer_sequence<int, T>{});
    tr_phase<NT, 1>(p, t, lds_w, j, lane, out_w, std::make_integer_sequence<int, T>{});
    tr_phase<NT, 2>(p, t, lds_w, j, lane, out_w, std::make_integer_sequence<int, T>{});
    tr_phase<NT, 3>(p, t, lds_w, j, lane, out_w, std::make_integer_sequence<int, T>{});
}


// rows in memory order (increasing fl_index offset): each lane group writes its block front to back
template <int R> struct MemRow {
    // the R-th row in memory order for T=32: group g = R/4, position p = R%4 -> row q*8+g, q = [0,2,1,3][p]
    static constexpr int q = (R % 4 == 1) ? 2 : (R % 4 == 2) ? 1 : (R % 4);
    static constexpr int row = q * 8 + R / 4;
};
template <int NT, int... Rs>
__device__ __forceinline__ void rows_memorder(const Vec16<T>* p, int lane0, uint32_t* out, int64_t base,
                                              std::integer_sequence<int, Rs...>) {
    EpiParams ep{};
    bool oob = false;
    (process_row<T, W, Epi::Plain, 0, NT, MemRow<Rs>::row, true>(p, lane0, out, base, 1ull << 40, ep, oob), ...);
}
// XM: XCD-aware workgroup order (workgroup g runs on XCD g % 8: give each XCD a contiguous range)
template <int NT, bool MEMORD, bool XM>
__global__ __launch_bounds__(256) void k_ord(const uint8_t* __restrict__ packed, uint32_t* __restrict__ out,
                                             uint64_t n_blocks) {
    uint64_t g = blockIdx.x;
    if constexpr (XM) g = (g % 8) * (gridDim.x / 8) + g / 8;
    const uint64_t blk = g * 32 + (threadIdx.x >> 3);
    const int t = int(threadIdx.x & 7);
    if (blk >= n_blocks) return;
    Vec16<T> p[W];
#pragma unroll
    for (int w = 0; w < W; w++) p[w] = load16<T>(packed + blk * (128 * W) + 128 * w + 16 * t);
    if constexpr (MEMORD) {
        rows_memorder<NT>(p, t * 4, out, int64_t(blk * 1024), std::make_integer_sequence<int, T>{});
    } else {
        EpiParams ep{};
        bool oob = false;
        process_rows<T, W, Epi::Plain, 0, NT, true>(p, t * 4, out, int64_t(blk * 1024), 1ull << 40, ep, oob,
                                                    std::make_integer_sequence<int, T>{});
    }
}
// persistent pipelined copy of the same bytes: each wave loads its next 7 KiB while storing
// the current 32 KiB (1 KiB per instruction)
template <int NT>
__global__ __launch_bounds__(256) void k_copy_pipe(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                   uint64_t n_blocks) {
    const uint64_t nw = uint64_t(gridDim.x) * 4;
    uint64_t wave = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const int lane = int(threadIdx.x & 63);
    const uint64_t n_units = n_blocks / 8;
    if (wave >= n_units) return;
    uint4 r[7], nx[7];
#pragma unroll
    for (int k = 0; k < 7; k++) r[k] = in[wave * 448 + k * 64 + lane];
    for (;;) {
        const uint64_t nwv = wave + nw;
        const bool more = nwv < n_units;
        if (more) {
#pragma unroll
            for (int k = 0; k < 7; k++) nx[k] = in[nwv * 448 + k * 64 + lane];
        }
        uint4 acc = r[0];
#pragma unroll
        for (int k = 1; k < 7; k++) { acc.x ^= r[k].x; acc.y ^= r[k].y; }
        uint4* dst = out + wave * 2048;
#pragma unroll
        for (int k = 0; k < 32; k++) {
            uint4 v = make_uint4(acc.x + k, acc.y, acc.z, acc.w);
            store_bytes<16, NT>(reinterpret_cast<uint8_t*>(dst + k * 64 + lane), &v);
        }
        if (!more) break;
#pragma unroll
        for (int k = 0; k < 7; k++) r[k] = nx[k];
        wave = nwv;
    }
}

// Roofline reference with the same bytes: each thread reads 7 x 16 B and writes 32 x 16 B,
// every wave-instruction fully contiguous (1 KiB).
template <int NT>
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n_blocks) {
    const uint64_t gid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t wave = gid >> 6;
    const int lane = int(gid & 63);
    if (wave * 8 >= n_blocks) return;
    const uint4* src = in + wave * 448;
    uint4* dst = out + wave * 2048;
    uint4 acc = make_uint4(0, 0, 0, 0);
    uint4 r[7];
#pragma unroll
    for (int k = 0; k < 7; k++) r[k] = src[k * 64 + lane];
#pragma unroll
    for (int k = 0; k < 7; k++) { acc.x ^= r[k].x; acc.y ^= r[k].y; acc.z ^= r[k].z; acc.w ^= r[k].w; }
#pragma unroll
    for (int k = 0; k < 32; k++) {
        uint4 v = make_uint4(acc.x + k, acc.y, acc.z, acc.w);
        if constexpr (NT) {
            using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
            u32x4 vv;
            __builtin_memcpy(&vv, &v, 16);
            __builtin_nontemporal_store(vv, reinterpret_cast<u32x4*>(dst + k * 64 + lane));
        } else {
            dst[k * 64 + lane] = v;
        }
    }
}

// burst copy reference: a workgroup reads its 32 blocks' packed bytes (28 KiB) into LDS in one
// burst, then writes its 128 KiB of output, each wave 32 KiB with 1 KiB contiguous instructions
// (plain or NT stores) -- do phase-separated reads and writes beat interleaved ones?
template <int NT, int NTL = 0>
__global__ __launch_bounds__(256) void k_burst(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n_blocks) {
    __shared__ uint4 s_in[32 * 56];  // 32 blocks x 896 B
    const uint64_t b0 = uint64_t(blockIdx.x) * 32;
    if (b0 >= n_blocks) return;
    const uint4* src = in + b0 * 56;
    for (int q = threadIdx.x; q < 32 * 56; q += 256) {
        if constexpr (NTL) {  // non-temporal loads (read once)
            using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
            const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + q);
            s_in[q] = make_uint4(v[0], v[1], v[2], v[3]);
        } else {
            s_in[q] = src[q];
        }
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint4 acc = s_in[wave * 448 + lane];
    uint4* dst = out + (b0 + wave * 8) * 256;
#pragma unroll
    for (int k = 0; k < 32; k++) {
        uint4 v = make_uint4(acc.x + k, acc.y, acc.z, acc.w);
        store_bytes<16, NT>(reinterpret_cast<uint8_t*>(dst + k * 64 + lane), &v);
    }
}

// Pipelined burst copy: persistent workgroups, two LDS buffers; the next group's input is requested
// with LDS-DMA (global_load_lds_dwordx4: no VGPRs) BEFORE the current group's stores, and waited for
// with a counted vmcnt (the stores issued after it may stay in flight) and a raw s_barrier.
template <int NT, int BPG>
__global__ __launch_bounds__(256) void k_burst_pipe(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                    uint64_t n_blocks) {
    constexpr int Q = BPG * 56;      // uint4 per group (BPG blocks x 896 B)
    constexpr int J = (Q + 255) / 256;  // DMA rounds per group (a wave-uniform guard on the last)
    static_assert(Q % 64 == 0, "group must be a whole number of 1 KiB wave DMAs");
    constexpr int ST = BPG * 256 / 64 / 4;  // 1 KiB stores per wave per group
    __shared__ __attribute__((aligned(16))) uint4 s_in[2][Q];
    const uint64_t n_groups = n_blocks / BPG;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint64_t g = blockIdx.x;
    auto dma = [&](uint64_t grp, int b) {
        // inline-asm LDS-DMA (cdna_hip_programming.md: hipcc does not count asm memory ops, so it
        // inserts no vmcnt(0) before the next ds_read of the OTHER buffer; the waits below are ours)
        const uint4* src = in + grp * Q;
#pragma unroll
        for (int j = 0; j < J; j++) {
            const int q = j * 256 + wave * 64;
            if (q < Q) {
                const uint32_t lds_dst = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(&s_in[b][q])));
                const uint4* gsrc = src + q + lane;
                unsigned keep;
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                             : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
            }
        }
    };
    if (g < n_groups) dma(g, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (no stores yet: the counted wait below would not wait)
    int b = 0;
    for (; g < n_groups; g += gridDim.x) {
        // this group's DMA was issued before the previous group's ST stores: wait for it only
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ST) : "memory");
        __builtin_amdgcn_s_barrier();
        const uint64_t gn = g + gridDim.x;
        if (gn < n_groups) dma(gn, b ^ 1);
        const uint4 acc = s_in[b][wave * (Q / 4) + lane];
        uint4* dst = out + (g * BPG + wave * (BPG / 4)) * 256;
#pragma unroll
        for (int k = 0; k < ST; k++) {
            uint4 v = make_uint4(acc.x + k, acc.y, acc.z, acc.w);
            store_bytes<16, NT>(reinterpret_cast<uint8_t*>(dst + k * 64 + lane), &v);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave is done reading buffer b before it is refilled
        b ^= 1;
    }
}

// K1 with burst reads + wave-contiguous stores: the workgroup reads its 32 blocks' packed bytes
// into LDS in one burst; then every wave decodes whole blocks, all 64 lanes on one block: in
// store k, lane group g (8 lanes) produces the row whose 128 output bytes sit at k*1 KiB + g*128
// of the block, lane t its 16-byte slice -- so each store instruction writes 1 KiB contiguous.
// The row index (hence the shift) is lane-dependent: runtime shifts on words read from LDS.
__device__ __forceinline__ int inv_row32(int seg128) {
    // byte offset of row r (T=32) = FL_ORDER[r/8]*64 + (r%8)*512 -> inverse over 128-B slots
    const int s = seg128 >> 2, q = seg128 & 3;        // 512-B segment s, 128-B quarter q
    const int o = (q == 0) ? 0 : (q == 1) ? 2 : (q == 2) ? 1 : 3;  // FL_ORDER[o]*64/128 == q
    return o * 8 + s;
}
template <int NT>
__global__ __launch_bounds__(256) void k_lds(const uint8_t* __restrict__ packed, uint32_t* __restrict__ out,
                                             uint64_t n_blocks) {
    constexpr int BPW = 32;
    __shared__ __attribute__((aligned(16))) uint8_t s_in[BPW * 128 * W];
    const uint64_t b0 = uint64_t(blockIdx.x) * BPW;
    if (b0 >= n_blocks) return;
    const uint4* src = reinterpret_cast<const uint4*>(packed + b0 * (128 * W));
    for (int q = threadIdx.x; q < BPW * 8 * W; q += 256) reinterpret_cast<uint4*>(s_in)[q] = src[q];
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 3, t = lane & 7;
    for (int b = wave; b < BPW; b += 4) {
        const uint8_t* blk = s_in + b * 128 * W;
        uint8_t* dst = reinterpret_cast<uint8_t*>(out) + (b0 + b) * 4096;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int r = inv_row32(k * 8 + g);
            const int start = r * W, w0 = start >> 5, sh = start & 31;
            const uint4 lo = *reinterpret_cast<const uint4*>(blk + w0 * 128 + 16 * t);
            uint4 v;
            const uint32_t m = (1u << W) - 1u;
            if (sh + W <= 32) {
                v = make_uint4((lo.x >> sh) & m, (lo.y >> sh) & m, (lo.z >> sh) & m, (lo.w >> sh) & m);
            } else {
                const uint4 hi = *reinterpret_cast<const uint4*>(blk + (w0 + 1) * 128 + 16 * t);
                const int c = 32 - sh;
                v = make_uint4(((lo.x >> sh) | (hi.x << c)) & m, ((lo.y >> sh) | (hi.y << c)) & m,
                               ((lo.z >> sh) | (hi.z << c)) & m, ((lo.w >> sh) | (hi.w << c)) & m);
            }
            store_bytes<16, NT>(dst + k * 1024 + 16 * lane, &v);
        }
    }
}

// lds2: as k_lds, but each wave decodes 8 CONSECUTIVE blocks (32 KiB of contiguous output per
// wave, like the burst copy) and the row extraction is branch-free: both words are always read
// and funnel-shifted (v_alignbit), the per-lane row parameters computed once.
template <int NT, int BPW = 32>
__global__ __launch_bounds__(256) void k_lds2(const uint8_t* __restrict__ packed, uint32_t* __restrict__ out,
                                              uint64_t n_blocks) {
    __shared__ __attribute__((aligned(16))) uint8_t s_in[BPW * 128 * W + 128];
    const uint64_t b0 = uint64_t(blockIdx.x) * BPW;
    if (b0 >= n_blocks) return;
    const uint4* src = reinterpret_cast<const uint4*>(packed + b0 * (128 * W));
    for (int q = threadIdx.x; q < BPW * 8 * W; q += 256) reinterpret_cast<uint4*>(s_in)[q] = src[q];
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 3, t = lane & 7;
    int off0[4], sh[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int r = inv_row32(k * 8 + g), start = r * W;
        off0[k] = (start >> 5) * 128 + 16 * t;
        sh[k] = start & 31;
    }
    const uint32_t m = (1u << W) - 1u;
#pragma unroll 2
    for (int j = 0; j < BPW / 4; j++) {
        const int b = wave * (BPW / 4) + j;
        const uint8_t* blk = s_in + b * 128 * W;
        uint8_t* dst = reinterpret_cast<uint8_t*>(out) + (b0 + b) * 4096;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 lo = *reinterpret_cast<const uint4*>(blk + off0[k]);
            const uint4 hi = *reinterpret_cast<const uint4*>(blk + off0[k] + 128);
            const uint32_t c = uint32_t(sh[k]);
            uint4 v;
            v.x = __builtin_amdgcn_alignbit(hi.x, lo.x, c) & m;
            v.y = __builtin_amdgcn_alignbit(hi.y, lo.y, c) & m;
            v.z = __builtin_amdgcn_alignbit(hi.z, lo.z, c) & m;
            v.w = __builtin_amdgcn_alignbit(hi.w, lo.w, c) & m;
            store_bytes<16, NT>(dst + k * 1024 + 16 * lane, &v);
        }
    }
}

// lds_k1: burst read into LDS, then the engine's K1 decode (8 threads per block, compile-time
// row extraction, K1 store shape) with the packed words read from LDS instead of HBM
template <int NT>
__global__ __launch_bounds__(256) void k_lds_k1(const uint8_t* __restrict__ packed, uint32_t* __restrict__ out,
                                                uint64_t n_blocks) {
    constexpr int BPW = 32;
    __shared__ __attribute__((aligned(16))) uint8_t s_in[BPW * 128 * W];
    const uint64_t b0 = uint64_t(blockIdx.x) * BPW;
    if (b0 >= n_blocks) return;
    const uint4* src = reinterpret_cast<const uint4*>(packed + b0 * (128 * W));
    for (int q = threadIdx.x; q < BPW * 8 * W; q += 256) reinterpret_cast<uint4*>(s_in)[q] = src[q];
    __syncthreads();
    const int b = threadIdx.x >> 3, t = threadIdx.x & 7;
    Vec16<T> p[W];
#pragma unroll
    for (int w = 0; w < W; w++) p[w] = load16<T>(s_in + b * 128 * W + 128 * w + 16 * t);
    EpiParams ep{};
    bool oob = false;
    process_rows<T, W, Epi::Plain, 0, NT, true>(p, t * 4, out, int64_t((b0 + b) * 1024), 1ull << 40, ep, oob,
                                                std::make_integer_sequence<int, T>{});
}

// write-only, wave-contiguous: each wave writes 32 KiB, 1 KiB per instruction, plain stores
__global__ __launch_bounds__(256) void k_write_wave(uint4* __restrict__ out, uint64_t n16) {
    const uint64_t wave = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wave * 2048 >= n16) return;
#pragma unroll
    for (int k = 0; k < 32; k++) out[wave * 2048 + k * 64 + lane] = make_uint4(unsigned(k), 1u, 2u, 3u);
}

// write-only reference: 268 MB of NT stores, nothing read
__global__ __launch_bounds__(256) void k_write(uint4* __restrict__ out, uint64_t n16) {
    using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
        u32x4 v = {unsigned(i), 1u, 2u, 3u};
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + i));
    }
}

__global__ void fill_rand(uint32_t* p, uint64_t n, uint32_t seed) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint32_t x = uint32_t(i) * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = x;
    }
}

int main(int argc, char** argv) {
    const bool flush = argc > 1 && std::strcmp(argv[1], "flush") == 0;
    const uint64_t n_vals = 64ull << 20, n_blocks = n_vals / 1024;
    const uint64_t in_bytes = n_blocks * 128 * W, out_bytes = n_vals * 4;
    const int copies = 8;
    std::vector<uint8_t*> in(copies);
    for (int c = 0; c < copies; c++) {
        CK(hipMalloc(&in[c], in_bytes));
        hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, (uint32_t*)in[c], in_bytes / 4, 1234u + c);
    }
    uint32_t *out, *ref;
    uint8_t* junk = nullptr;
    CK(hipMalloc(&out, out_bytes));
    CK(hipMalloc(&ref, out_bytes));
    if (flush) CK(hipMalloc(&junk, 512ull << 20));
    CK(hipDeviceSynchronize());
    const unsigned grid_base = unsigned(n_blocks * 8 / 256);
    hipLaunchKernelGGL(k_base<0>, dim3(grid_base), dim3(256), 0, 0, in[0], ref, n_blocks);
    CK(hipDeviceSynchronize());
    int cus = 256;
    {
        hipDeviceProp_t p;
        CK(hipGetDeviceProperties(&p, 0));
        cus = p.multiProcessorCount;
    }

    struct Var { const char* name; int id; };
    std::vector<Var> vars_all = {{"base_nt", 1}, {"pipe_nt_x2", 2}, {"pipe_nt_x4", 3}, {"pipe_nt_x8", 4},
                             {"split2_nt", 5}, {"split4_nt", 6}, {"copy_ref_nt", 7}, {"write_only_nt", 8},
                             {"base_plain", 11}, {"copy_ref_plain", 12},
                             {"memord_nt", 13}, {"memord_plain", 14}, {"xcd_nt", 15}, {"xcd_memord_nt", 16},
                             {"copy_pipe_x4_plain", 17}, {"copy_pipe_x8_plain", 18}, {"copy_pipe_x8_nt", 19},
                             {"tr_plain", 9}, {"tr_nt", 10}, {"burst_plain", 20}, {"burst_nt", 21},
                             {"write_wave_plain", 22}, {"lds_plain", 23}, {"lds_nt", 24},
                             {"lds2_plain", 25}, {"lds2_nt", 26}, {"lds_k1_plain", 27}, {"lds_k1_nt", 28},
                             {"lds2_nt_bpw16", 29}, {"lds2_nt_bpw64", 30}, {"lds2_nt_bpw8", 31},
                             {"bpipe32_nt_x2", 32}, {"bpipe16_nt_x4", 33}, {"bpipe16_nt_x3", 34}, {"bpipe32_plain_x2", 35},
                             {"bpipe16_plain_x4", 36}, {"burst_nt_ntload", 37}};
    std::vector<Var> vars;
    for (auto& v : vars_all)
        if (std::getenv("UB_ALL") || v.id == 1 || v.id == 7 || v.id == 20 || v.id == 21 || v.id == 22 || v.id >= 25)
            vars.push_back(v);
    auto launch = [&](int id, const uint8_t* src) {
        switch (id) {
        case 1: hipLaunchKernelGGL(k_base<1>, dim3(grid_base), dim3(256), 0, 0, src, out, n_blocks); break;
        case 2: hipLaunchKernelGGL(k_pipe<1>, dim3(cus * 2), dim3(256), 0, 0, src, out, n_blocks); break;
        case 3: hipLaunchKernelGGL(k_pipe<1>, dim3(cus * 4), dim3(256), 0, 0, src, out, n_blocks); break;
        case 4: hipLaunchKernelGGL(k_pipe<1>, dim3(cus * 8), dim3(256), 0, 0, src, out, n_blocks); break;
        case 5: hipLaunchKernelGGL((k_split<1, 2>), dim3(unsigned(n_blocks / 16)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 6: hipLaunchKernelGGL((k_split<1, 4>), dim3(unsigned(n_blocks / 8)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 7: hipLaunchKernelGGL(k_copy<1>, dim3(unsigned(n_blocks / 8 * 64 / 256)), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 9: hipLaunchKernelGGL(k_tr<0>, dim3(grid_base), dim3(256), 0, 0, src, out, n_blocks); break;
        case 10: hipLaunchKernelGGL(k_tr<1>, dim3(grid_base), dim3(256), 0, 0, src, out, n_blocks); break;
        case 11: hipLaunchKernelGGL(k_base<0>, dim3(grid_base), dim3(256), 0, 0, src, out, n_blocks); break;
        case 12: hipLaunchKernelGGL(k_copy<0>, dim3(unsigned(n_blocks / 8 * 64 / 256)), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 13: hipLaunchKernelGGL((k_ord<1, true, false>), dim3(grid_base), dim3(256), 0, 0, src, out, n_blocks); break;
        case 14: hipLaunchKernelGGL((k_ord<0, true, false>), dim3(grid_base), dim3(256), 0, 0, src, out, n_blocks); break;
        case 15: hipLaunchKernelGGL((k_ord<1, false, true>), dim3(grid_base), dim3(256), 0, 0, src, out, n_blocks); break;
        case 16: hipLaunchKernelGGL((k_ord<1, true, true>), dim3(grid_base), dim3(256), 0, 0, src, out, n_blocks); break;
        case 17: hipLaunchKernelGGL(k_copy_pipe<0>, dim3(cus * 4), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 18: hipLaunchKernelGGL(k_copy_pipe<0>, dim3(cus * 8), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 19: hipLaunchKernelGGL(k_copy_pipe<1>, dim3(cus * 8), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 20: hipLaunchKernelGGL(k_burst<0>, dim3(unsigned(n_blocks / 32)), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 21: hipLaunchKernelGGL(k_burst<1>, dim3(unsigned(n_blocks / 32)), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 22: hipLaunchKernelGGL(k_write_wave, dim3(unsigned(out_bytes / 16 / 2048 / 4)), dim3(256), 0, 0, (uint4*)out, out_bytes / 16); break;
        case 23: hipLaunchKernelGGL(k_lds<0>, dim3(unsigned(n_blocks / 32)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 24: hipLaunchKernelGGL(k_lds<1>, dim3(unsigned(n_blocks / 32)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 25: hipLaunchKernelGGL(k_lds2<0>, dim3(unsigned(n_blocks / 32)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 26: hipLaunchKernelGGL(k_lds2<1>, dim3(unsigned(n_blocks / 32)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 27: hipLaunchKernelGGL(k_lds_k1<0>, dim3(unsigned(n_blocks / 32)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 28: hipLaunchKernelGGL(k_lds_k1<1>, dim3(unsigned(n_blocks / 32)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 29: hipLaunchKernelGGL((k_lds2<1, 16>), dim3(unsigned(n_blocks / 16)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 30: hipLaunchKernelGGL((k_lds2<1, 64>), dim3(unsigned(n_blocks / 64)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 31: hipLaunchKernelGGL((k_lds2<1, 8>), dim3(unsigned(n_blocks / 8)), dim3(256), 0, 0, src, out, n_blocks); break;
        case 32: hipLaunchKernelGGL((k_burst_pipe<1, 32>), dim3(cus * 2), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 33: hipLaunchKernelGGL((k_burst_pipe<1, 16>), dim3(cus * 4), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 34: hipLaunchKernelGGL((k_burst_pipe<1, 16>), dim3(cus * 3), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 35: hipLaunchKernelGGL((k_burst_pipe<0, 32>), dim3(cus * 2), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 36: hipLaunchKernelGGL((k_burst_pipe<0, 16>), dim3(cus * 4), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 37: hipLaunchKernelGGL((k_burst<1, 1>), dim3(unsigned(n_blocks / 32)), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 8: hipLaunchKernelGGL(k_write, dim3(cus * 8), dim3(256), 0, 0, (uint4*)out, out_bytes / 16); break;
        }
    };
    std::vector<uint32_t> h_ref(n_vals), h_out(n_vals);
    CK(hipMemcpy(h_ref.data(), ref, out_bytes, hipMemcpyDeviceToHost));
    for (auto& v : vars) {
        if (v.id == 7 || v.id == 8 || v.id == 12 || (v.id >= 17 && v.id != 9 && v.id != 10 && v.id < 23) || v.id >= 32) continue;
        CK(hipMemset(out, 0, out_bytes));
        launch(v.id, in[0]);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h_out.data(), out, out_bytes, hipMemcpyDeviceToHost));
        printf("check %-16s %s\n", v.name, h_out == h_ref ? "OK" : "MISMATCH");
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int rounds = 7, reps = 20;
    std::vector<std::vector<float>> t(vars.size());
    int rot = 0;
    for (int r = 0; r < rounds; r++) {
        for (size_t vi = 0; vi < vars.size(); vi++) {
            for (int k = 0; k < 3; k++) launch(vars[vi].id, in[(rot++) % copies]);
            for (int k = 0; k < reps; k++) {
                if (flush) CK(hipMemsetAsync(junk, k & 0xff, 512ull << 20, 0));
                CK(hipEventRecord(a, 0));
                launch(vars[vi].id, in[(rot++) % copies]);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                t[vi].push_back(ms);
            }
        }
    }
    printf("copies=%d (%.0f MB of inputs) flush=%d\n", copies, copies * in_bytes / 1e6, int(flush));
    const double bytes = double(in_bytes + out_bytes);
    for (size_t vi = 0; vi < vars.size(); vi++) {
        auto v = t[vi];
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2], mn = v[0];
        const double by = (vars[vi].id == 8 || vars[vi].id == 22) ? double(out_bytes) : bytes;
        printf("%-16s median %8.2f us  min %8.2f us  algo %7.1f GB/s (%.1f%% of 8 TB/s)\n",
               vars[vi].name, med * 1e3, mn * 1e3, by / (med * 1e-3) / 1e9, 100.0 * by / (med * 1e-3) / 8e12);
    }
    return 0;
}
