// ubench_dict.hip — A/B variants of the FastLanes unpack kernel on the C3 shape (Dict over
// BitPacked u64 codes, W=10, 1024 u64 dictionary entries, 16 Mi values = one GPU's share of C3),
// timed interleaved in one process.  Questions: does a 16 Mi-value launch (512 workgroups,
// 2 waves/SIMD) starve the chip, and does splitting each block's rows over SPLIT waves help?
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/ubench_dict.hip -o tools/ubench_dict
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../vortex_amd/csrc/fl_unpack_impl.hpp"

namespace vxg {
vxg_status set_error(vxg_status s, const std::string&) { return s; }
vxg_status hip_check(hipError_t e, const char*) { return e == hipSuccess ? VXG_OK : VXG_ERR_HIP; }
}  // namespace vxg

using namespace vxg;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int T = 64, W = 10, VW = 8;

template <int T_, int W_, Epi EPI, int VW_, int NT, int R0, int... Rs>
__device__ __forceinline__ void rows_from(const Vec16<T_>* p, int lane0, typename EpiOut<T_, EPI, VW_>::type* out,
                                          int64_t out_base, uint64_t len, const EpiParams& ep,
                                          std::integer_sequence<int, Rs...>) {
    bool oob = false;
    (process_row<T_, W_, EPI, VW_, NT, R0 + Rs, true>(p, lane0, out, out_base, len, ep, oob), ...);
}

template <int T_, int W_, Epi EPI, int VW_, int R0, int R1>
__device__ __forceinline__ void unpack_rows(const uint8_t* __restrict__ blk, int t,
                                            typename EpiOut<T_, EPI, VW_>::type* out, int64_t out_base, uint64_t len,
                                            const EpiParams& ep) {
    constexpr int WA = (R0 * W_) / T_, WB = (R1 * W_ - 1) / T_;
    Vec16<T_> p[W_];
#pragma unroll
    for (int w = WA; w <= WB; w++) p[w] = load16<T_>(blk + 128 * w + 16 * t);
    rows_from<T_, W_, EPI, VW_, 1, R0>(p, t * (16 / (T_ / 8)), out, out_base, len, ep,
                                      std::make_integer_sequence<int, R1 - R0>{});
}

template <int T_, int W_, Epi EPI, int VW_, int SPLIT, bool LDSD>
__global__ __launch_bounds__(256) void k_split(const uint8_t* __restrict__ packed,
                                               typename EpiOut<T_, EPI, VW_>::type* __restrict__ out,
                                               uint64_t n_blocks, EpiParams ep) {
    if constexpr (LDSD) {
        __shared__ __attribute__((aligned(16))) uint8_t s_dict[kDictLdsBytes];
        stage_dict<VW_>(s_dict, ep.dict, ep.dict_len);
        ep.dict = s_dict;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int part = __builtin_amdgcn_readfirstlane(wave % SPLIT);
    const uint64_t blk = (uint64_t(blockIdx.x) * (4 / SPLIT) + wave / SPLIT) * 8 + (lane >> 3);
    const int t = lane & 7;
    if (blk >= n_blocks) return;
    const uint8_t* b = packed + blk * (128 * W_);
    const int64_t ob = int64_t(blk * 1024);
    const uint64_t len = n_blocks * 1024;
    constexpr int RS = T_ / SPLIT;
    if constexpr (SPLIT == 1) {
        unpack_rows<T_, W_, EPI, VW_, 0, T_>(b, t, out, ob, len, ep);
    } else if constexpr (SPLIT == 2) {
        if (part == 0) unpack_rows<T_, W_, EPI, VW_, 0, RS>(b, t, out, ob, len, ep);
        else unpack_rows<T_, W_, EPI, VW_, RS, T_>(b, t, out, ob, len, ep);
    } else {
        static_assert(SPLIT == 4);
        if (part == 0) unpack_rows<T_, W_, EPI, VW_, 0, RS>(b, t, out, ob, len, ep);
        else if (part == 1) unpack_rows<T_, W_, EPI, VW_, RS, 2 * RS>(b, t, out, ob, len, ep);
        else if (part == 2) unpack_rows<T_, W_, EPI, VW_, 2 * RS, 3 * RS>(b, t, out, ob, len, ep);
        else unpack_rows<T_, W_, EPI, VW_, 3 * RS, T_>(b, t, out, ob, len, ep);
    }
}

template <int NT>
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n_waves,
                                              int rd, int wr) {
    const uint64_t gid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t wave = gid >> 6;
    const int lane = int(gid & 63);
    if (wave >= n_waves) return;
    const uint4* src = in + wave * rd * 64;
    uint4* dst = out + wave * wr * 64;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int k = 0; k < rd; k++) {
        const uint4 r = src[k * 64 + lane];
        acc.x ^= r.x; acc.y ^= r.y; acc.z ^= r.z; acc.w ^= r.w;
    }
    for (int k = 0; k < wr; k++) {
        using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
        u32x4 vv = {acc.x + k, acc.y, acc.z, acc.w};
        __builtin_nontemporal_store(vv, reinterpret_cast<u32x4*>(dst + k * 64 + lane));
    }
}

__global__ void fill_rand(uint32_t* p, uint64_t n, uint32_t seed, uint32_t mask) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint32_t x = uint32_t(i) * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = x & mask;
    }
}

int main(int argc, char** argv) {
    const int mi = argc > 1 ? atoi(argv[1]) : 16;
    const uint64_t n_vals = uint64_t(mi) << 20, n_blocks = n_vals / 1024;
    const uint64_t in_bytes = n_blocks * 128 * W, out_bytes = n_vals * 8;
    const int copies = 4;
    std::vector<uint8_t*> in(copies);
    for (int c = 0; c < copies; c++) {
        CK(hipMalloc(&in[c], in_bytes));
        hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, (uint32_t*)in[c], in_bytes / 4, 1234u + c,
                           0xFFFFFFFFu);
    }
    uint64_t* dict;
    CK(hipMalloc(&dict, 1024 * 8));
    hipLaunchKernelGGL(fill_rand, dim3(8), dim3(256), 0, 0, (uint32_t*)dict, 2048, 99u, 0xFFFFFFFFu);
    uint64_t *out, *ref, *junk;
    CK(hipMalloc(&out, out_bytes));
    CK(hipMalloc(&ref, out_bytes));
    CK(hipMalloc(&junk, 512ull << 20));
    uint32_t* err;
    CK(hipMalloc(&err, 16));
    CK(hipMemset(err, 0, 16));
    CK(hipDeviceSynchronize());
    EpiParams ep{};
    ep.dict = dict;
    ep.dict_len = 1024;
    ep.err = err;
    const unsigned g1 = unsigned(n_blocks / 32), g2 = unsigned(n_blocks / 16), g4 = unsigned(n_blocks / 8);
    // the library kernel takes a chunk table (one chunk here)
    auto tab_of = [&](const uint8_t* src, void* dst) {
        ChunkTable t{};
        t.n = 1;
        t.err = err;
        t.c[0].packed = src;
        t.c[0].out = dst;
        t.c[0].n_blocks = n_blocks;
        t.c[0].len = n_vals;
        t.c[0].dict = dict;
        t.c[0].dict_len = 1024;
        return t;
    };
    hipLaunchKernelGGL((fl_unpack_kernel<T, W, Epi::Dict, VW>), dim3(g1), dim3(256), 0, 0, tab_of(in[0], ref));
    CK(hipDeviceSynchronize());

    struct Var { const char* name; int id; };
    std::vector<Var> vars = {{"lib_global_dict", 0}, {"lib_lds_dict", 1}, {"split1_lds", 2}, {"split2_lds", 3},
                             {"split4_lds", 4}, {"split4_global", 5}, {"plain_u64_w10", 6}, {"plain_split4", 7},
                             {"copy_ref", 8}};
    const uint64_t cw = n_blocks / 8;  // copy: a wave per 8 blocks: reads 8*1280 B = 80 x 1 KiB? use rd=10 (x1KiB / 64 lanes*16B)
    auto launch = [&](int id, const uint8_t* src) {
        switch (id) {
        case 0: hipLaunchKernelGGL((fl_unpack_kernel<T, W, Epi::Dict, VW, false>), dim3(g1), dim3(256), 0, 0, tab_of(src, out)); break;
        case 1: hipLaunchKernelGGL((fl_unpack_kernel<T, W, Epi::Dict, VW, true>), dim3(g1), dim3(256), 0, 0, tab_of(src, out)); break;
        case 2: hipLaunchKernelGGL((k_split<T, W, Epi::Dict, VW, 1, true>), dim3(g1), dim3(256), 0, 0, src, out, n_blocks, ep); break;
        case 3: hipLaunchKernelGGL((k_split<T, W, Epi::Dict, VW, 2, true>), dim3(g2), dim3(256), 0, 0, src, out, n_blocks, ep); break;
        case 4: hipLaunchKernelGGL((k_split<T, W, Epi::Dict, VW, 4, true>), dim3(g4), dim3(256), 0, 0, src, out, n_blocks, ep); break;
        case 5: hipLaunchKernelGGL((k_split<T, W, Epi::Dict, VW, 4, false>), dim3(g4), dim3(256), 0, 0, src, out, n_blocks, ep); break;
        case 6: hipLaunchKernelGGL((fl_unpack_kernel<T, W, Epi::Plain, 0>), dim3(g1), dim3(256), 0, 0, tab_of(src, out)); break;
        case 7: hipLaunchKernelGGL((k_split<T, W, Epi::Plain, 0, 4, false>), dim3(g4), dim3(256), 0, 0, src, out, n_blocks, ep); break;
        case 8: hipLaunchKernelGGL(k_copy<1>, dim3(unsigned(cw * 64 / 256)), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, cw, 10, 64); break;
        }
    };
    std::vector<uint64_t> h_ref(n_vals), h_out(n_vals);
    CK(hipMemcpy(h_ref.data(), ref, out_bytes, hipMemcpyDeviceToHost));
    for (auto& v : vars) {
        if (v.id >= 6) continue;
        CK(hipMemset(out, 0, out_bytes));
        launch(v.id, in[0]);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h_out.data(), out, out_bytes, hipMemcpyDeviceToHost));
        printf("check %-16s %s\n", v.name, h_out == h_ref ? "OK" : "MISMATCH");
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 30;
    std::vector<std::vector<float>> ms(vars.size());
    for (int r = 0; r < reps; r++) {
        for (size_t k = 0; k < vars.size(); k++) {
            hipLaunchKernelGGL(fill_rand, dim3(2048), dim3(256), 0, 0, (uint32_t*)junk, (512ull << 20) / 4, r, 0xFFFFFFFFu);
            CK(hipEventRecord(e0));
            launch(vars[k].id, in[r % copies]);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[k].push_back(t);
        }
    }
    const double bytes = double(in_bytes) + double(out_bytes);
    printf("n_vals=%llu Mi, algorithmic bytes %.1f MB (read %.1f MB, write %.1f MB)\n",
           (unsigned long long)(n_vals >> 20), bytes / 1e6, in_bytes / 1e6, out_bytes / 1e6);
    for (size_t k = 0; k < vars.size(); k++) {
        std::sort(ms[k].begin(), ms[k].end());
        const double med = ms[k][reps / 2];
        printf("%-16s median %8.2f us  min %8.2f us  %7.1f GB/s  %5.1f%% of 8 TB/s\n", vars[k].name, med * 1e3,
               ms[k][0] * 1e3, bytes / (med * 1e-3) / 1e9, 100.0 * bytes / (med * 1e-3) / 8e12);
    }
    return 0;
}
