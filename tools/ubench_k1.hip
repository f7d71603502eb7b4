// ubench_k1.hip — A/B variants of the FastLanes unpack kernel on the C1 shape
// (u32, W=7, 64 Mi values), timed interleaved in one process (cdna_hip_programming.md §5.4
// rule 24).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -I../vortex_amd/csrc
//                   tools/ubench_k1.hip -o tools/ubench_k1
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

constexpr int T = 32, W = 7;

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

// persistent grid-stride: each 8-thread group walks blocks g, g+G, ...
template <int NT>
__global__ __launch_bounds__(256) void k_stride(const uint8_t* __restrict__ packed, uint32_t* __restrict__ out,
                                                uint64_t n_blocks) {
    const uint64_t gid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t groups = uint64_t(gridDim.x) * blockDim.x / 8;
    EpiParams ep{};
    for (uint64_t blk = gid >> 3; blk < n_blocks; blk += groups)
        unpack_block<T, W, Epi::Plain, 0, NT>(packed + blk * (128 * W), int(gid & 7), out, int64_t(blk * 1024),
                                              true, n_blocks * 1024, ep);
}

// block-major within the workgroup: 256 threads = 32 consecutive blocks, but thread t's slice
// and block are swapped so a wave's 64 lanes cover 8 slices x 8 blocks (same as base) — kept as
// the control; plus a 2-blocks-per-group variant that issues both blocks' loads up front.
template <int NT>
__global__ __launch_bounds__(256) void k_two(const uint8_t* __restrict__ packed, uint32_t* __restrict__ out,
                                             uint64_t n_blocks) {
    const uint64_t gid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t blk0 = (gid >> 3) * 2;
    const int t = int(gid & 7);
    if (blk0 >= n_blocks) return;
    Vec16<T> p0[W], p1[W];
#pragma unroll
    for (int w = 0; w < W; w++) p0[w] = load16<T>(packed + blk0 * (128 * W) + 128 * w + 16 * t);
#pragma unroll
    for (int w = 0; w < W; w++) p1[w] = load16<T>(packed + (blk0 + 1) * (128 * W) + 128 * w + 16 * t);
    EpiParams ep{};
    bool oob = false;
    process_rows<T, W, Epi::Plain, 0, NT, true>(p0, t * 4, out, int64_t(blk0 * 1024), n_blocks * 1024, ep, oob,
                                          std::make_integer_sequence<int, T>{});
    process_rows<T, W, Epi::Plain, 0, NT, true>(p1, t * 4, out, int64_t((blk0 + 1) * 1024), n_blocks * 1024, ep, oob,
                                          std::make_integer_sequence<int, T>{});
}

// Roofline reference with the same bytes: each thread reads 7 x 16 B and writes 32 x 16 B,
// every wave-instruction fully contiguous (1 KiB).
template <int NT>
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n_blocks) {
    const uint64_t gid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t wave = gid >> 6;
    const int lane = int(gid & 63);
    if (wave * 8 >= n_blocks) return;
    // a wave owns 8 blocks: reads 8*128*7 B = 448 uint4, writes 8*4096 B = 2048 uint4
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

__global__ void fill_rand(uint32_t* p, uint64_t n, uint32_t seed) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint32_t x = uint32_t(i) * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = x;
    }
}

int main(int argc, char** argv) {
    const uint64_t n_vals = 64ull << 20, n_blocks = n_vals / 1024;
    const uint64_t in_bytes = n_blocks * 128 * W, out_bytes = n_vals * 4;
    const int copies = 4;
    std::vector<uint8_t*> in(copies);
    for (int c = 0; c < copies; c++) {
        CK(hipMalloc(&in[c], in_bytes));
        hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, (uint32_t*)in[c], in_bytes / 4, 1234u + c);
    }
    uint32_t *out, *ref;
    CK(hipMalloc(&out, out_bytes));
    CK(hipMalloc(&ref, out_bytes));
    CK(hipDeviceSynchronize());
    const unsigned grid_base = unsigned(n_blocks * 8 / 256);
    hipLaunchKernelGGL(k_base<0>, dim3(grid_base), dim3(256), 0, 0, in[0], ref, n_blocks);
    CK(hipDeviceSynchronize());

    struct Var { const char* name; int id; };
    std::vector<Var> vars = {{"base", 0}, {"base_nt", 1}, {"stride2048", 2}, {"stride2048_nt", 3}, {"two_blocks", 4},
                             {"two_blocks_nt", 5}, {"copy_ref", 6}, {"copy_ref_nt", 7}, {"stride4096_nt", 8}};
    auto launch = [&](int id, const uint8_t* src) {
        switch (id) {
        case 0: hipLaunchKernelGGL(k_base<0>, dim3(grid_base), dim3(256), 0, 0, src, out, n_blocks); break;
        case 1: hipLaunchKernelGGL(k_base<1>, dim3(grid_base), dim3(256), 0, 0, src, out, n_blocks); break;
        case 2: hipLaunchKernelGGL(k_stride<0>, dim3(2048), dim3(256), 0, 0, src, out, n_blocks); break;
        case 3: hipLaunchKernelGGL(k_stride<1>, dim3(2048), dim3(256), 0, 0, src, out, n_blocks); break;
        case 4: hipLaunchKernelGGL(k_two<0>, dim3(grid_base / 2), dim3(256), 0, 0, src, out, n_blocks); break;
        case 5: hipLaunchKernelGGL(k_two<1>, dim3(grid_base / 2), dim3(256), 0, 0, src, out, n_blocks); break;
        case 6: hipLaunchKernelGGL(k_copy<0>, dim3(unsigned(n_blocks / 8 * 64 / 256)), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 7: hipLaunchKernelGGL(k_copy<1>, dim3(unsigned(n_blocks / 8 * 64 / 256)), dim3(256), 0, 0, (const uint4*)src, (uint4*)out, n_blocks); break;
        case 8: hipLaunchKernelGGL(k_stride<1>, dim3(4096), dim3(256), 0, 0, src, out, n_blocks); break;
        }
    };
    // correctness of the decode variants vs base
    std::vector<uint32_t> h_ref(n_vals), h_out(n_vals);
    CK(hipMemcpy(h_ref.data(), ref, out_bytes, hipMemcpyDeviceToHost));
    for (auto& v : vars) {
        if (v.id >= 6 && v.id <= 7) continue;
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
    const double bytes = double(in_bytes + out_bytes);
    for (size_t vi = 0; vi < vars.size(); vi++) {
        auto v = t[vi];
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2], mn = v[0];
        printf("%-16s median %8.2f us  min %8.2f us  algo %7.1f GB/s (%.1f%% of 8 TB/s)  decoded %7.1f GB/s\n",
               vars[vi].name, med * 1e3, mn * 1e3, bytes / (med * 1e-3) / 1e9,
               100.0 * bytes / (med * 1e-3) / 8e12, out_bytes / (med * 1e-3) / 1e9);
    }
    return 0;
}
