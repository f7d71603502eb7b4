// ubench_write.hip — what write pattern reaches the highest HBM store rate on MI355X?  Pure
// 268 MB writes (the C1 output size) in several shapes; plus a read-only pass over 8 rotated
// 58.7 MB inputs.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/ubench_write.hip -o tools/ubench_write
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ void st(uint4* p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else *reinterpret_cast<u32x4*>(p) = v;
}

// grid-stride, 1 KiB per wave-instruction
template <int NT>
__global__ __launch_bounds__(256) void w_stride(uint4* __restrict__ out, uint64_t n16) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x)
        st<NT>(out + i, u32x4{unsigned(i), 1u, 2u, 3u});
}

// one shot: each wave writes KB consecutive KiB (KB instructions of 1 KiB)
template <int NT, int KB>
__global__ __launch_bounds__(256) void w_wave(uint4* __restrict__ out, uint64_t n16) {
    const uint64_t wave = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    uint4* base = out + wave * (KB * 64);
    if (wave * KB * 64 >= n16) return;
#pragma unroll
    for (int k = 0; k < KB; k++) st<NT>(base + k * 64 + lane, u32x4{unsigned(k), 1u, 2u, 3u});
}

// the K1 shape: 8 threads per 4 KiB block, each instruction = 8 blocks x 128 B
template <int NT>
__global__ __launch_bounds__(256) void w_k1(uint4* __restrict__ out, uint64_t n16) {
    const uint64_t gid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t blk = gid >> 3;
    const int t = int(gid & 7);
    if (blk * 256 >= n16) return;
    uint4* b = out + blk * 256;
#pragma unroll
    for (int r = 0; r < 32; r++) st<NT>(b + r * 8 + t, u32x4{unsigned(r), 1u, 2u, 3u});
}

__global__ __launch_bounds__(256) void r_only(const uint4* __restrict__ in, uint64_t n16, unsigned* sink) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
        uint4 v = in[i];
        acc.x ^= v.x; acc.y ^= v.y;
    }
    if ((acc.x ^ acc.y) == 0x12345678u) sink[0] = 1;
}

int main() {
    const uint64_t out_bytes = 256ull << 20, in_bytes = 58720256;
    const int copies = 8;
    uint4* out;
    CK(hipMalloc(&out, out_bytes));
    std::vector<uint4*> in(copies);
    for (auto& p : in) { CK(hipMalloc(&p, in_bytes)); CK(hipMemset(p, 1, in_bytes)); }
    unsigned* sink;
    CK(hipMalloc(&sink, 4));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const uint64_t n16 = out_bytes / 16;
    struct V { const char* name; int id; };
    std::vector<V> vs = {{"stride_x8_nt", 0}, {"stride_x8_plain", 1}, {"stride_x32_nt", 2}, {"wave32KB_nt", 3},
                         {"wave32KB_plain", 4}, {"wave8KB_nt", 5}, {"wave128KB_nt", 6}, {"k1shape_nt", 7},
                         {"k1shape_plain", 8}, {"read_only_x8", 9}};
    int rot = 0;
    auto launch = [&](int id) {
        switch (id) {
        case 0: hipLaunchKernelGGL(w_stride<1>, dim3(cus * 8), dim3(256), 0, 0, out, n16); break;
        case 1: hipLaunchKernelGGL(w_stride<0>, dim3(cus * 8), dim3(256), 0, 0, out, n16); break;
        case 2: hipLaunchKernelGGL(w_stride<1>, dim3(cus * 32), dim3(256), 0, 0, out, n16); break;
        case 3: hipLaunchKernelGGL((w_wave<1, 32>), dim3(unsigned(n16 / (32 * 64) / 4)), dim3(256), 0, 0, out, n16); break;
        case 4: hipLaunchKernelGGL((w_wave<0, 32>), dim3(unsigned(n16 / (32 * 64) / 4)), dim3(256), 0, 0, out, n16); break;
        case 5: hipLaunchKernelGGL((w_wave<1, 8>), dim3(unsigned(n16 / (8 * 64) / 4)), dim3(256), 0, 0, out, n16); break;
        case 6: hipLaunchKernelGGL((w_wave<1, 128>), dim3(unsigned(n16 / (128 * 64) / 4)), dim3(256), 0, 0, out, n16); break;
        case 7: hipLaunchKernelGGL(w_k1<1>, dim3(unsigned(n16 / 256 * 8 / 256)), dim3(256), 0, 0, out, n16); break;
        case 8: hipLaunchKernelGGL(w_k1<0>, dim3(unsigned(n16 / 256 * 8 / 256)), dim3(256), 0, 0, out, n16); break;
        case 9: hipLaunchKernelGGL(r_only, dim3(cus * 8), dim3(256), 0, 0, in[(rot++) % copies], in_bytes / 16, sink); break;
        }
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < 5; r++)
        for (size_t i = 0; i < vs.size(); i++) {
            for (int k = 0; k < 3; k++) launch(vs[i].id);
            for (int k = 0; k < 20; k++) {
                CK(hipEventRecord(a, 0));
                launch(vs[i].id);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                t[i].push_back(ms);
            }
        }
    for (size_t i = 0; i < vs.size(); i++) {
        auto v = t[i];
        std::sort(v.begin(), v.end());
        const double by = vs[i].id == 9 ? double(in_bytes) : double(out_bytes);
        printf("%-18s median %8.2f us  min %8.2f us  %7.1f GB/s\n", vs[i].name, v[v.size() / 2] * 1e3, v[0] * 1e3,
               by / (v[v.size() / 2] * 1e-3) / 1e9);
    }
    return 0;
}
