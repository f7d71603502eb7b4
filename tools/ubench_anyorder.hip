// ubench_anyorder.hip — does a chain of independent streaming launches (C5's seven numeric K1w
// groups: 48 MB written + 8 MB read each, ~1,500 workgroups) lose its ramp/drain between
// launches when the later packets are enqueued WITHOUT the AQL barrier bit
// (hipExtLaunchKernel(..., hipExtAnyOrderLaunch))?  Compared with: plain launches on one stream,
// launches alternated over two streams (event fork/join), and one launch doing all the work.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/ubench_anyorder.hip -o tools/ubench_anyorder
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

// each workgroup: reads 2 KiB (the packed input share), writes 12 KiB (K1w-like 1:6 ratio)
__global__ __launch_bounds__(256) void job(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t groups) {
    const uint64_t g = blockIdx.x;
    if (g >= groups) return;
    const int t = threadIdx.x;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (t < 128) v = in[g * 128 + t];
    const uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
#pragma unroll
    for (int k = 0; k < 3; k++)
        __builtin_nontemporal_store(u32x4{x + k, x, x ^ k, unsigned(g)}, reinterpret_cast<u32x4*>(out + g * 768 + k * 256 + t));
}

int main(int argc, char** argv) {
    const int K = 7;
    const uint64_t groups = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 4096;  // 48 MB written per launch
    const int copies = 4;  // rotate past the Infinity Cache
    std::vector<uint4*> in(copies * K), out(copies * K);
    for (auto& p : in) { CK(hipMalloc(&p, groups * 2048)); CK(hipMemset(p, 1, groups * 2048)); }
    for (auto& p : out) CK(hipMalloc(&p, groups * 12288));
    uint4 *big_in, *big_out;
    CK(hipMalloc(&big_in, K * groups * 2048));
    CK(hipMalloc(&big_out, K * groups * 12288));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t a, b, f0, f1;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreateWithFlags(&f0, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&f1, hipEventDisableTiming));
    int rot = 0;
    auto seq = [&](int mode) {
        const int c = (rot++) % copies;
        switch (mode) {
        case 0:  // plain
            for (int k = 0; k < K; k++) hipLaunchKernelGGL(job, dim3(unsigned(groups)), dim3(256), 0, s0, in[c * K + k], out[c * K + k], groups);
            break;
        case 1:  // any order after the first
            for (int k = 0; k < K; k++)
                hipExtLaunchKernelGGL(job, dim3(unsigned(groups)), dim3(256), 0, s0, nullptr, nullptr, k ? hipExtAnyOrderLaunch : 0u,
                                      (const uint4*)in[c * K + k], out[c * K + k], groups);
            break;
        case 2:  // two streams
            CK(hipEventRecord(f0, s0));
            CK(hipStreamWaitEvent(s1, f0, 0));
            for (int k = 0; k < K; k++)
                hipLaunchKernelGGL(job, dim3(unsigned(groups)), dim3(256), 0, (k & 1) ? s1 : s0, in[c * K + k], out[c * K + k], groups);
            CK(hipEventRecord(f1, s1));
            CK(hipStreamWaitEvent(s0, f1, 0));
            break;
        case 4:  // any order, then a plain empty launch (does the event already wait for them?)
            for (int k = 0; k < K; k++)
                hipExtLaunchKernelGGL(job, dim3(unsigned(groups)), dim3(256), 0, s0, nullptr, nullptr, k ? hipExtAnyOrderLaunch : 0u,
                                      (const uint4*)in[c * K + k], out[c * K + k], groups);
            hipLaunchKernelGGL(job, dim3(1), dim3(256), 0, s0, in[c * K], out[c * K], uint64_t(0));
            break;
        case 3:  // one launch
            hipLaunchKernelGGL(job, dim3(unsigned(K * groups)), dim3(256), 0, s0, big_in, big_out, K * groups);
            break;
        }
    };
    const char* names[] = {"plain", "anyorder", "two_streams", "one_launch", "anyorder+tail"};
    std::vector<std::vector<float>> t(5);
    for (int r = 0; r < 5; r++)
        for (int m = 0; m < 5; m++) {
            for (int k = 0; k < 3; k++) seq(m);
            for (int k = 0; k < 20; k++) {
                CK(hipEventRecord(a, s0));
                seq(m);
                CK(hipEventRecord(b, s0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                t[m].push_back(ms);
            }
        }
    CK(hipDeviceSynchronize());
    const double bytes = double(K) * groups * (2048 + 12288);
    for (int m = 0; m < 5; m++) {
        auto v = t[m];
        std::sort(v.begin(), v.end());
        printf("%-12s groups %llu  median %8.2f us  min %8.2f us  %7.1f GB/s\n", names[m], (unsigned long long)groups,
               v[v.size() / 2] * 1e3, v[0] * 1e3, bytes / (v[v.size() / 2] * 1e-3) / 1e9);
    }
    return 0;
}
