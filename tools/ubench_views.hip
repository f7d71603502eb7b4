// ubench_views.hip — the store shape of a string-dictionary column (C5's l_shipmode & co: 6,001,215
// rows -> 96 MB of 16-byte views): how fast can a launch of that shape write, and what does the
// per-workgroup prologue (a dependent load pair before the first store) cost?
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/ubench_views.hip -o tools/ubench_views
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ void st(uint4* p, uint4 v) {
    if constexpr (NT) __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(p));
    else *p = v;
}

// K1g's row order: workgroup = RPW rows (RPW / 1024 FastLanes blocks), thread tid writes rows
// blk*1024 + k*256 + tid (k = 0..3) of every block.  DEP: the values come from a 16-entry table
// that is first built from two dependent global loads (the VarBin dictionary's offsets, then its
// bytes), as the K1g VarBin-dictionary job does.
template <int NT, int DEP>
__global__ __launch_bounds__(256) void w_views(uint4* __restrict__ out, uint64_t n, int rpw, const uint32_t* __restrict__ offs,
                                               const uint8_t* __restrict__ heap, const uint8_t* __restrict__ codes) {
    __shared__ uint4 s_tab[16];
    const int tid = threadIdx.x;
    const uint64_t r0 = uint64_t(blockIdx.x) * rpw;
    if constexpr (DEP) {
        if (tid < 16) {
            const uint32_t a = offs[tid], e = offs[tid + 1];
            const uint32_t p = *reinterpret_cast<const uint32_t*>(heap + a);
            s_tab[tid] = make_uint4(e - a, p, 0, a);
        }
        __syncthreads();
    }
    for (int q = 0; q < rpw; q += 256) {
        const uint64_t r = r0 + q + tid;
        if (r >= n) break;
        uint4 v;
        if constexpr (DEP) v = s_tab[codes[r] & 15];
        else v = make_uint4(uint32_t(r), 1u, 2u, 3u);
        st<NT>(out + r, v);
    }
}

int main() {
    const uint64_t n = 6001215;
    const int copies = 4;  // 4 columns' outputs: rotate past the 256 MiB MALL
    std::vector<uint4*> out(copies);
    for (auto& p : out) CK(hipMalloc(&p, n * 16));
    uint32_t* offs;
    uint8_t *heap, *codes;
    CK(hipMalloc(&offs, 17 * 4));
    CK(hipMalloc(&heap, 4096));
    CK(hipMalloc(&codes, n));
    std::vector<uint32_t> ho(17);
    for (int i = 0; i <= 16; i++) ho[i] = 7 * i;
    CK(hipMemcpy(offs, ho.data(), 17 * 4, hipMemcpyHostToDevice));
    CK(hipMemset(heap, 65, 4096));
    CK(hipMemset(codes, 3, n));
    struct V { const char* name; int nt, dep, rpw; };
    std::vector<V> vs = {{"rows4096_nt", 1, 0, 4096},  {"rows4096_plain", 0, 0, 4096}, {"rows8192_nt", 1, 0, 8192},
                         {"rows2048_nt", 1, 0, 2048},  {"rows1024_nt", 1, 0, 1024},    {"rows4096_nt_dep", 1, 1, 4096},
                         {"rows2048_nt_dep", 1, 1, 2048}, {"rows1024_nt_dep", 1, 1, 1024}, {"rows8192_nt_dep", 1, 1, 8192}};
    int rot = 0;
    auto launch = [&](const V& v) {
        const unsigned g = unsigned((n + v.rpw - 1) / v.rpw);
        uint4* o = out[(rot++) % copies];
        if (v.nt && v.dep) hipLaunchKernelGGL((w_views<1, 1>), dim3(g), dim3(256), 0, 0, o, n, v.rpw, offs, heap, codes);
        else if (v.nt) hipLaunchKernelGGL((w_views<1, 0>), dim3(g), dim3(256), 0, 0, o, n, v.rpw, offs, heap, codes);
        else hipLaunchKernelGGL((w_views<0, 0>), dim3(g), dim3(256), 0, 0, o, n, v.rpw, offs, heap, codes);
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int K = 40;
    for (int rep = 0; rep < 3; rep++)
        for (const V& v : vs) {
            for (int k = 0; k < 5; k++) launch(v);
            CK(hipEventRecord(a, 0));
            for (int k = 0; k < K; k++) launch(v);  // back to back: the two-event mean of bench.py
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            const double us = ms * 1e3 / K;
            if (rep == 2) printf("%-18s %8.2f us per launch  %7.1f GB/s  (%.3f of 8 TB/s)\n", v.name, us, n * 16 / (us * 1e3),
                                 n * 16 / (us * 1e3) / 8000.0);
        }
    return 0;
}
