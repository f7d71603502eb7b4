// ubench_lds.hip -- LDS store flavours for the FSST image writer (gfx950): cycles per
// wave-instruction and correctness of misaligned ds_write_b32 / ds_write_b64.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_lds.hip -o tools/ubench_lds && ./tools/ubench_lds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int kThreads = 256, kIters = 256, kStride = 52;  // bytes between lanes' regions

template <int MODE>
__global__ void k(uint32_t* out, long long* cyc) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[kThreads * kStride + 64];
    const int tid = threadIdx.x;
    for (int i = tid; i < (kThreads * kStride + 64) / 4; i += kThreads) reinterpret_cast<uint32_t*>(buf)[i] = 0;
    __syncthreads();
    const uint32_t base = uint32_t(reinterpret_cast<uintptr_t>(buf));  // LDS byte address (low bits)
    long long t0 = clock64();
    for (int it = 0; it < kIters; it++) {
        const uint32_t a = tid * kStride + ((MODE == 0 || MODE == 3) ? 0 : 1 + (it & 1));
        const uint32_t v = 0x01010101u * uint32_t(it & 0xFF) + uint32_t(tid);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if constexpr (MODE == 0 || MODE == 1) {        // ds_write_b32 aligned / misaligned
                asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(base + a), "v"(v + j), "i"(4 * j) : "memory");
            } else if constexpr (MODE == 2) {              // ds_write_b64 misaligned
                uint64_t w = (uint64_t(v) << 32) | (v + j);
                asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(base + a), "v"(w), "i"(4 * j) : "memory");
            } else {                                       // ds_or_b32 aligned atomic
                asm volatile("ds_or_b32 %0, %1 offset:%2" ::"v"(base + a), "v"(v + j), "i"(4 * j) : "memory");
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long t1 = clock64();
    __syncthreads();
    for (int i = tid; i < kThreads * kStride; i += kThreads) out[blockIdx.x * kThreads * kStride + i] = buf[i];
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    const int blocks = 1024;
    uint32_t* d_out;
    long long* d_cyc;
    hipMalloc(&d_out, sizeof(uint32_t) * blocks * kThreads * kStride);
    hipMalloc(&d_cyc, sizeof(long long) * blocks);
    std::vector<uint32_t> h(kThreads * kStride);
    std::vector<long long> c(blocks);
    const char* names[] = {"ds_write_b32 aligned", "ds_write_b32 misaligned", "ds_write_b64 misaligned",
                           "ds_or_b32 aligned"};
    for (int mode = 0; mode < 4; mode++) {
        for (int rep = 0; rep < 2; rep++) {
            if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(kThreads), 0, 0, d_out, d_cyc);
            if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(kThreads), 0, 0, d_out, d_cyc);
            if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(kThreads), 0, 0, d_out, d_cyc);
            if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(kThreads), 0, 0, d_out, d_cyc);
        }
        hipDeviceSynchronize();
        hipMemcpy(h.data(), d_out, sizeof(uint32_t) * kThreads * kStride, hipMemcpyDeviceToHost);
        hipMemcpy(c.data(), d_cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
        double avg = 0;
        for (auto x : c) avg += double(x);
        avg /= blocks;
        // expected bytes of lane 5 after the last iteration (it = kIters-1, odd -> offset 2)
        const int tid = 5, it = kIters - 1;
        const uint32_t a = tid * kStride + ((mode == 0 || mode == 3) ? 0 : 1 + (it & 1));
        const uint32_t v = 0x01010101u * uint32_t(it & 0xFF) + uint32_t(tid);
        bool ok = true;
        if (mode == 1) {
            for (int j = 0; j < 8; j++)
                for (int b = 0; b < 4; b++) ok &= h[a + 4 * j + b] == (((v + j) >> (8 * b)) & 0xFF);
        } else if (mode == 2) {
            for (int b = 0; b < 4; b++) ok &= h[a + 4 * 7 + b] == (((v + 7) >> (8 * b)) & 0xFF);
            for (int b = 0; b < 4; b++) ok &= h[a + 4 * 7 + 4 + b] == ((v >> (8 * b)) & 0xFF);
        }
        printf("%-26s %8.1f cycles per wave-instruction (per-wave clock)  data %s\n", names[mode],
               avg / (kIters * 8.0), (mode == 1 || mode == 2) ? (ok ? "OK" : "WRONG") : "-");
    }
    return 0;
}
