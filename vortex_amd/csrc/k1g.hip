// k1g.hip — K1g: the K1 decodes of a recorded plan with DIFFERENT kernels in one launch
// (k1g.hpp).  Same decode and epilogues as K1 (fl_unpack_impl.hpp: FoR for/compress.rs:100-117,
// ZigZag zigzag/compress.rs:35-57, ALP alp/mod.rs:161-163, Dict dict/array.rs:68-73), but the
// bit width is a runtime value: a 256-thread workgroup stages `bpw` FastLanes blocks' packed words
// (128 * W bytes each) in LDS and thread t produces values t, t + 256, t + 512, t + 768 of every
// block (64 consecutive values per store wave-instruction); value i of a block is unpack_single's
// (lane, row) -> one or two T-bit words of that lane.  The body (T, epilogue, value width) is a
// workgroup-uniform switch on the job's kind.
#include <algorithm>

#include "k1g_impl.hpp"

namespace vxg {

namespace {

__global__ __launch_bounds__(kGenThreads) void k1_generic_kernel(const GenChunk* __restrict__ tab, uint32_t n,
                                                                 uint32_t dict_off, bool dict_lds, uint32_t* err,
                                                                 uint64_t gpe) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint64_t g = blockIdx.x;
    const GenChunk& gc = tab[ext_chunk_index_gpe(tab, n, g, gpe, [](const GenChunk& d) { return d.d.first_group; })];
    gen_dispatch(int(gc.kind), gc, g, lds, dict_off, dict_lds, err);
}

}  // namespace

int gen_runs_kind(int value_width) {
    switch (value_width) {
    case 1: return 38;
    case 2: return 39;
    case 4: return 40;
    case 8: return 41;
    case 16: return 42;
    default: return -1;
    }
}

int gen_kind(int T, int epi, int vw, bool varbin_dict) {
    const int ti = T == 8 ? 0 : T == 16 ? 1 : T == 32 ? 2 : T == 64 ? 3 : -1;
    if (ti < 0) return -1;
    if (varbin_dict) return Epi(epi) == Epi::Dict && vw == 16 ? 34 + ti : -1;
    switch (Epi(epi)) {
    case Epi::Plain: return 3 * ti;
    case Epi::For: return 3 * ti + 1;
    case Epi::ForZigZag: return 3 * ti + 2;
    case Epi::AlpF32: return T == 32 ? 12 : -1;
    case Epi::AlpF64: return T == 64 ? 13 : -1;
    case Epi::Dict: {
        const int vi = vw == 1 ? 0 : vw == 2 ? 1 : vw == 4 ? 2 : vw == 8 ? 3 : vw == 16 ? 4 : -1;
        return vi < 0 ? -1 : 14 + 5 * ti + vi;
    }
    }
    return -1;
}

// Blocks per K1g workgroup: as many as kGenPackedLds of packed words hold, at most the launch's
// cap (gen_bpw_cap; VXG_K1G_BPW, read once, fixes it for every launch).
static long gen_bpw_env() {
    static const long v = [] {
        const char* e = std::getenv("VXG_K1G_BPW");
        const long x = e ? std::strtol(e, nullptr, 10) : 0;
        return x >= 1 && x <= 32 ? x : 0L;
    }();
    return v;
}

// 8 blocks per workgroup halve the per-workgroup prologue (job lookup, descriptor, dictionary
// staging) per block, but only pay while the grid still has work for every CU's slots: C5 at one
// GPU (the fused launch's ~29 K blocks) 0.2672 -> 0.2591 ms with 8, its 8-GPU shard (~3.7 K
// blocks) 0.0387 -> 0.0406 (session r06v, profiles/r06_c5_plan.md).
constexpr uint64_t kGenWideMinGroups = 2048;
uint32_t gen_bpw_cap(uint64_t blocks) {
    if (const long v = gen_bpw_env()) return uint32_t(v);
    return blocks / 8 >= kGenWideMinGroups ? 8u : 4u;
}

uint32_t gen_bpw(int T, int W, uint32_t cap) {
    (void)T;
    const uint32_t per = 128u * uint32_t(W > 0 ? W : 1);
    const uint32_t b = kGenPackedLds / per, m = cap ? cap : (gen_bpw_env() ? uint32_t(gen_bpw_env()) : 4u);
    return b > m ? m : (b < 1 ? 1 : b);
}

// Dict-over-VarBin jobs: every workgroup builds the dictionary's views (one dependent round trip)
// and then writes 16-byte views.  Alone in a launch (a one-generation grid: one C5 column is
// ~1,500 workgroups of 4 blocks) 1,024-row workgroups write faster -- C5's four string columns
// each as its own plan 0.56-0.59 -> 0.60-0.66 of 8 TB/s with 1 block (0.62-0.63 with 2; session
// r06j; pure 96 MB view stores: 15.4 / 17.1 us for 1,024 / 4,096-row workgroups,
// profiles/r04_ubench_views.txt) -- while beside FSST tiles in the fused launch 4 blocks stay
// best (C5 1 GPU 0.272-0.280 ms with 4 and 2, 0.305 with 1; session r06k).
uint32_t gen_vb_bpw(int T, int W, bool alone, uint32_t cap) {
    static const long v = [] {
        const char* e = std::getenv("VXG_K1G_VB_BPW");
        return e ? std::strtol(e, nullptr, 10) : 0L;
    }();
    // (VXG_K1G_VB_BPW set: that many blocks, above the launch's cap too, as LDS allows)
    const uint32_t b = gen_bpw(T, W, v >= 1 && uint32_t(v) > cap ? uint32_t(v) : cap);
    const uint32_t want = v >= 1 ? uint32_t(v) : (alone ? 1u : b);
    return want < b ? want : b;
}

uint32_t gen_runs_lds_bytes(int value_width) {
    switch (value_width) {
    case 1: return uint32_t(runs_lds_bytes<uint8_t>());
    case 2: return uint32_t(runs_lds_bytes<uint16_t>());
    case 4: return uint32_t(runs_lds_bytes<uint32_t>());
    case 8: return uint32_t(runs_lds_bytes<uint64_t>());
    default: return uint32_t(runs_lds_bytes<uint4>());
    }
}

vxg_status launch_k1_generic(const GenChunk* ext, uint32_t n, uint64_t groups, bool dict_lds, uint32_t packed_bytes,
                             uint32_t dict_bytes, uint32_t runs_bytes, uint32_t* err, hipStream_t s,
                             uint64_t gpe, const FsstFused* fuse) {
    static_assert(kGenVarBinDictMax * 16 <= uint64_t(kDictLdsBytes), "VarBin views must fit the dictionary stage");
    if (n == 0) groups = 0;
    if (groups == 0 && !(fuse && fuse->valid)) return VXG_OK;
    if (groups > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "array too long for one launch");
    if (packed_bytes > kGenPackedLds || dict_bytes > uint32_t(kDictLdsBytes))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "K1g stage sizes");
    // LDS = the largest packed stage + the largest dictionary stage, or a RunEnd expansion's
    // (sized by the launch's jobs, so small jobs keep residency high)
    // (+ one 128-byte word row of slack past the packed stage: gen_body_w reads, and masks, the
    // row after a block's last)
    const uint32_t dict_off = (packed_bytes + 128 + 15) & ~15u;
    const size_t shm = std::max<size_t>({size_t(dict_off) + dict_bytes, size_t(runs_bytes), 16});
    if (fuse && fuse->valid) return launch_fsst_k1g(*fuse, ext, n, groups, dict_off, dict_lds, shm, err, s, gpe);
    hipLaunchKernelGGL(k1_generic_kernel, dim3(unsigned(groups)), dim3(kGenThreads), shm, s, ext, n, dict_off, dict_lds,
                       err, gpe);
    return hip_check(hipGetLastError(), "k1_generic_kernel launch");
}

}  // namespace vxg
