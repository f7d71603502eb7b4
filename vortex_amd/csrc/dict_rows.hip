// dict_rows.hip — K14: Dict(codes = BitPacked) canonicalize for wide dictionary values (8-byte
// primitives, 16-byte BinaryViews of a string dictionary), thread per output value.
//
// Reference: DictArray::into_canonical = take(values.into_canonical(), codes)
// (encodings/dict/src/array.rs:68-73; primitive/compute/take.rs:58-67; varbinview/compute.rs:
// 68-76 for views), the codes unpacked by fastlanes unpack_single (bitpacking/compress.rs:
// 295-306).
//
// Why a second kernel next to K1's Dict epilogue: K1 gives 8 threads one 1024-value block and
// writes a block's output as 8 x 128-byte row segments per wave-instruction; for 8/16-byte
// values that is 8-16 KiB of output per 8 threads and, on the lineitem string columns (92
// chunks x 64 blocks), only ~3 waves per CU.  Here a 256-thread workgroup owns BPW blocks:
// the blocks' packed words and the dictionary are staged in LDS once, and thread t produces
// outputs t, t+256, t+512, t+768 of each block, so every store wave-instruction writes 64
// consecutive values (512 B / 1 KiB contiguous, non-temporal) and the grid has one workgroup
// per BPW blocks.  The code of output i is unpack_single's (lane, row) -> one or two words of
// that lane from LDS.
#include "fl_unpack_impl.hpp"

namespace vxg {

namespace {

constexpr int kRowsThreads = 256;
constexpr int kRowsMaxW = 16;  // codes bit width (kDictFusedMaxW)

template <int VW> struct DVal;
template <> struct DVal<8> { using t = uint64_t; };
template <> struct DVal<16> { using t = uint4; };

template <int T, int VW, int BPW, bool LDSD, bool EXT>
__global__ __launch_bounds__(kRowsThreads) void dict_rows_kernel(ChunkTable tab, unsigned W) {
    using E = typename Fl<T>::E;
    using V = typename DVal<VW>::t;
    constexpr unsigned LANES = 1024 / T;
    const uint64_t g = blockIdx.x;
    uint32_t ci;
    if constexpr (EXT) {
        ci = ext_chunk_index(tab.ext, tab.n, g, [](const ChunkDev& d) { return d.first_group; });
    } else {
        uint32_t lo = 0, hi = tab.n;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tab.c[mid].first_group <= g) lo = mid; else hi = mid;
        }
        ci = lo;
    }
    const ChunkDev& c = EXT ? tab.ext[ci] : tab.c[ci];
    __shared__ __attribute__((aligned(16))) E s_packed[BPW * 128 * kRowsMaxW / sizeof(E)];
    __shared__ __attribute__((aligned(16))) uint8_t s_dict[LDSD ? kDictLdsBytes : 16];
    const unsigned tid = threadIdx.x;
    const uint64_t blk0 = (g - c.first_group) * BPW;
    const unsigned nb = unsigned(c.n_blocks - blk0 < uint64_t(BPW) ? c.n_blocks - blk0 : uint64_t(BPW));
    // stage the blocks' packed words (128 * W bytes each, 16-byte loads) and the dictionary
    const unsigned q16 = nb * 8 * W;
    for (unsigned q = tid; q < q16; q += kRowsThreads)
        reinterpret_cast<uint4*>(s_packed)[q] = reinterpret_cast<const uint4*>(c.packed + blk0 * (128ull * W))[q];
    const V* dict = static_cast<const V*>(c.dict);
    if constexpr (LDSD) {
        const unsigned n16 = unsigned((c.dict_len * VW + 15) / 16);
        for (unsigned q = tid; q < n16; q += kRowsThreads)
            reinterpret_cast<uint4*>(s_dict)[q] = static_cast<const uint4*>(c.dict)[q];
        dict = reinterpret_cast<const V*>(s_dict);
    }
    __syncthreads();
    V* __restrict__ out = static_cast<V*>(c.out);
    const RtRows<T> rows(W);
    bool oob = false;
    for (unsigned b = 0; b < nb; b++) {
        const E* __restrict__ pw = s_packed + b * (LANES * W);
        const int64_t base = int64_t((blk0 + b) * 1024) - int64_t(c.offset);
        const bool whole = base >= 0 && uint64_t(base) + 1024 <= c.len;  // uniform
#pragma unroll
        for (unsigned k = 0; k < 4; k++) {
            const int64_t o = base + int64_t(k * kRowsThreads + tid);
            if (!whole && (o < 0 || uint64_t(o) >= c.len)) continue;
            const uint64_t code = W ? uint64_t(rows.get(pw, k)) : 0;
            const bool bad = code >= c.dict_len;
            oob |= bad;
            nt_store(out + o, dict[bad ? 0 : code]);
        }
    }
    if (oob) __hip_atomic_fetch_or(tab.err, kErrTakeOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int T, int VW, int BPW, bool LDSD, bool EXT>
vxg_status launch_rows(ChunkTable tab, unsigned W, hipStream_t s) {
    ChunkDev* cs = tab.ext ? tab.host : tab.c;
    uint64_t groups = 0;
    for (uint32_t k = 0; k < tab.n; k++) {
        cs[k].first_group = groups;
        groups += (cs[k].n_blocks + BPW - 1) / BPW;
    }
    if (groups == 0) return VXG_OK;
    if (groups > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "array too long for one launch");
    hipLaunchKernelGGL((dict_rows_kernel<T, VW, BPW, LDSD, EXT>), dim3(unsigned(groups)), dim3(kRowsThreads), 0, s,
                       tab, W);
    return hip_check(hipGetLastError(), "dict_rows_kernel launch");
}

template <int T, int VW, int BPW>
vxg_status launch_rows_b(const ChunkTable& tab, unsigned W, bool lds, hipStream_t s) {
    if (tab.ext) return lds ? launch_rows<T, VW, BPW, true, true>(tab, W, s) : launch_rows<T, VW, BPW, false, true>(tab, W, s);
    return lds ? launch_rows<T, VW, BPW, true, false>(tab, W, s) : launch_rows<T, VW, BPW, false, false>(tab, W, s);
}

template <int T, int VW>
vxg_status launch_rows_t(const ChunkTable& tab, unsigned W, hipStream_t s) {
    const ChunkDev* cs = tab.ext ? tab.host : tab.c;
    bool lds = true;
    uint64_t max_dict = 0;
    for (uint32_t k = 0; k < tab.n; k++) {
        lds = lds && cs[k].dict_len * VW <= uint64_t(kDictLdsBytes) && (reinterpret_cast<uintptr_t>(cs[k].dict) & 15) == 0;
        max_dict = cs[k].dict_len * VW > max_dict ? cs[k].dict_len * VW : max_dict;
    }
    // a large dictionary is staged once per 8 blocks (its LDS copy costs as much as a block's
    // output at 8 KiB), a small one per block (more workgroups for small chunks)
    if (lds && max_dict > 1024) return launch_rows_b<T, VW, 8>(tab, W, lds, s);
    return launch_rows_b<T, VW, 1>(tab, W, lds, s);
}

}  // namespace

vxg_status launch_dict_rows(int T, int W, int vw, const ChunkTable& tab, hipStream_t s) {
    if (W < 0 || W > kRowsMaxW || W > T) return VXG_ERR_NOT_IMPLEMENTED;
    const unsigned w = unsigned(W);
#define VXG_ROWS(TT, VV) \
    if (T == TT && vw == VV) return launch_rows_t<TT, VV>(tab, w, s);
    VXG_ROWS(8, 8) VXG_ROWS(16, 8) VXG_ROWS(32, 8) VXG_ROWS(64, 8)
    VXG_ROWS(8, 16) VXG_ROWS(16, 16) VXG_ROWS(32, 16) VXG_ROWS(64, 16)
#undef VXG_ROWS
    return VXG_ERR_NOT_IMPLEMENTED;
}

}  // namespace vxg
