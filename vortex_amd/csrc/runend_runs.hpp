// runend_runs.hpp — K8r body: RunEnd expansion of chunks with short runs, 1024 runs per
// 256-thread workgroup (runend/compress.rs:115-148).  Shared by the K8r launch (kernels.hip) and
// the K1g launch of a plan batch (k1g.hip), which hands it LDS of its own.
#pragma once

#include "fl_unpack_impl.hpp"
#include "intcol.hpp"

namespace vxg {

// Short runs (C5's l_orderkey: 1-7 rows per order): a workgroup takes 1024 consecutive RUNS
// (not an output span), so no search is needed: thread t reads ends[r] and values[r] of runs
// r0 + 4 t + k (k < 4) in one round trip -- from plain buffers, or unpacked in place from
// patch-free [FoR](BitPacked) children (fastlanes unpack_single, bitpacking/compress.rs:295-306),
// so the children are never materialised.  Run r covers the trimmed range
// [min(ends[r-1] - offset, len), min(ends[r] - offset, len)) (runend_decode_primitive,
// runend/compress.rs:138-146; the previous end is the thread's own, its left lane's, or the
// previous wave's last, through LDS), and the workgroup's runs cover
// one contiguous output range.  That range is expanded in windows of 4096 outputs: each
// non-empty run writes its index at its first output (a run head), a max-scan fills the window,
// and the window is written with coalesced non-temporal stores (the run carried into the next
// window is the last scanned one).  Chunks whose runs average > kRunEndShortRun rows take the
// span kernel above.
template <typename V>
__device__ __forceinline__ V runend_value(const IntCol& c, uint64_t r) {
    if constexpr (sizeof(V) == 4 || sizeof(V) == 8) {
        if (c.packed) return V(uint64_t(intcol_get(c, r)));  // low bytes: the value's bits
    }
    return gload(static_cast<const V*>(c.p) + r);
}

constexpr int kRunsThreads = 256;
constexpr int kRunsSpan = 4096;  // outputs per expansion window
// Run heads are u16 entries padded by one every 16 (entry p at p + p / 16): thread t's 16
// consecutive entries of the max-scan sit 17 entries apart from thread t + 1's, so the scan's
// reads and writes hit 32 distinct banks (unpadded, 32-byte strides put 8 lanes on one bank).
constexpr int kRunsHeadSlots = kRunsSpan + kRunsSpan / 16;
__device__ __forceinline__ int runs_pad(int p) { return p + (p >> 4); }
// LDS of one workgroup: run heads (u16, padded; 8.5 KiB, also the staging area of the ends'
// packed words and the decoded ends), run values (kRunEndRunsPerGroup V; also the staging area
// of the values' packed words), scratch
template <typename V>
constexpr size_t runs_lds_bytes() {
    return kRunsHeadSlots * 2 + kRunEndRunsPerGroup * sizeof(V) + 128;
}

// A child read block-wise: a packed [FoR](BitPacked) u32/u64 column (slice offset 0) whose block
// the workgroup's 1024 runs are -- staged in LDS with coalesced 16-byte loads (no per-element
// unpack_single: its index math and two global loads per element were most of K8r's VALU).
__device__ __forceinline__ bool runs_blockwise(const IntCol& c, size_t stage_bytes) {
    return c.packed && c.offset == 0 && (c.width == 4 || c.width == 8) && size_t(128) * c.W <= stage_bytes;
}
__device__ __forceinline__ void runs_stage(const IntCol& c, uint64_t blk, uint8_t* s) {
    const uint32_t n16 = 8 * c.W;  // 128 * W bytes
    const uint4* src = reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(c.p) + blk * (128ull * c.W));
    for (uint32_t q = threadIdx.x; q < n16; q += kRunsThreads) reinterpret_cast<uint4*>(s)[q] = gload(src + q);
}
// values 256 k + threadIdx.x (k < 4) of the staged block, FoR applied, as intcol_get returns them
__device__ __forceinline__ void runs_extract(const IntCol& c, const uint8_t* s, int64_t out[4]) {
    if (c.width == 8) {
        const RtRows<64> rows(c.W);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t v = c.W ? rows.get(reinterpret_cast<const uint64_t*>(s), uint32_t(k)) : 0;
            out[k] = int64_t((v << c.shift) + c.reference);
        }
    } else {
        const RtRows<32> rows(c.W);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t v = c.W ? rows.get(reinterpret_cast<const uint32_t*>(s), uint32_t(k)) : 0;
            const uint32_t r = uint32_t(v << c.shift) + uint32_t(c.reference);
            out[k] = c.sgn ? int64_t(int32_t(r)) : int64_t(r);
        }
    }
}

// Workgroup g of the launch expands its 1024 runs of chunk c (c.first_group = its first
// workgroup).  `lds` = runs_lds_bytes<V>() bytes, 16-byte aligned.
template <typename V>
__device__ __forceinline__ void runend_runs_body(const RunEndChunk& c, uint64_t g, uint32_t* err, uint8_t* lds) {
    constexpr int kBlock = kRunsThreads;
    constexpr int SPAN = kRunsSpan, PER = SPAN / kBlock, RPG = int(kRunEndRunsPerGroup), RPT = RPG / kBlock;
    // run heads as 16-bit run indices (<= 1024 runs per workgroup): 8 KiB instead of 16, so the
    // LDS of a u64 expansion (16.6 KiB) allows 8 workgroups per CU instead of 6
    static_assert(RPG < 65536, "run index must fit 16 bits");
    static_assert(RPG == 4 * kBlock && RPT == 4, "one FastLanes block of runs per workgroup, 4 per thread");
    constexpr size_t kHeadBytes = size_t(kRunsHeadSlots) * 2;
    uint16_t* const s_head = reinterpret_cast<uint16_t*>(lds);
    V* const s_val = reinterpret_cast<V*>(lds + kHeadBytes);
    uint8_t* const misc = lds + kHeadBytes + RPG * sizeof(V);
    uint64_t* const s_wlast = reinterpret_cast<uint64_t*>(misc);           // kBlock / 64
    uint64_t& s_lo = reinterpret_cast<uint64_t*>(misc)[4];
    uint64_t& s_hi = reinterpret_cast<uint64_t*>(misc)[5];
    uint32_t* const s_wmax = reinterpret_cast<uint32_t*>(misc + 48);       // kBlock / 64
    uint32_t& s_carry = reinterpret_cast<uint32_t*>(misc + 48)[4];
    const int tid = threadIdx.x;
    const uint64_t r0 = (g - c.first_group) * uint64_t(RPG);
    const int nr = int(c.n_runs - r0 < uint64_t(RPG) ? c.n_runs - r0 : uint64_t(RPG));
    auto trim = [&](uint64_t e) { return e > c.offset ? (e - c.offset < c.len ? e - c.offset : c.len) : 0; };
    // thread t owns runs RPT t .. RPT t + RPT - 1; every load of the round trip issued before
    // any is used
    uint64_t e[RPT];
    V v[RPT];
    const uint64_t eprev = tid == 0 && r0 > 0 ? uint64_t(intcol_get(c.ends, r0 - 1)) : 0;
    // block-wise children (uniform): the ends' words staged in the head area, the values' in the
    // value area, extracted (value 256 k + t per thread), then exchanged through LDS into
    // run order -- ends as u64 in the head area, values straight into s_val
    const bool bwe = runs_blockwise(c.ends, kHeadBytes);
    const bool bwv = (sizeof(V) == 4 || sizeof(V) == 8) && runs_blockwise(c.values, RPG * sizeof(V)) &&
                     c.values.width == int(sizeof(V));
    if (bwe || bwv) {
        const uint64_t blk = r0 / uint64_t(RPG);
        if (bwe) runs_stage(c.ends, blk, lds);
        if (bwv) runs_stage(c.values, blk, reinterpret_cast<uint8_t*>(s_val));
        __syncthreads();
        int64_t xe[4], xv[4];
        if (bwe) runs_extract(c.ends, lds, xe);
        if (bwv) runs_extract(c.values, reinterpret_cast<const uint8_t*>(s_val), xv);
        __syncthreads();
        uint64_t* const s_e64 = reinterpret_cast<uint64_t*>(lds);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (bwe) s_e64[tid + kBlock * k] = uint64_t(xe[k]);
            if (bwv) {
                V x;
                const uint64_t u = uint64_t(xv[k]);
                __builtin_memcpy(&x, &u, sizeof(V));  // low bytes: the value's bits
                s_val[tid + kBlock * k] = x;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < RPT; k++) {
        const int i = RPT * tid + k;
        const uint64_t rr = r0 + uint64_t(i < nr ? i : 0);
        e[k] = bwe ? reinterpret_cast<const uint64_t*>(lds)[RPT * tid + k] : uint64_t(intcol_get(c.ends, rr));
        if (!bwv) v[k] = runend_value<V>(c.values, rr);
    }
    uint64_t en[RPT], st[RPT];
#pragma unroll
    for (int k = 0; k < RPT; k++) {
        const int i = RPT * tid + k;
        en[k] = trim(e[k]);
        if (i < nr) {
            if (!bwv) s_val[i] = v[k];
            if (i == nr - 1) s_hi = en[k];
            if (r0 + uint64_t(i) + 1 == c.n_runs && en[k] < c.len)  // the ends do not reach the end of the array
                __hip_atomic_fetch_or(err, kErrRunEnd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // a run starts at the previous run's trimmed end: in this thread, in lane t - 1, or in the
    // previous wave's last lane
    const uint64_t left = __shfl_up(en[RPT - 1], 1, 64);
    if ((tid & 63) == 63) s_wlast[tid >> 6] = en[RPT - 1];
    if (tid == 0) s_lo = r0 > 0 ? trim(eprev) : 0;
    __syncthreads();
    const uint64_t lo = s_lo, hi = s_hi;
    st[0] = tid == 0 ? lo : ((tid & 63) == 0 ? s_wlast[(tid >> 6) - 1] : left);
#pragma unroll
    for (int k = 1; k < RPT; k++) st[k] = en[k - 1];
#pragma unroll
    for (int k = 0; k < RPT; k++)
        if (RPT * tid + k >= nr) st[k] = en[k] = 0;  // no run here
    V* __restrict__ out = static_cast<V*>(c.out);
    uint32_t carry = 0;
    for (uint64_t wb = lo; wb < hi; wb += SPAN) {
        const int wn = int(hi - wb < uint64_t(SPAN) ? hi - wb : uint64_t(SPAN));
        for (int q = tid; q < kRunsHeadSlots / 8; q += kBlock) reinterpret_cast<uint4*>(s_head)[q] = make_uint4(0, 0, 0, 0);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < RPT; k++)
            if (en[k] > st[k] && st[k] >= wb && st[k] < wb + uint64_t(wn))
                s_head[runs_pad(int(st[k] - wb))] = uint16_t(RPT * tid + k + 1);
        __syncthreads();
        // inclusive max-scan of s_head (thread t owns entries [PER t, PER t + PER)), seeded
        // with the run carried over from the previous window
        uint32_t vv[PER];
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < PER; k++) {
            m = max(m, uint32_t(s_head[tid * (PER + 1) + k]));
            vv[k] = m;
        }
        uint32_t x = m;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if ((tid & 63) >= d) x = max(x, y);
        }
        if ((tid & 63) == 63) s_wmax[tid >> 6] = x;
        __syncthreads();
        uint32_t before = __shfl_up(x, 1, 64);
        if ((tid & 63) == 0) before = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; w++)
            if (w < (tid >> 6)) before = max(before, s_wmax[w]);
        before = max(before, carry);
#pragma unroll
        for (int k = 0; k < PER; k++) s_head[tid * (PER + 1) + k] = uint16_t(max(vv[k], before));
        __syncthreads();
        if constexpr (sizeof(V) == 4 || sizeof(V) == 8) {
            // two consecutive outputs per lane, one 8/16-byte store (half the per-output address
            // work of a VALU-bound loop; 1 KiB per store instruction for u64)
            using P = std::conditional_t<sizeof(V) == 8, uint4, uint64_t>;
            // pairs start at a 2V-aligned output (the window's first output alone if it is not)
            const int a = int((reinterpret_cast<uintptr_t>(out + wb) / sizeof(V)) & 1);
            if (a && tid == 0 && wn > 0) nt_store(out + wb, s_val[s_head[0] - 1]);
            for (int i = a + 2 * tid; i < wn; i += 2 * kBlock) {
                const V v0 = s_val[s_head[runs_pad(i)] - 1];
                if (i + 1 < wn) {
                    const V v1 = s_val[s_head[runs_pad(i + 1)] - 1];
                    P pv;
                    __builtin_memcpy(&pv, &v0, sizeof(V));
                    __builtin_memcpy(reinterpret_cast<uint8_t*>(&pv) + sizeof(V), &v1, sizeof(V));
                    nt_store(reinterpret_cast<P*>(out + wb + i), pv);
                } else {
                    nt_store(out + wb + i, v0);
                }
            }
        } else {
            for (int i = tid; i < wn; i += kBlock) nt_store(out + wb + i, s_val[s_head[runs_pad(i)] - 1]);
        }
        if (tid == 0) s_carry = s_head[runs_pad(wn - 1)];
        __syncthreads();
        carry = s_carry;
    }
}

}  // namespace vxg
