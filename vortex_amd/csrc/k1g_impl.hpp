// k1g_impl.hpp — K1g's device code (the job bodies and their dispatch), shared by the K1g
// launch (k1g.hip) and the plan launch that runs K1g jobs beside FSST decode tiles (fsst.hip).
// See k1g.hip for the design.
#pragma once

#include "fl_unpack_impl.hpp"
#include "k1g.hpp"
#include "runend_runs.hpp"

namespace vxg {

namespace {

constexpr int kGenThreads = 256;
// 32/64-bit numeric jobs decoded with the K1w store shape (gen_body_w); a -DVXG_K1G_WIDE=0 build
// keeps the thread-per-value body for A/B.
#ifndef VXG_K1G_WIDE
#define VXG_K1G_WIDE 1
#endif
constexpr bool kGenWideStores = VXG_K1G_WIDE;
constexpr uint32_t kGenPackedLds = 16 * 1024;  // staged packed words per workgroup

// FL_ORDER[i] (0, 4, 2, 6, 1, 5, 3, 7) is the 3-bit reversal of i
__device__ __forceinline__ uint32_t fl_order_rt(uint32_t i) { return ((i & 1u) << 2) | (i & 2u) | (i >> 2); }

template <typename O>
__device__ __forceinline__ void gen_store(O* p, const O& v) {
    if constexpr (sizeof(O) >= 4) nt_store(p, v);
    else gstore(p, v);
}

// arrow-array 53.2 make_view (as kernels.hip: len <= 12 inline, else prefix + buffer + offset);
// byte(j) = the dictionary's byte j (global memory or its LDS copy)
template <class Byte>
__device__ __forceinline__ uint4 vb_view(Byte byte, uint64_t start, uint32_t len, uint32_t bidx) {
    uint32_t w[3] = {0, 0, 0};
    if (len <= 12) {
        for (uint32_t j = 0; j < len; j++) w[j >> 2] |= uint32_t(byte(start + j)) << (8 * (j & 3));
        return make_uint4(len, w[0], w[1], w[2]);
    }
    for (uint32_t j = 0; j < 4; j++) w[0] |= uint32_t(byte(start + j)) << (8 * j);
    return make_uint4(len, w[0], bidx, uint32_t(start));
}

// The views of a VarBin dictionary (<= kGenVarBinDictMax entries) into s_views.  Bytes staged
// (gen_vb_heap_lds): every thread's offsets (entries tid + 256 k, clamped) and dictionary bytes
// are requested before any is used -- one memory round trip -- then the bytes go to s_vbh and,
// after a barrier, the views are built from LDS.  Otherwise the views read the bytes from global
// memory (a second, dependent round trip).
template <class Off>
__device__ __forceinline__ void vb_views(const GenChunk& gc, uint64_t dict_len, uint4* s_views, uint8_t* s_vbh, bool hl,
                                         uint32_t* err) {
    constexpr int KO = int(kGenVarBinDictMax / kGenThreads), KB = int(kGenVarBinHeapLds / kGenThreads);
    const uint32_t tid = threadIdx.x;
    const Off* const offs = static_cast<const Off*>(gc.vb_offs);
    uint64_t oa[KO], oe[KO];
#pragma unroll
    for (int k = 0; k < KO; k++) {
        const uint64_t i = tid + uint64_t(kGenThreads) * k, ic = i < dict_len ? i : 0;
        oa[k] = gload(offs + ic);
        oe[k] = gload(offs + ic + 1);
    }
    auto build = [&](auto byte) {
#pragma unroll
        for (int k = 0; k < KO; k++) {
            const uint64_t i = tid + uint64_t(kGenThreads) * k;
            if (i >= dict_len) continue;
            if (oa[k] > oe[k] || oe[k] > gc.vb_bytes) {  // malformed offsets: zero view + error bit
                __hip_atomic_fetch_or(err, kErrVarBin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_views[i] = make_uint4(0, 0, 0, 0);
            } else {
                s_views[i] = vb_view(byte, oa[k], uint32_t(oe[k] - oa[k]), gc.vb_bidx);
            }
        }
    };
    if (hl) {
        uint8_t hb[KB];
#pragma unroll
        for (int k = 0; k < KB; k++) {
            const uint64_t b = tid + uint64_t(kGenThreads) * k;
            hb[k] = b < gc.vb_bytes ? gload(gc.vb_src + b) : uint8_t(0);
        }
#pragma unroll
        for (int k = 0; k < KB; k++)
            if (tid + uint64_t(kGenThreads) * k < gc.vb_bytes) s_vbh[tid + kGenThreads * k] = hb[k];
        __syncthreads();
        build([&](uint64_t j) { return s_vbh[j]; });
    } else {
        build([&](uint64_t j) { return gload(gc.vb_src + j); });
    }
}

template <int T, Epi EPI, int VW, bool VB = false>
__device__ __forceinline__ void gen_body(const GenChunk& gc, uint64_t g, uint8_t* lds, uint32_t dict_off, bool dict_lds,
                                         uint32_t* err) {
    using E = typename Fl<T>::E;
    using O = typename EpiOut<T, EPI, VW>::type;
    constexpr uint32_t LANES = 1024 / T;
    const ChunkDev& c = gc.d;
    const uint32_t W = gc.W, tid = threadIdx.x;
    const uint64_t blk0 = (g - c.first_group) * gc.bpw;
    const uint32_t nb = uint32_t(c.n_blocks - blk0 < uint64_t(gc.bpw) ? c.n_blocks - blk0 : uint64_t(gc.bpw));
    E* const s_packed = reinterpret_cast<E*>(lds);
    const uint32_t q16 = nb * 8 * W;
    for (uint32_t q = tid; q < q16; q += kGenThreads)
        reinterpret_cast<uint4*>(s_packed)[q] = gload(reinterpret_cast<const uint4*>(c.packed + blk0 * (128ull * W)) + q);
    EpiParams ep;
    ep.reference = c.reference;
    ep.shift = c.shift;
    ep.alp_a = c.alp_a;
    ep.alp_b = c.alp_b;
    ep.dict = c.dict;
    ep.dict_len = c.dict_len;
    ep.err = err;
    if constexpr (VB) {
        static_assert(EPI == Epi::Dict && VW == 16, "VarBin dictionaries are string views");
        // this workgroup's share of the dictionary bytes -> the output data buffer
        const uint64_t ng = (c.n_blocks + gc.bpw - 1) / gc.bpw, lg = g - c.first_group;
        const uint64_t per = (gc.vb_bytes + ng - 1) / ng;
        const uint64_t b1 = (lg + 1) * per < gc.vb_bytes ? (lg + 1) * per : gc.vb_bytes;
        for (uint64_t b = lg * per + tid; b < b1; b += kGenThreads) gstore(gc.vb_dst + b, gload(gc.vb_src + b));
        // the dictionary's views, in LDS (offsets width: a uniform switch outside the loads)
        uint4* const s_views = reinterpret_cast<uint4*>(lds + dict_off);
        uint8_t* const s_vbh = lds + dict_off + 16 * c.dict_len;
        const bool hl = gen_vb_heap_lds(c.dict_len, gc.vb_bytes);
        switch (gc.vb_offs_width) {  // VarBin offsets are non-negative: signedness does not matter
        case 1: vb_views<uint8_t>(gc, c.dict_len, s_views, s_vbh, hl, err); break;
        case 2: vb_views<uint16_t>(gc, c.dict_len, s_views, s_vbh, hl, err); break;
        case 4: vb_views<uint32_t>(gc, c.dict_len, s_views, s_vbh, hl, err); break;
        default: vb_views<uint64_t>(gc, c.dict_len, s_views, s_vbh, hl, err); break;
        }
        ep.dict = s_views;
        ep.dict_lds = true;
    } else if constexpr (EPI == Epi::Dict) {
        if (dict_lds) {
            uint8_t* const s_dict = lds + dict_off;
            const uint32_t n16 = uint32_t((c.dict_len * VW + 15) / 16);
            for (uint32_t q = tid; q < n16; q += kGenThreads)
                reinterpret_cast<uint4*>(s_dict)[q] = gload(static_cast<const uint4*>(c.dict) + q);
            ep.dict = s_dict;
            ep.dict_lds = true;
        }
    }
    __syncthreads();
    O* __restrict__ out = static_cast<O*>(c.out);
    const RtRows<T> rows(W);
    bool oob = false;
    for (uint32_t b = 0; b < nb; b++) {
        const E* __restrict__ pw = s_packed + b * (LANES * W);
        const int64_t base = int64_t((blk0 + b) * 1024) - int64_t(c.offset);
        if (base >= 0 && uint64_t(base) + 1024 <= c.len) {  // whole block inside the array (uniform)
            O* __restrict__ ob = out + base + threadIdx.x;
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const E v = W ? rows.get(pw, k) : E(0);
                gen_store(ob + k * kGenThreads, apply_epi<T, EPI, VW>(v, ep, oob));
            }
        } else {
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const int64_t o = base + int64_t(k * kGenThreads + tid);
                if (o < 0 || uint64_t(o) >= c.len) continue;
                const E v = W ? rows.get(pw, k) : E(0);
                gen_store(out + o, apply_epi<T, EPI, VW>(v, ep, oob));
            }
        }
    }
    if constexpr (EPI == Epi::Dict)
        if (oob) __hip_atomic_fetch_or(err, kErrTakeOOB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The K1w store shape with a runtime width (round 6) for the 32/64-bit numeric kinds: the
// staged blocks are decoded one per wave (wave v takes blocks v, v + 4, ...); in store k lane
// group gq (8 lanes) produces the row whose 128 output bytes are slot 8k + gq of the block and
// lane t its 16-byte slice, funnel-shifted out of the two LDS word rows holding it -- every store
// instruction writes 1 KiB contiguous (K1w, fl_unpack_impl.hpp kw_block / kw_extract; there W is
// a template parameter).  The thread-per-value body (gen_body) stores 256 or 512 bytes per
// instruction and reads LDS per value.  Word row w0 + 1 of a block's last row may be the next
// block's or the stage's slack row (launch_k1_generic sizes the LDS with 128 bytes of slack): its
// bits are masked off.
template <int T>
__device__ __forceinline__ Vec16<T> kw_extract_rt(const uint8_t* blk, int r, int t, uint32_t W) {
    using U = typename Fl<T>::U;
    constexpr int NV = Vec16<T>::NV;
    const int start = r * int(W), w0 = start / T, sh = start % T;
    const Vec16<T> lo = load16<T>(blk + w0 * 128 + 16 * t);
    const Vec16<T> hi = load16<T>(blk + (w0 + 1) * 128 + 16 * t);
    const int cur = T - sh;  // bits of the value held by word w0
    const int nlo = cur < int(W) ? cur : int(W), nhi = int(W) - nlo;
    const U mlo = Fl<T>::rep(kw_mask<U>(nlo)), mhi = Fl<T>::rep(kw_mask<U>(nhi));
    const int hs = cur & (int(8 * sizeof(U)) - 1);  // == cur whenever mhi != 0
    Vec16<T> v;
#pragma unroll
    for (int k = 0; k < NV; k++) v.w[k] = ((lo.w[k] >> sh) & mlo) | ((hi.w[k] & mhi) << hs);
    return v;
}

template <int T, Epi EPI>
__device__ __forceinline__ void gen_body_w(const GenChunk& gc, uint64_t g, uint8_t* lds, uint32_t* err) {
    using E = typename Fl<T>::E;
    using O = typename EpiOut<T, EPI, 0>::type;
    constexpr int EPV = 16 / int(sizeof(E));
    const ChunkDev& c = gc.d;
    const uint32_t W = gc.W, tid = threadIdx.x;
    const uint64_t blk0 = (g - c.first_group) * gc.bpw;
    const uint32_t nb = uint32_t(c.n_blocks - blk0 < uint64_t(gc.bpw) ? c.n_blocks - blk0 : uint64_t(gc.bpw));
    const uint32_t q16 = nb * 8 * W;
    for (uint32_t q = tid; q < q16; q += kGenThreads)
        reinterpret_cast<uint4*>(lds)[q] = gload(reinterpret_cast<const uint4*>(c.packed + blk0 * (128ull * W)) + q);
    EpiParams ep;
    ep.reference = c.reference;
    ep.shift = c.shift;
    ep.alp_a = c.alp_a;
    ep.alp_b = c.alp_b;
    ep.err = err;
    __syncthreads();
    O* __restrict__ out = static_cast<O*>(c.out);
    const bool aligned = (reinterpret_cast<uintptr_t>(c.out) & 15) == 0;
    const int lane = int(tid & 63), gq = lane >> 3, t = lane & 7;
    bool oob = false;
    for (uint32_t b = tid >> 6; b < nb; b += kGenThreads / 64) {  // wave-uniform
        const uint8_t* pk = lds + b * (128 * W);
        const uint64_t blk = blk0 + b;
        const int64_t out_base = int64_t(blk * 1024) - int64_t(c.offset);
        const bool full = c.offset == 0 && (blk + 1) * 1024 <= c.len && aligned;
#pragma unroll 2  // (fully unrolled, the hoisted LDS reads took 101 VGPRs: 4 waves per SIMD)
        for (int k = 0; k < T / 8; k++) {
            const int q = 8 * k + gq;
            const Vec16<T> v = W ? kw_extract_rt<T>(pk, kw_row<T>(q), t, W) : Vec16<T>{};
            const int idx = q * (1024 / T) + t * EPV;  // element index of the slice in the block
            if (full) {
                O* dst = out + (out_base + idx);
                if constexpr (EPI == Epi::Plain) {
                    store_bytes<16, kOutNT>(reinterpret_cast<uint8_t*>(dst), v.w);
                } else {
                    O o[EPV];
#pragma unroll
                    for (int j = 0; j < EPV; j++) o[j] = apply_epi<T, EPI, 0>(v.elem(j), ep, oob);
                    store_bytes<EPV * int(sizeof(O)), kOutNT>(reinterpret_cast<uint8_t*>(dst), o);
                }
            } else {
#pragma unroll
                for (int j = 0; j < EPV; j++) {
                    const int64_t o = out_base + idx + j;
                    if (o >= 0 && uint64_t(o) < c.len) gstore(out + o, apply_epi<T, EPI, 0>(v.elem(j), ep, oob));
                }
            }
        }
    }
}

// kinds: T index ti (8, 16, 32, 64 -> 0..3); Plain/For/ForZigZag 3 ti + e (0..11); AlpF32 12;
// AlpF64 13; Dict 14 + 5 ti + value-width index (1, 2, 4, 8, 16 -> 0..4) (14..33); Dict over a
// VarBin dictionary 34 + ti (34..37); RunEnd short runs 38 + value-width index (38..42)
constexpr int kGenKinds = 43;

template <int K>
__device__ __forceinline__ void gen_dispatch_one(const GenChunk& gc, uint64_t g, uint8_t* lds, uint32_t doff, bool dl,
                                                 uint32_t* err) {
    constexpr int Ts[4] = {8, 16, 32, 64};
    constexpr int VWs[5] = {1, 2, 4, 8, 16};
    if constexpr (K < 12) {
        constexpr Epi e = K % 3 == 0 ? Epi::Plain : (K % 3 == 1 ? Epi::For : Epi::ForZigZag);
        if constexpr (K >= 6 && kGenWideStores) gen_body_w<Ts[K / 3], e>(gc, g, lds, err);  // T = 32, 64
        else gen_body<Ts[K / 3], e, 0>(gc, g, lds, doff, dl, err);
    } else if constexpr (K == 12) {
        if constexpr (kGenWideStores) gen_body_w<32, Epi::AlpF32>(gc, g, lds, err);
        else gen_body<32, Epi::AlpF32, 0>(gc, g, lds, doff, dl, err);
    } else if constexpr (K == 13) {
        if constexpr (kGenWideStores) gen_body_w<64, Epi::AlpF64>(gc, g, lds, err);
        else gen_body<64, Epi::AlpF64, 0>(gc, g, lds, doff, dl, err);
    } else if constexpr (K < 34) {
        gen_body<Ts[(K - 14) / 5], Epi::Dict, VWs[(K - 14) % 5]>(gc, g, lds, doff, dl, err);
    } else if constexpr (K < 38) {
        gen_body<Ts[K - 34], Epi::Dict, 16, true>(gc, g, lds, doff, dl, err);
    } else {
        using V = std::conditional_t<
            VWs[K - 38] == 1, uint8_t,
            std::conditional_t<VWs[K - 38] == 2, uint16_t,
                               std::conditional_t<VWs[K - 38] == 4, uint32_t,
                                                  std::conditional_t<VWs[K - 38] == 8, uint64_t, uint4>>>>;
        RunEndChunk rc = gc.re;
        rc.first_group = gc.d.first_group;
        runend_runs_body<V>(rc, g, err, lds);
    }
}

// The job's body: a switch (one jump-table dispatch; a fold over 43 compares cost the late kinds
// -- VarBin dictionaries, RunEnd -- ~80 scalar instructions per wave).
__device__ __forceinline__ void gen_dispatch(int kind, const GenChunk& gc, uint64_t g, uint8_t* lds, uint32_t doff, bool dl,
                                             uint32_t* err) {
    // a padded table (launch_k1_jobs: every job as many workgroups as the largest): the
    // workgroups past a job's own have nothing to do
    const uint64_t lg = g - gc.d.first_group;
    const uint64_t own = kind >= 38 ? (gc.re.n_runs + kRunEndRunsPerGroup - 1) / kRunEndRunsPerGroup
                                    : (gc.d.n_blocks + gc.bpw - 1) / (gc.bpw ? gc.bpw : 1);
    if (lg >= own) return;
#define VXG_K1G_CASE(K) \
    case K: gen_dispatch_one<K>(gc, g, lds, doff, dl, err); break;
    switch (kind) {
        VXG_K1G_CASE(0) VXG_K1G_CASE(1) VXG_K1G_CASE(2) VXG_K1G_CASE(3) VXG_K1G_CASE(4) VXG_K1G_CASE(5)
        VXG_K1G_CASE(6) VXG_K1G_CASE(7) VXG_K1G_CASE(8) VXG_K1G_CASE(9) VXG_K1G_CASE(10) VXG_K1G_CASE(11)
        VXG_K1G_CASE(12) VXG_K1G_CASE(13) VXG_K1G_CASE(14) VXG_K1G_CASE(15) VXG_K1G_CASE(16) VXG_K1G_CASE(17)
        VXG_K1G_CASE(18) VXG_K1G_CASE(19) VXG_K1G_CASE(20) VXG_K1G_CASE(21) VXG_K1G_CASE(22) VXG_K1G_CASE(23)
        VXG_K1G_CASE(24) VXG_K1G_CASE(25) VXG_K1G_CASE(26) VXG_K1G_CASE(27) VXG_K1G_CASE(28) VXG_K1G_CASE(29)
        VXG_K1G_CASE(30) VXG_K1G_CASE(31) VXG_K1G_CASE(32) VXG_K1G_CASE(33) VXG_K1G_CASE(34) VXG_K1G_CASE(35)
        VXG_K1G_CASE(36) VXG_K1G_CASE(37) VXG_K1G_CASE(38) VXG_K1G_CASE(39) VXG_K1G_CASE(40) VXG_K1G_CASE(41)
        VXG_K1G_CASE(42)
    default: break;
    }
#undef VXG_K1G_CASE
}
static_assert(kGenKinds == 43, "gen_dispatch's switch lists every kind");

}  // namespace

}  // namespace vxg
