// capi.hip — the C ABI (include/vortex_gpu.h) and the canonicalize planner.
//
// The planner is the host-side mirror of the reference's dispatch: Array::into_canonical
// (vortex-array/src/canonical.rs:353-357) -> ArrayEncoding::canonicalize (encoding/mod.rs:53)
// -> per-encoding IntoCanonical.  Where the reference materialises one buffer per cascade
// level (e.g. ALP -> FoR -> BitPacked is 3-4 passes, SURVEY.md §3 stack B) the planner
// recognises the cascade and issues ONE fused K1 launch (+ tiny patch scatters); anything it
// does not recognise is decoded child-first into temporaries exactly like the reference.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <memory>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "encode_gpu.hpp"
#include "filter.hpp"
#include "k1g.hpp"
#include "take.hpp"
#include "vxg_internal.hpp"

struct vxg_ctx {
    vxg::Ctx c;
};

// Chunk tables travel as kernel arguments: they must fit the 4 KiB kernarg segment.
static_assert(sizeof(vxg::ChunkTable) <= 4096, "ChunkTable exceeds the kernarg limit");
static_assert(sizeof(vxg::FsstTable) <= 4096, "FsstTable exceeds the kernarg limit");
static_assert(sizeof(vxg::RunEndTable) <= 4096, "RunEndTable exceeds the kernarg limit");
static_assert(sizeof(vxg::VarBinTable) <= 4096, "VarBinTable exceeds the kernarg limit");

namespace vxg {

const float kF10f[11] = {1.0f, 10.0f, 100.0f, 1000.0f, 10000.0f, 100000.0f, 1000000.0f,
                         10000000.0f, 100000000.0f, 1000000000.0f, 10000000000.0f};
const float kIF10f[11] = {1.0f, 0.1f, 0.01f, 0.001f, 0.0001f, 0.00001f, 0.000001f,
                          0.0000001f, 0.00000001f, 0.000000001f, 0.0000000001f};
const double kF10d[24] = {
    1.0, 10.0, 100.0, 1000.0, 10000.0, 100000.0, 1000000.0, 10000000.0, 100000000.0,
    1000000000.0, 10000000000.0, 100000000000.0, 1000000000000.0, 10000000000000.0,
    100000000000000.0, 1000000000000000.0, 10000000000000000.0, 100000000000000000.0,
    1000000000000000000.0, 10000000000000000000.0, 100000000000000000000.0,
    1000000000000000000000.0, 10000000000000000000000.0, 100000000000000000000000.0};
const double kIF10d[24] = {
    1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001, 0.00000001, 0.000000001,
    0.0000000001, 0.00000000001, 0.000000000001, 0.0000000000001, 0.00000000000001,
    0.000000000000001, 0.0000000000000001, 0.00000000000000001, 0.000000000000000001,
    0.0000000000000000001, 0.00000000000000000001, 0.000000000000000000001,
    0.0000000000000000000001, 0.00000000000000000000001};

static thread_local std::string g_last_error;

vxg_status set_error(vxg_status s, const std::string& msg) {
    if (s != VXG_OK) g_last_error = msg;
    return s;
}

vxg_status hip_check(hipError_t e, const char* what) {
    if (e == hipSuccess) return VXG_OK;
    return set_error(e == hipErrorOutOfMemory ? VXG_ERR_OUT_OF_MEMORY : VXG_ERR_HIP,
                     std::string(what) + ": " + hipGetErrorString(e));
}

// K14 (dict_rows.hip) for 8/16-byte dictionary values; VXG_DICT_ROWS=0 selects K1's Dict
// epilogue instead (A/B measurements).
static bool dict_rows_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("VXG_DICT_ROWS");
        return !(e && e[0] == '0');
    }();
    return on;
}

// VXG_PLAN_VB_K1G=0 (read at every plan recording): an unbatched plan canonicalizes chunked
// Dict(VarBin) string columns with a views launch + K14 instead of one K1g launch (A/B).
static bool plan_vb_k1g() {
    const char* e = std::getenv("VXG_PLAN_VB_K1G");
    return !(e && e[0] == '0');
}

// VXG_FUSED_PATCHES=0 (read at every decode): ALP's outer patches take the separate scatter
// launch instead of the K1w launch (A/B measurements, parity tests of both paths).
static bool fused_patches_enabled() {
    const char* e = std::getenv("VXG_FUSED_PATCHES");
    return !(e && e[0] == '0');
}

thread_local bool g_k1w_wrote_patches = false;
thread_local Ctx* g_cur_ctx = nullptr;

Options default_options() {
    static const Options d = [] {
        Options o;
        if (const char* e = std::getenv("VXG_K1W_MIN_GROUPS")) o.k1w_min_groups = int64_t(std::strtoll(e, nullptr, 10));
        return o;
    }();
    return d;
}

void note_k1w_launch(uint32_t bpw, uint32_t bpw_max, uint64_t groups) {
    if (!g_cur_ctx) return;
    std::lock_guard<std::mutex> lk(g_cur_ctx->mu);
    LaunchStats& st = g_cur_ctx->st;
    st.k1w_min_bpw = st.k1w_launches == 0 ? bpw : std::min(st.k1w_min_bpw, bpw);
    st.k1w_max_bpw = st.k1w_launches == 0 ? bpw : std::max(st.k1w_max_bpw, bpw);
    st.k1w_launches++;
    st.k1w_last_bpw = bpw;
    st.k1w_last_bpw_max = bpw_max;
    st.k1w_last_groups = groups;
}

// launch_one's choice (fl_unpack_impl.hpp) for a kernel-argument table: K1w unless the launch is
// small enough for the row split (T = 32/64) or the K1_WAVE option / VXG_K1_WAVE says otherwise.
bool k1_takes_wave(int T, int W, Epi epi, uint64_t groups32) {
    const int mode = k1_wave_mode();
    const bool split = (T == 32 || T == 64) && W > 0 && groups32 < split_below_groups();
    return groups32 > 0 && (mode == 2 || (mode == 1 && !split && epi != Epi::Dict));
}

// K1 dispatch over the instantiation units.
vxg_status launch_fl_unpack(int T, int W, Epi epi, int vw, const ChunkTable& t, uint64_t g, hipStream_t s) {
    if (W < 0 || W > T) return set_error(VXG_ERR_INVALID_ARGUMENT, "bit width out of range");
    switch (epi) {
    case Epi::Plain:
    case Epi::For:
    case Epi::ForZigZag:
        switch (T) {
        case 8: return fl_plain_8(W, epi, t, g, s);
        case 16: return fl_plain_16(W, epi, t, g, s);
        case 32: return fl_plain_32(W, epi, t, g, s);
        case 64: return fl_plain_64(W, epi, t, g, s);
        }
        return set_error(VXG_ERR_INVALID_ARGUMENT, "bad FastLanes width");
    case Epi::AlpF32:
    case Epi::AlpF64:
        return fl_alp(T, W, epi, t, g, s);
    case Epi::Dict:
        if (W > kDictFusedMaxW) return VXG_ERR_NOT_IMPLEMENTED;
        // K14 for string dictionaries (16-byte views): 2.2-2.4x K1 on the lineitem columns;
        // 8-byte values stay on K1 (C3, 8 KiB dictionaries: K1 4 % faster, profiles/r02_*)
        if (vw == 16 && dict_rows_enabled()) return launch_dict_rows(T, W, vw, t, s);
        switch (vw) {
        case 1: return fl_dict_1(T, W, t, g, s);
        case 2: return fl_dict_2(T, W, t, g, s);
        case 4: return fl_dict_4(T, W, t, g, s);
        case 8: return fl_dict_8(T, W, t, g, s);
        case 16: return fl_dict_16(T, W, t, g, s);
        }
        return set_error(VXG_ERR_INVALID_ARGUMENT, "bad dictionary value width");
    }
    return VXG_ERR_INVALID_ARGUMENT;
}

}  // namespace vxg

using namespace vxg;

namespace {

#define VXG_TRY_S(expr)                       \
    do {                                      \
        vxg_status _s = (expr);               \
        if (_s != VXG_OK) return _s;          \
    } while (0)

// One K1 decode (a whole BitPacked-rooted cascade of one array or one chunk) and the kernel
// it needs.  Jobs with the same kernel share launches.
struct K1Job {
    int T, W;
    Epi epi;
    int vw;
    ChunkDev d;
    // a plan batch's Dict over a small VarBin dictionary: K1g builds the dictionary's views
    // (d.dict unused) and copies its bytes (vb.src -> vb.dst); only K1g runs such a job
    bool vb = false;
    VarBinChunk vbc{};
};

bool same_kernel(const K1Job& a, const K1Job& b) {
    return a.T == b.T && a.W == b.W && a.epi == b.epi && a.vw == b.vw && a.vb == b.vb;
}

// Output bytes below which a plan batch's kernel group goes to the one K1g launch instead of its
// own K1 launch (VXG_K1G_MAX_BYTES overrides; 0 disables K1g).  Round 5, C5 (same box, ms per
// step): 1 GPU 0.289 with 64 MiB (every numeric column in K1g: unbatched kept) vs 0.272 with
// 16 MiB (batched kept); 2-GPU shard 0.163 vs 0.145; 4-GPU shard 0.0715 vs 0.0784 (its 18 MB
// date-column group then leaves K1g); 8-GPU shard equal.  20 MiB sits between.
static uint64_t k1g_max_bytes() {
    static const uint64_t v = [] {
        const char* e = std::getenv("VXG_K1G_MAX_BYTES");
        return e ? uint64_t(std::strtoull(e, nullptr, 10)) : uint64_t(20) << 20;
    }();
    return v;
}

static int k1_out_width(const K1Job& j) {
    return j.epi == Epi::Dict ? j.vw : (j.epi == Epi::AlpF32 ? 4 : (j.epi == Epi::AlpF64 ? 8 : j.T / 8));
}

// Launch K1 jobs grouped by kernel (T, W, epilogue, value width), kArgChunks chunks per launch
// with the chunk table as the kernel argument (no device table, no upload, no host sync).
// While a plan is recorded (dt set), a group of any size is one launch over a device table, and
// (generic_small: a plan's batch) the groups whose output is small all share ONE K1g launch
// (k1g.hpp): a sharded scan's many small per-column kernels cost more in ramp, drain and graph
// edges than in data.
vxg_status launch_k1_jobs(std::vector<K1Job>& jobs, uint32_t* err, hipStream_t s, DevTables* dt = nullptr,
                          bool generic_small = false,
                          const std::vector<std::pair<int, RunEndChunk>>* gen_runs = nullptr,
                          const PatchCol* patch = nullptr, const FsstFused* fuse = nullptr) {
    std::stable_sort(jobs.begin(), jobs.end(), [](const K1Job& a, const K1Job& b) {
        return std::make_tuple(a.T, a.W, int(a.epi), a.vw, a.vb) < std::make_tuple(b.T, b.W, int(b.epi), b.vw, b.vb);
    });
    std::vector<const K1Job*> gen;  // jobs for the shared K1g launch
    // (VXG_PLAN_K1G_FIRST=1, read at every recording: a plan batch records its K1g launch before
    // the large groups' own launches -- A/B of the chain order)
    const char* kf = std::getenv("VXG_PLAN_K1G_FIRST");
    const bool k1g_first = generic_small && dt && kf && kf[0] == '1';
    std::vector<std::pair<size_t, size_t>> deferred;  // large groups launched after K1g
    auto launch_group = [&](size_t i, size_t j) -> vxg_status {
        size_t live = 0;
        for (size_t k = i; k < j; k++) live += jobs[k].d.n_blocks != 0;
        ChunkTable tab{};
        tab.err = err;
        if (patch && jobs.size() == 1) tab.patch = *patch;  // a single array's K1w (k1_takes_wave)
        ChunkDev* cs = tab.c;
        if (live > size_t(kArgChunks)) {  // only when dt is set
            if (live > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "too many chunks");
            VXG_TRY_S(dt->table(live, &tab.host, &tab.ext));
            cs = tab.host;
        }
        uint64_t groups = 0;
        for (size_t k = i; k < j; k++) {
            if (jobs[k].d.n_blocks == 0) continue;
            ChunkDev& c = cs[tab.n++];
            c = jobs[k].d;
            c.first_group = groups;
            groups += (c.n_blocks + 31) / 32;
        }
        if (groups > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "array too long for one launch");
        if (tab.n) return launch_fl_unpack(jobs[i].T, jobs[i].W, jobs[i].epi, jobs[i].vw, tab, groups, s);
        return VXG_OK;
    };
    size_t i = 0;
    while (i < jobs.size()) {
        size_t j = i, live = 0;
        uint64_t out_bytes = 0;
        while (j < jobs.size() && (dt || j - i < size_t(kArgChunks)) && same_kernel(jobs[i], jobs[j])) {
            live += jobs[j].d.n_blocks != 0;
            out_bytes += jobs[j].d.len * uint64_t(k1_out_width(jobs[j]));
            j++;
        }
        if (jobs[i].vb || (dt && generic_small && out_bytes < k1g_max_bytes() &&
                           gen_kind(jobs[i].T, int(jobs[i].epi), jobs[i].vw) >= 0)) {
            if (!dt) return set_error(VXG_ERR_INVALID_ARGUMENT, "VarBin-dictionary K1 jobs need a plan");
            for (size_t k = i; k < j; k++)
                if (jobs[k].d.n_blocks) gen.push_back(&jobs[k]);
            i = j;
            continue;
        }
        (void)live;
        if (k1g_first) deferred.emplace_back(i, j);
        else VXG_TRY_S(launch_group(i, j));
        i = j;
    }
    const size_t n_runs = gen_runs ? gen_runs->size() : 0;
    if (!gen.empty() || n_runs || (fuse && fuse->valid)) {
        if (!dt) return set_error(VXG_ERR_INVALID_ARGUMENT, "internal: K1g launch outside a plan");
        if (gen.size() + n_runs > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "too many chunks");
        GenChunk* host;
        const GenChunk* ext;
        VXG_TRY_S(dt->table(gen.size() + n_runs, &host, &ext));
        uint64_t groups = 0;
        bool dict_lds = true;
        uint32_t packed_bytes = 0, dict_bytes = 0, runs_bytes = 0;
        // a launch of string-dictionary jobs alone (an unbatched plan's chunked Dict(VarBin)
        // column): one FastLanes block of codes per workgroup (gen_vb_bpw)
        const bool vb_alone = n_runs == 0 && !(fuse && fuse->valid) &&
                              std::all_of(gen.begin(), gen.end(), [](const K1Job* jp) { return jp->vb; });
        uint64_t gen_blocks = 0;
        for (const K1Job* jp : gen) gen_blocks += jp->d.n_blocks;
        const uint32_t bpw_cap = gen_bpw_cap(gen_blocks);
        for (size_t k = 0; k < gen.size(); k++) {
            const K1Job& jb = *gen[k];
            GenChunk& g = host[k];
            g.d = jb.d;
            g.kind = uint32_t(gen_kind(jb.T, int(jb.epi), jb.vw, jb.vb));
            g.W = uint32_t(jb.W);
            g.bpw = jb.vb ? gen_vb_bpw(jb.T, jb.W, vb_alone, bpw_cap) : gen_bpw(jb.T, jb.W, bpw_cap);
            g.d.first_group = groups;
            groups += (jb.d.n_blocks + g.bpw - 1) / g.bpw;
            packed_bytes = std::max(packed_bytes, g.bpw * 128u * uint32_t(jb.W));
            if (jb.vb) {
                dict_bytes = std::max(dict_bytes, gen_vb_stage_bytes(jb.d.dict_len, jb.vbc.bytes));
                g.vb_src = jb.vbc.src;
                g.vb_offs = jb.vbc.offsets;
                g.vb_offs_width = jb.vbc.offs_width;
                g.vb_dst = jb.vbc.dst;
                g.vb_bytes = jb.vbc.bytes;
                g.vb_bidx = jb.vbc.bidx;
            } else if (jb.epi == Epi::Dict) {
                dict_lds = dict_lds && jb.d.dict_len * uint64_t(jb.vw) <= uint64_t(kDictLdsBytes) &&
                           (reinterpret_cast<uintptr_t>(jb.d.dict) & 15) == 0;
            }
        }
        if (dict_lds)  // every plain Dict job stages its dictionary
            for (const K1Job* jp : gen)
                if (jp->epi == Epi::Dict && !jp->vb)
                    dict_bytes = std::max(dict_bytes, uint32_t((jp->d.dict_len * uint64_t(jp->vw) + 15) & ~15ull));
        for (size_t k = 0; k < n_runs; k++) {  // short-run RunEnd expansions (runend_runs.hpp)
            const auto& [w, r] = (*gen_runs)[k];
            GenChunk& g = host[gen.size() + k];
            g.kind = uint32_t(gen_runs_kind(w));
            g.re = r;
            g.d.first_group = groups;
            g.d.n_blocks = r.n_runs;  // (unused by the body; keeps the entry self-describing)
            groups += (r.n_runs + kRunEndRunsPerGroup - 1) / kRunEndRunsPerGroup;
            runs_bytes = std::max(runs_bytes, gen_runs_lds_bytes(w));
        }
        std::vector<uint64_t> cnt(gen.size() + n_runs);  // workgroups per job (direct job lookup when equal)
        for (size_t k = 0; k < cnt.size(); k++)
            cnt[k] = (k + 1 < cnt.size() ? host[k + 1].d.first_group : groups) - host[k].d.first_group;
        uint64_t gpe = common_groups(cnt.data(), cnt.size());
        // Nearly equal counts (C5's RunEnd chunks: 16 or 17 workgroups; every column's last chunk
        // smaller): every job padded to the largest count when that adds <= 1/10 idle workgroups,
        // so a workgroup finds its job by one division instead of a wave-wide search over the
        // table (one or more dependent round trips before its loads; gen_dispatch returns at once
        // on a padding workgroup).  VXG_K1G_PAD=0 (read at every recording) keeps the search.
        const char* pe = std::getenv("VXG_K1G_PAD");
        if (!gpe && cnt.size() > 1 && !(pe && pe[0] == '0')) {
            const uint64_t m = *std::max_element(cnt.begin(), cnt.end());
            if (m * cnt.size() - groups <= groups / 10) {
                for (size_t k = 0; k < cnt.size(); k++) host[k].d.first_group = k * m;
                groups = m * cnt.size();
                gpe = m;
            }
        }
        VXG_TRY_S(launch_k1_generic(ext, uint32_t(gen.size() + n_runs), groups, dict_lds, packed_bytes, dict_bytes,
                                    runs_bytes, err, s, gpe, fuse));
    }
    for (const auto& [a, b] : deferred) VXG_TRY_S(launch_group(a, b));
    return VXG_OK;
}

#define VXG_TRY(expr)                         \
    do {                                      \
        vxg_status _s = (expr);               \
        if (_s != VXG_OK) return _s;          \
    } while (0)

inline hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }

vxg_status use_device(vxg_ctx* ctx) {
    if (!ctx) return set_error(VXG_ERR_INVALID_ARGUMENT, "null vxg_ctx");
    g_cur_ctx = &ctx->c;  // this entry point's launches follow ctx's options
    return hip_check(hipSetDevice(ctx->c.device), "hipSetDevice");
}

// Validate one BitPacked buffer (bitpacking/mod.rs:54-130) and describe its K1 decode.
vxg_status make_k1_job(int T, unsigned W, unsigned offset, uint64_t len, const void* packed, uint64_t packed_bytes,
                       Epi epi, int vw, const UnpackArgs& a, void* out, K1Job& j) {
    if (offset > 1023) return set_error(VXG_ERR_INVALID_ARGUMENT, "Offset must be less than full block, i.e. 1024");
    if (W > unsigned(T)) return set_error(VXG_ERR_INVALID_ARGUMENT, "Unsupported bit width");
    const uint64_t nblk = (len + offset + 1023) / 1024;
    if (W > 0 && packed_bytes != nblk * 128ull * W)  // bitpacking/mod.rs:80-88
        return set_error(VXG_ERR_INVALID_ARGUMENT, "Expected " + std::to_string(nblk * 128ull * W) +
                                                       " packed bytes, got " + std::to_string(packed_bytes));
    if (W > 0 && (reinterpret_cast<uintptr_t>(packed) & 15))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "packed buffer must be 16-byte aligned");
    const int ow = epi == Epi::Dict ? vw : (epi == Epi::AlpF32 ? 4 : (epi == Epi::AlpF64 ? 8 : T / 8));
    if (reinterpret_cast<uintptr_t>(out) % uint64_t(ow))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "output buffer must be aligned to the value width");
    if (epi == Epi::Dict && W > unsigned(kDictFusedMaxW)) return VXG_ERR_NOT_IMPLEMENTED;
    // every code is out of bounds of an empty dictionary (whose buffer may be null)
    if (epi == Epi::Dict && a.dict_len == 0 && len > 0)
        return set_error(VXG_ERR_OUT_OF_BOUNDS, "take: index out of bounds");
    j.T = T;
    j.W = int(W);
    j.epi = epi;
    j.vw = epi == Epi::Dict ? vw : 0;
    j.d = ChunkDev{};
    j.d.packed = static_cast<const uint8_t*>(packed);
    j.d.out = out;
    j.d.n_blocks = len ? nblk : 0;
    j.d.len = len;
    j.d.reference = a.reference;
    j.d.alp_a = a.alp_a;
    j.d.alp_b = a.alp_b;
    j.d.dict = a.dict;
    j.d.dict_len = a.dict_len;
    j.d.offset = offset;
    j.d.shift = a.shift;
    return VXG_OK;
}

vxg_status bitunpack_common(vxg_ctx* ctx, int T, unsigned W, unsigned offset, uint64_t len,
                            const void* packed, uint64_t packed_bytes, Epi epi, int vw,
                            UnpackArgs a, void* out, void* stream) {
    std::vector<K1Job> jobs(1);
    VXG_TRY(make_k1_job(T, W, offset, len, packed, packed_bytes, epi, vw, a, out, jobs[0]));
    return launch_k1_jobs(jobs, ctx->c.err_word, S(stream));
}

// RunEnd expansions of one value width: short runs thread-per-run (K8r), long runs workgroup
// per kRunEndSpan outputs (K8), kRunEndArgChunks chunks per launch (a plan: one launch per kind
// over a device table).
vxg_status launch_runs(std::vector<RunEndChunk> runs, int w, uint32_t* err, hipStream_t s, DevTables* dt) {
    runs.erase(std::remove_if(runs.begin(), runs.end(), [](const RunEndChunk& r) { return r.len == 0; }), runs.end());
    std::vector<RunEndChunk> short_runs, long_runs;
    for (const RunEndChunk& r : runs) (r.len <= kRunEndShortRun * r.n_runs ? short_runs : long_runs).push_back(r);
    for (int pass = 0; pass < 2; pass++) {
        std::vector<RunEndChunk>& rs = pass == 0 ? short_runs : long_runs;
        const size_t per = dt && rs.size() > size_t(kRunEndArgChunks) ? rs.size() : size_t(kRunEndArgChunks);
        for (size_t i = 0; i < rs.size(); i += per) {
            RunEndTable tab{};
            tab.err = err;
            RunEndChunk* cs = tab.c;
            RunEndChunk* host = nullptr;
            if (per > size_t(kRunEndArgChunks)) {
                VXG_TRY_S(dt->table(rs.size(), &host, &tab.ext));
                cs = host;
            }
            uint64_t groups = 0;
            for (size_t k = i; k < rs.size() && k - i < per; k++) {
                RunEndChunk& r = cs[tab.n++];
                r = rs[k];
                r.first_group = groups;
                groups += pass == 0 ? (r.n_runs + kRunEndRunsPerGroup - 1) / kRunEndRunsPerGroup
                                    : (r.len + kRunEndSpan - 1) / kRunEndSpan;
            }
            VXG_TRY_S(pass == 0 ? launch_runend_runs(w, tab, groups, s) : launch_runend_chunks(w, tab, groups, s));
        }
    }
    return VXG_OK;
}

// A recorded plan's deferred launches, shared by the planners of all its arrays: the K1 decodes,
// RunEnd expansions and string-dictionary views of every chunked column, launched together at
// the end of recording on one graph branch (dictionary views, then one launch per large K1 kernel
// group + one K1g launch for all the small ones, then the expansions), instead of per column.
struct PlanBatch {
    struct Run {
        int w;             // value width
        RunEndChunk c;
        bool indep;        // ends/values read in place (no K1 decode of this batch feeds it)
    };
    std::vector<VarBinChunk> dicts;
    std::vector<K1Job> jobs;
    std::vector<Run> runs;
    std::vector<FsstChunk> fssts;  // FSST chunks of chunked columns
    bool empty() const { return dicts.empty() && jobs.empty() && runs.empty() && fssts.empty(); }
};

// VXG_PLAN_FUSE=0 (read at every flush): a batched plan's FSST decode keeps its own launch
// instead of running inside the K1g launch (A/B).
static bool plan_fuse_enabled() {
    const char* e = std::getenv("VXG_PLAN_FUSE");
    return !(e && e[0] == '0');
}

vxg_status launch_varbin_dicts(const std::vector<VarBinChunk>& dicts, uint32_t* err, hipStream_t s, DevTables* dt) {
    const size_t per = dt && dicts.size() > size_t(kVarBinArgChunks) ? dicts.size() : size_t(kVarBinArgChunks);
    for (size_t i = 0; i < dicts.size(); i += per) {
        VarBinTable tab{};
        tab.err = err;
        VarBinChunk* cs = tab.c;
        if (per > size_t(kVarBinArgChunks)) {
            VarBinChunk* host;
            VXG_TRY_S(dt->table(dicts.size(), &host, &tab.ext));
            cs = host;
        }
        uint64_t groups = 0;
        for (size_t j = i; j < dicts.size() && j - i < per; j++) {
            VarBinChunk& d = cs[tab.n++];
            d = dicts[j];
            d.first_group = groups;
            groups += d.n ? (d.n + 255) / 256 : 1;
        }
        VXG_TRY_S(launch_varbin_chunks(tab, groups, s));
    }
    return VXG_OK;
}

vxg_status flush_plan_batch(PlanBatch& b, uint32_t* err, hipStream_t s, DevTables* dt) {
    // FSST chunks: pre-passes first; one accessor group's decode tiles then run inside the K1g
    // launch (fsst_k1g_kernel), beside the K1 jobs, the other groups' decodes here
    FsstFused ff;
    if (!b.fssts.empty()) {
        void* scratch = nullptr;
        VXG_TRY_S(hip_check(hipMalloc(&scratch, (fsst_batch_scratch_bytes(b.fssts.data(), b.fssts.size()) + 15) & ~15ull),
                            "hipMalloc (plan FSST scratch)"));
        dt->allocs.push_back(scratch);
        VXG_TRY_S(launch_fsst_batch(b.fssts, scratch, err, s, dt, plan_fuse_enabled() ? &ff : nullptr));
    }
    VXG_TRY_S(launch_varbin_dicts(b.dicts, err, s, dt));
    // short-run expansions that read their children in place join the K1g launch; the others
    // follow the K1 decodes that produce their children
    std::vector<std::pair<int, RunEndChunk>> gen_runs;
    std::vector<PlanBatch::Run> rest;
    for (const PlanBatch::Run& r : b.runs) {
        if (r.c.len == 0) continue;
        if (r.indep && r.c.len <= kRunEndShortRun * r.c.n_runs && gen_runs_kind(r.w) >= 0) gen_runs.emplace_back(r.w, r.c);
        else rest.push_back(r);
    }
    VXG_TRY_S(launch_k1_jobs(b.jobs, err, s, dt, true, &gen_runs, nullptr, &ff));
    std::vector<int> widths;
    for (const auto& r : rest) widths.push_back(r.w);
    std::sort(widths.begin(), widths.end());
    widths.erase(std::unique(widths.begin(), widths.end()), widths.end());
    for (int w : widths) {
        std::vector<RunEndChunk> rs;
        for (const auto& r : rest)
            if (r.w == w) rs.push_back(r.c);
        VXG_TRY_S(launch_runs(rs, w, err, s, dt));
    }
    return VXG_OK;
}

// ===================================================================================
// Planner
// ===================================================================================
class Planner {
  public:
    Planner(vxg_ctx* ctx, hipStream_t s, DevTables* plan = nullptr, PlanBatch* batch = nullptr)
        : ctx_(ctx), s_(s), plan_(plan), batch_(batch) {}
    ~Planner() {
        for (void* p : temps_) (void)hipFreeAsync(p, s_);
    }

    vxg_status canonical(const vxg_array& a, vxg_canonical& out);
    // compute::take on the compressed tree (take.hip): values + validity.take(indices)
    vxg_status take(const vxg_array& a, const void* idx, int iw, bool isg, uint64_t n, vxg_canonical& out);
    // compute::filter (filter.hip): the rows whose predicate bit is set + validity.filter
    vxg_status filter(const vxg_array& a, const vxg_array& pred, vxg_canonical& out);
    vxg_status canonical_size(const vxg_array& a, uint64_t& vb, uint64_t& db);
    // Data buffers of a string canonical, placed 16-byte aligned in one allocation.
    vxg_status string_layout(const vxg_array& a, std::vector<vxg_data_buffer>& bufs, uint64_t& extent);
    static vxg_status string_buffer_count(const vxg_array& a, uint32_t& n);

  private:
    vxg_ctx* ctx_;
    hipStream_t s_;
    std::vector<void*> temps_;
    // Recording a plan: temporaries are plain allocations owned by the plan (alive for all its
    // replays) instead of stream-ordered ones, and chunk tables longer than a kernel argument
    // holds become device tables (one launch per kernel group).
    DevTables* plan_ = nullptr;
    PlanBatch* batch_ = nullptr;  // a plan's deferred launches (all its arrays), or null
    // The array canonical() was called on.  Only a ChunkedArray that IS this root defers its
    // launches into batch_: its chunks write straight into the caller's output and nothing
    // recorded after it reads them.  A nested ChunkedArray (Dict values, FoR/ZigZag/ALP child,
    // Sparse/RunEnd children, views of a string dictionary) feeds a consumer recorded right
    // after it, so it launches immediately.
    const vxg_array* root_ = nullptr;
    bool defer(const vxg_array& a) const { return batch_ && &a == root_; }
    // Deferred K1 decodes of the chunks of a ChunkedArray (grouped into shared launches) and
    // the patch scatters that must follow them; null = launch immediately.
    struct PatchJob {
        const vxg_array* sp;
        int T;
        Epi epi;
        int vw;
        UnpackArgs a;
        void* dst;
        uint64_t out_len;
    };
    std::vector<K1Job>* k1_batch_ = nullptr;
    std::vector<PatchJob>* patch_batch_ = nullptr;
    const PatchCol* fused_patch_ = nullptr;  // decode_alp -> decode_bitpacked: patches K1w writes
    std::vector<FsstChunk>* fsst_batch_ = nullptr;  // FSST chunks of a chunked string array
    bool k1_fusable(const vxg_array& c) const;

    vxg_status temp(uint64_t bytes, void** p) {
        if (bytes == 0) bytes = 16;
        if (plan_) {
            VXG_TRY(hip_check(hipMalloc(p, (bytes + 15) & ~15ull), "hipMalloc (plan temporary)"));
            plan_->allocs.push_back(*p);
            return VXG_OK;
        }
        VXG_TRY(hip_check(hipMallocAsync(p, (bytes + 15) & ~15ull, s_), "hipMallocAsync"));
        temps_.push_back(*p);
        return VXG_OK;
    }

    static bool is_primitive_dtype(const vxg_array& a) { return a.dtype == VXG_DTYPE_PRIMITIVE; }
    static int width(const vxg_array& a) { return ptype_width(a.ptype); }

    const vxg_buffer* buf(const vxg_array& a, uint32_t i) const {
        return i < a.n_buffers ? &a.buffers[i] : nullptr;
    }
    const vxg_array* child(const vxg_array& a, uint32_t i) const {
        return i < a.n_children ? &a.children[i] : nullptr;
    }

    // Decode a primitive-typed array into dst (len * width bytes, 16-B aligned).
    vxg_status decode_into(const vxg_array& a, void* dst);
    // Canonical primitive values of `a` as a device pointer (aliases PRIMITIVE buffers).
    vxg_status view_primitive(const vxg_array& a, const void** p);
    vxg_status int_column(const vxg_array& a, IntCol& c);
    // a patch-free 32/64-bit [FoR](BitPacked) integer column as a packed IntCol (*packed = true),
    // validated; otherwise *packed = false and nothing is decoded
    vxg_status packed_column(const vxg_array& a, IntCol& c, bool* packed);
    vxg_status runend_column(const vxg_array& a, bool in_place, IntCol& c);

    vxg_status decode_bitpacked(const vxg_array& bp, Epi epi, int vw, UnpackArgs a, void* dst);
    bool patch_fusable(const vxg_array& sparse, int value_width) const;
    vxg_status sparse_patch_col(const vxg_array& sparse, PatchCol& pc);
    vxg_status apply_sparse_patches(const vxg_array& sparse, int T, Epi epi, int vw, const UnpackArgs& a,
                                    void* dst, uint64_t out_len);
    vxg_status decode_alp(const vxg_array& a, void* dst);
    vxg_status decode_dict_primitive(const vxg_array& a, void* dst);
    vxg_status decode_chunked_primitive(const vxg_array& a, void* dst);
    vxg_status decode_alprd(const vxg_array& a, void* dst);
    vxg_status decode_sparse_values(const vxg_array& a, void* dst);

    vxg_status take_values(const vxg_array& a, const void* idx, int iw, bool isg, uint64_t n, void* dst);
    vxg_status take_patches(const vxg_array& sp, TakePatches& p);
    vxg_status validity_into(const vxg_array& a, void** bitmap);
    // OR the values of a Bool-dtype array into the zeroed bit buffer `bits` at bit `off`.
    vxg_status bools_into(const vxg_array& a, void* bits, uint64_t off);
    vxg_status validity_source(const vxg_array& a, const vxg_array** node, int* kind);
    vxg_status string_canonical(const vxg_array& a, vxg_canonical& out);
    vxg_status string_lens(const vxg_array& a, std::vector<uint64_t>& lens,
                           std::vector<std::pair<size_t, const vxg_array*>>& fsst) const;
    vxg_status strings_into(const vxg_array& a, uint8_t* views, uint8_t* data, const vxg_data_buffer* bufs,
                            uint32_t bidx, const uint8_t* validity);
};

vxg_status Planner::view_primitive(const vxg_array& a, const void** p) {
    if (a.encoding == VXG_ENC_PRIMITIVE) {
        const vxg_buffer* b = buf(a, 0);
        if (!b && a.len) return set_error(VXG_ERR_INVALID_ARGUMENT, "Primitive array without buffer");
        if (b && b->len < a.len * width(a))
            return set_error(VXG_ERR_INVALID_ARGUMENT, "Primitive buffer shorter than len * width");
        *p = b ? b->ptr : nullptr;
        return VXG_OK;
    }
    void* t;
    VXG_TRY(temp(a.len * width(a), &t));
    VXG_TRY(decode_into(a, t));
    *p = t;
    return VXG_OK;
}

vxg_status Planner::int_column(const vxg_array& a, IntCol& c) {
    // An integer child read in place by a consumer kernel: a patch-free 32/64-bit
    // [FoR](BitPacked) column stays packed (elements unpacked where used); anything else is
    // canonicalized to a primitive buffer first.
    if (!ptype_is_int(a.ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "expected an integer array");
    bool packed = false;
    VXG_TRY(packed_column(a, c, &packed));
    return packed ? VXG_OK : view_primitive(a, &c.p);
}

vxg_status Planner::runend_column(const vxg_array& a, bool in_place, IntCol& c) {
    // RunEnd ends/values: read in place by the short-run kernel when packable, else a plain
    // buffer (canonicalized child-first).  Non-integer values (floats) are plain bits.
    bool packed = false;
    if (in_place && ptype_is_int(a.ptype)) VXG_TRY(packed_column(a, c, &packed));
    if (packed) return VXG_OK;
    c = IntCol{};
    c.width = width(a);
    c.sgn = ptype_is_signed(a.ptype);
    return view_primitive(a, &c.p);
}

vxg_status Planner::packed_column(const vxg_array& a, IntCol& c, bool* packed) {
    *packed = false;
    c = IntCol{};
    c.width = width(a);
    c.sgn = ptype_is_signed(a.ptype);
    const vxg_array* bp = nullptr;
    if (a.encoding == VXG_ENC_FL_FOR && child(a, 0) && child(a, 0)->encoding == VXG_ENC_FL_BITPACKED) {
        bp = child(a, 0);
        c.reference = a.meta.for_.reference;
        c.shift = a.meta.for_.shift;
    } else if (a.encoding == VXG_ENC_FL_BITPACKED) {
        bp = &a;
    }
    if (bp && !bp->meta.bitpacked.has_patches && width(*bp) == c.width && (c.width == 4 || c.width == 8) &&
        bp->len == a.len) {
        const vxg_buffer* pk = buf(*bp, 0);
        const unsigned W = bp->meta.bitpacked.bit_width, off = bp->meta.bitpacked.offset;
        const uint64_t nblk = (bp->len + off + 1023) / 1024;
        if (off > 1023) return set_error(VXG_ERR_INVALID_ARGUMENT, "Offset must be less than full block, i.e. 1024");
        if (W > unsigned(8 * c.width)) return set_error(VXG_ERR_INVALID_ARGUMENT, "Unsupported bit width");
        const uint64_t have = pk ? pk->len : 0;
        if (W > 0 && have != nblk * 128ull * W)  // bitpacking/mod.rs:80-88
            return set_error(VXG_ERR_INVALID_ARGUMENT, "Expected " + std::to_string(nblk * 128ull * W) +
                                                           " packed bytes, got " + std::to_string(have));
        c.packed = true;
        c.p = pk ? pk->ptr : nullptr;
        c.W = W;
        c.offset = off;
        *packed = true;
    }
    return VXG_OK;
}

vxg_status Planner::apply_sparse_patches(const vxg_array& sp, int T, Epi epi, int vw, const UnpackArgs& a,
                                         void* dst, uint64_t out_len) {
    // bitpacking/compress.rs:191-207 / alp/compress.rs:80-96: only SparseArray patches.
    if (sp.encoding != VXG_ENC_SPARSE)
        return set_error(VXG_ERR_INVALID_ARGUMENT, "Can't patch with a non-Sparse array");
    const vxg_array* idx = child(sp, 0);
    const vxg_array* val = child(sp, 1);
    if (!idx || !val) return set_error(VXG_ERR_INVALID_ARGUMENT, "Sparse patches need indices and values");
    if (idx->len != val->len) return set_error(VXG_ERR_INVALID_ARGUMENT, "Sparse indices/values length mismatch");
    PatchCol pc;  // a packed index column is unpacked by the scatter itself (no temporary)
    VXG_TRY(int_column(*idx, pc.idx));
    VXG_TRY(view_primitive(*val, &pc.vals));
    return launch_patch(vw, pc.idx, epi, T, dst, out_len, sp.meta.sparse.indices_offset, pc.vals, idx->len, a, s_);
}

bool Planner::patch_fusable(const vxg_array& sp, int value_width) const {
    const vxg_array* idx = child(sp, 0);
    const vxg_array* val = child(sp, 1);
    return sp.encoding == VXG_ENC_SPARSE && idx && val && idx->len == val->len && idx->len > 0 &&
           width(*val) == value_width && width(*idx) == 8 && ptype_is_int(idx->ptype);
}

vxg_status Planner::sparse_patch_col(const vxg_array& sp, PatchCol& pc) {
    // patch_fusable(sp) holds
    const vxg_array* idx = child(sp, 0);
    VXG_TRY(int_column(*idx, pc.idx));
    VXG_TRY(view_primitive(*child(sp, 1), &pc.vals));
    pc.n = idx->len;
    pc.idx_off = sp.meta.sparse.indices_offset;
    return VXG_OK;
}

vxg_status Planner::decode_bitpacked(const vxg_array& bp, Epi epi, int vw, UnpackArgs a, void* dst) {
    // bitpacking/mod.rs:215-219 -> compress.rs:167-189 (patches: child 0 when has_patches)
    const int T = 8 * width(bp);
    if (!ptype_is_int(bp.ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "BitPacked needs an integer ptype");
    const vxg_buffer* packed = buf(bp, 0);
    const unsigned W = bp.meta.bitpacked.bit_width;
    a.err = ctx_->c.err_word;
    K1Job j;
    VXG_TRY(make_k1_job(T, W, bp.meta.bitpacked.offset, bp.len, packed ? packed->ptr : nullptr,
                        packed ? packed->len : 0, epi, vw, a, dst, j));
    const vxg_array* p = nullptr;
    if (bp.meta.bitpacked.has_patches) {
        p = child(bp, 0);
        if (!p) return set_error(VXG_ERR_INVALID_ARGUMENT, "BitPackedArray: patches child missing");
    }
    if (k1_batch_) {  // a chunk of a ChunkedArray: launched with the other chunks
        k1_batch_->push_back(j);
        if (p) patch_batch_->push_back(PatchJob{p, T, epi, vw, a, dst, bp.len});
        return VXG_OK;
    }
    std::vector<K1Job> one{j};
    VXG_TRY(launch_k1_jobs(one, ctx_->c.err_word, s_, plan_, false, nullptr, fused_patch_));
    if (p) VXG_TRY(apply_sparse_patches(*p, T, epi, vw, a, dst, bp.len));
    return VXG_OK;
}

vxg_status Planner::decode_alp(const vxg_array& a, void* dst) {
    // alp/array.rs:269 -> alp/compress.rs:61-78 (+ patch_decoded :80-96)
    const vxg_array* enc = child(a, 0);
    if (!enc) return set_error(VXG_ERR_INVALID_ARGUMENT, "ALPArray: encoded child missing");
    const bool f32 = a.ptype == VXG_F32;
    if (!f32 && a.ptype != VXG_F64) return set_error(VXG_ERR_MISMATCHED_TYPES, "ALP can only encode f32 and f64");
    const unsigned e = a.meta.alp.e, f = a.meta.alp.f;
    if ((f32 && (e > 10 || f > 10)) || (!f32 && (e > 23 || f > 23)))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "ALP exponents out of range");
    UnpackArgs ua{};
    ua.alp_a = f32 ? double(kF10f[f]) : kF10d[f];
    ua.alp_b = f32 ? double(kIF10f[e]) : kIF10d[e];
    const Epi epi = f32 ? Epi::AlpF32 : Epi::AlpF64;
    const vxg_array* bp = nullptr;
    if (enc->encoding == VXG_ENC_FL_FOR && child(*enc, 0) &&
        child(*enc, 0)->encoding == VXG_ENC_FL_BITPACKED) {
        ua.reference = enc->meta.for_.reference;
        ua.shift = enc->meta.for_.shift;
        bp = child(*enc, 0);
    } else if (enc->encoding == VXG_ENC_FL_BITPACKED) {
        bp = enc;
    }
    bool fused = false;  // the outer patches written by the K1w launch itself
    if (bp && width(*bp) == (f32 ? 4 : 8)) {
        PatchCol pc{};
        const vxg_array* p = a.meta.alp.has_patches ? child(a, 1) : nullptr;
        if (p && !k1_batch_ && !patch_batch_ && !bp->meta.bitpacked.has_patches && bp->len == a.len &&
            patch_fusable(*p, f32 ? 4 : 8) && fused_patches_enabled()) {
            const uint64_t nblk = (bp->len + bp->meta.bitpacked.offset + 1023) / 1024;
            if (k1_takes_wave(f32 ? 32 : 64, int(bp->meta.bitpacked.bit_width), epi, (nblk + 31) / 32)) {
                VXG_TRY(sparse_patch_col(*p, pc));
                fused = !pc.idx.packed || pc.idx.W > 0;  // K1w reads 8-byte index words directly
            }
        }
        fused_patch_ = fused ? &pc : nullptr;
        g_k1w_wrote_patches = false;
        const vxg_status st = decode_bitpacked(*bp, epi, 0, ua, dst);  // fused unpack+FoR+ALP (+patches)
        fused_patch_ = nullptr;
        VXG_TRY(st);
        fused = fused && g_k1w_wrote_patches;  // any other K1 path left them to the scatter below
    } else {
        const void* penc;
        VXG_TRY(view_primitive(*enc, &penc));
        VXG_TRY(launch_alp(a.ptype, penc, a.len, ua.alp_a, ua.alp_b, dst, s_));
    }
    if (a.meta.alp.has_patches && !fused) {
        const vxg_array* p = child(a, 1);
        if (!p) return set_error(VXG_ERR_INVALID_ARGUMENT, "ALPArray: patches child missing");
        UnpackArgs plain{};
        plain.err = ctx_->c.err_word;
        if (patch_batch_) {  // after the chunk's K1 decode and its inner patches
            patch_batch_->push_back(PatchJob{p, f32 ? 32 : 64, Epi::Plain, 0, plain, dst, a.len});
            return VXG_OK;
        }
        VXG_TRY(apply_sparse_patches(*p, f32 ? 32 : 64, Epi::Plain, 0, plain, dst, a.len));
    }
    return VXG_OK;
}

vxg_status Planner::decode_dict_primitive(const vxg_array& a, void* dst) {
    // dict/array.rs:68-73: take(canonical(values), codes)
    const vxg_array* values = child(a, 0);
    const vxg_array* codes = child(a, 1);
    if (!values || !codes) return set_error(VXG_ERR_INVALID_ARGUMENT, "DictArray needs values and codes");
    if (!ptype_is_unsigned(codes->ptype) || codes->nullable)
        return set_error(VXG_ERR_MISMATCHED_TYPES, "Dict codes must be non-nullable unsigned int");
    const void* pv;
    VXG_TRY(view_primitive(*values, &pv));
    const int vw = width(*values);
    if (codes->encoding == VXG_ENC_FL_BITPACKED && codes->meta.bitpacked.bit_width <= kDictFusedMaxW) {
        UnpackArgs ua{};
        ua.dict = pv;
        ua.dict_len = values->len;
        return decode_bitpacked(*codes, Epi::Dict, vw, ua, dst);
    }
    const void* pc;
    VXG_TRY(view_primitive(*codes, &pc));
    return launch_take(vw, pv, values->len, width(*codes), false, pc, a.len, dst, ctx_->c.err_word, s_);
}

// Chunks whose whole decode is one K1 launch (+ patch scatters): BitPacked, FoR/ZigZag/ALP over
// BitPacked of the same width, Dict(Primitive values, BitPacked codes).  Their decodes are
// deferred and grouped across chunks; nothing in them reads another deferred output.
bool Planner::k1_fusable(const vxg_array& c) const {
    auto bp_of_width = [&](const vxg_array* x, int w) {
        return x && x->encoding == VXG_ENC_FL_BITPACKED && width(*x) == w && ptype_is_int(x->ptype);
    };
    const int w = width(c);
    switch (c.encoding) {
    case VXG_ENC_FL_BITPACKED: return ptype_is_int(c.ptype);
    case VXG_ENC_FL_FOR: return ptype_is_int(c.ptype) && bp_of_width(child(c, 0), w);
    case VXG_ENC_ZIGZAG: return ptype_is_signed(c.ptype) && bp_of_width(child(c, 0), w);
    case VXG_ENC_ALP: {
        if (c.ptype != VXG_F32 && c.ptype != VXG_F64) return false;
        const vxg_array* e = child(c, 0);
        if (e && e->encoding == VXG_ENC_FL_FOR) e = child(*e, 0);
        return bp_of_width(e, w);
    }
    case VXG_ENC_DICT: {
        const vxg_array* v = child(c, 0);
        const vxg_array* k = child(c, 1);
        return v && k && v->encoding == VXG_ENC_PRIMITIVE && k->encoding == VXG_ENC_FL_BITPACKED &&
               ptype_is_unsigned(k->ptype) && !k->nullable && k->meta.bitpacked.bit_width <= kDictFusedMaxW;
    }
    default: return false;
    }
}

vxg_status Planner::decode_chunked_primitive(const vxg_array& a, void* dst) {
    // chunked/canonical.rs:27-122 / pack_primitives :170-187 -- every chunk decodes straight
    // into its slice of the output (no per-chunk materialisation + memcpy).  Launches are
    // shared across chunks, level by level:
    //   level 0  K1 decodes: chunks that are one K1 decode, and the ends/values children of
    //            RunEnd chunks (into one temporary)      -> grouped by kernel, 32 per launch
    //   level 1  their patch scatters
    //   level 2  RunEnd expansions                         -> 48 chunks per launch
    // Other chunks decode one by one.
    const uint64_t n = a.meta.chunked.nchunks;
    if (a.n_children != n + 1) return set_error(VXG_ERR_INVALID_ARGUMENT, "Chunked child count != nchunks + 1");
    const int w = width(a);
    std::vector<K1Job> jobs;
    std::vector<PatchJob> patches;
    std::vector<RunEndChunk> runs;
    std::vector<uint8_t> runs_indep;  // the run's children are read in place (no level-0 decode)
    // RunEnd chunks whose ends/values are primitive or one K1 decode: their temporaries
    auto child_ok = [&](const vxg_array* x) {
        return x && ptype_is_int(x->ptype) && (x->encoding == VXG_ENC_PRIMITIVE || k1_fusable(*x));
    };
    auto batch_runend = [&](const vxg_array& c) {
        const vxg_array* e = child(c, 0);
        const vxg_array* v = child(c, 1);
        return c.encoding == VXG_ENC_RUN_END && child_ok(e) && v && width(*v) == w && e->len == v->len &&
               (v->encoding == VXG_ENC_PRIMITIVE || k1_fusable(*v)) && e->len > 0;
    };
    // short-run chunks read packed ends/values in place (no temporary, no level-0 launch)
    std::vector<IntCol> inplace(2 * n);
    std::vector<uint8_t> is_inplace(2 * n, 0);
    uint64_t tmp_bytes = 0;
    for (uint64_t i = 0; i < n; i++) {
        const vxg_array& c = a.children[i + 1];
        if (!batch_runend(c)) continue;
        const vxg_array* e = child(c, 0);
        const vxg_array* v = child(c, 1);
        const bool short_runs = c.len <= kRunEndShortRun * e->len;
        const vxg_array* xs[2] = {e, v};
        for (int k = 0; k < 2; k++) {
            bool pk = false;
            if (short_runs && ptype_is_int(xs[k]->ptype)) VXG_TRY(packed_column(*xs[k], inplace[2 * i + k], &pk));
            is_inplace[2 * i + k] = pk;
            if (!pk && xs[k]->encoding != VXG_ENC_PRIMITIVE) tmp_bytes += (xs[k]->len * width(*xs[k]) + 15) & ~15ull;
        }
    }
    uint8_t* tmp = nullptr;
    if (tmp_bytes) {
        void* t;
        VXG_TRY(temp(tmp_bytes, &t));
        tmp = static_cast<uint8_t*>(t);
    }
    // decode `x` (primitive or one K1 decode) for a RunEnd chunk: pointer into the temporary
    auto level0 = [&](const vxg_array& x, const void** p) -> vxg_status {
        if (x.encoding == VXG_ENC_PRIMITIVE) return view_primitive(x, p);
        *p = tmp;
        tmp += (x.len * width(x) + 15) & ~15ull;
        k1_batch_ = &jobs;
        patch_batch_ = &patches;
        const vxg_status st = decode_into(x, const_cast<void*>(*p));
        k1_batch_ = nullptr;
        patch_batch_ = nullptr;
        return st;
    };
    uint64_t off = 0;
    for (uint64_t i = 0; i < n; i++) {
        const vxg_array& c = a.children[i + 1];
        if (c.ptype != a.ptype || c.dtype != a.dtype)
            return set_error(VXG_ERR_MISMATCHED_TYPES, "Chunks must have the ChunkedArray's dtype");
        uint8_t* slice = static_cast<uint8_t*>(dst) + off * w;
        if (k1_fusable(c)) {
            k1_batch_ = &jobs;
            patch_batch_ = &patches;
            const vxg_status st = decode_into(c, slice);
            k1_batch_ = nullptr;
            patch_batch_ = nullptr;
            VXG_TRY(st);
        } else if (batch_runend(c)) {
            // runend/compress.rs:115-148 (runend/array.rs:191-197)
            const vxg_array& e = *child(c, 0);
            const vxg_array& v = *child(c, 1);
            RunEndChunk r{};
            IntCol* cols[2] = {&r.ends, &r.values};
            const vxg_array* xs[2] = {&e, &v};
            for (int k = 0; k < 2; k++) {
                if (is_inplace[2 * i + k]) {
                    *cols[k] = inplace[2 * i + k];
                } else {
                    cols[k]->width = width(*xs[k]);
                    cols[k]->sgn = ptype_is_signed(xs[k]->ptype);
                    VXG_TRY(level0(*xs[k], &cols[k]->p));
                }
            }
            r.out = slice;
            r.n_runs = e.len;
            r.offset = c.meta.runend.offset;
            r.len = c.len;
            runs.push_back(r);
            runs_indep.push_back(uint8_t((is_inplace[2 * i] || e.encoding == VXG_ENC_PRIMITIVE) &&
                                         (is_inplace[2 * i + 1] || v.encoding == VXG_ENC_PRIMITIVE)));
        } else if ((reinterpret_cast<uintptr_t>(slice) & 15) == 0) {
            VXG_TRY(decode_into(c, slice));
        } else {
            const void* p;
            VXG_TRY(view_primitive(c, &p));
            VXG_TRY(launch_copy_bytes(slice, p, c.len * w, s_));
        }
        off += c.len;
    }
    if (off != a.len) return set_error(VXG_ERR_INVALID_ARGUMENT, "Chunked len != sum of chunk lens");
    if (defer(a) && patches.empty()) {  // a plan's root: launched with the other arrays' jobs (PlanBatch)
        batch_->jobs.insert(batch_->jobs.end(), jobs.begin(), jobs.end());
        for (size_t k = 0; k < runs.size(); k++) batch_->runs.push_back(PlanBatch::Run{w, runs[k], runs_indep[k] != 0});
        return VXG_OK;
    }
    VXG_TRY(launch_k1_jobs(jobs, ctx_->c.err_word, s_, plan_));
    for (const PatchJob& p : patches) VXG_TRY(apply_sparse_patches(*p.sp, p.T, p.epi, p.vw, p.a, p.dst, p.out_len));
    return launch_runs(runs, w, ctx_->c.err_word, s_, plan_);
}

vxg_status Planner::decode_alprd(const vxg_array& a, void* dst) {
    // alp_rd/array.rs:179-235 -> alp_rd/mod.rs:260-301
    const vxg_array* left = child(a, 0);
    const vxg_array* right = child(a, 1);
    if (!left || !right) return set_error(VXG_ERR_INVALID_ARGUMENT, "ALPRDArray needs left/right parts");
    if (left->ptype != VXG_U16) return set_error(VXG_ERR_MISMATCHED_TYPES, "ALP-RD left parts must be u16");
    const void *pl, *pr;
    VXG_TRY(view_primitive(*left, &pl));
    VXG_TRY(view_primitive(*right, &pr));
    const void* pos = nullptr;
    const void* exc = nullptr;
    uint64_t n_exc = 0, pos_off = 0;
    int pw = 8;
    bool psg = false;
    if (a.meta.alprd.has_exceptions) {
        const vxg_array* sp = child(a, 2);
        if (!sp || sp->encoding != VXG_ENC_SPARSE)
            return set_error(VXG_ERR_INVALID_ARGUMENT, "left_parts_exceptions must be SparseArray encoded");
        const vxg_array* si = child(*sp, 0);
        const vxg_array* sv = child(*sp, 1);
        VXG_TRY(view_primitive(*si, &pos));
        VXG_TRY(view_primitive(*sv, &exc));
        n_exc = si->len;
        pos_off = sp->meta.sparse.indices_offset;
        pw = width(*si);
        psg = ptype_is_signed(si->ptype);
    }
    return launch_alprd(a.ptype, static_cast<const uint16_t*>(pl), a.meta.alprd.dict, a.meta.alprd.dict_len,
                        a.meta.alprd.right_bit_width, pr, a.len, pos, pw, psg, pos_off,
                        static_cast<const uint16_t*>(exc), n_exc, dst, ctx_->c.err_word, s_);
}

vxg_status Planner::decode_sparse_values(const vxg_array& a, void* dst) {
    // array/sparse/flatten.rs:68-98: fill (null fill -> default 0), then scatter values.
    uint8_t fill[16] = {0};
    if (!a.meta.sparse.fill_is_null) std::memcpy(fill, a.meta.sparse.fill, 16);
    VXG_TRY(launch_fill(width(a), fill, a.len, dst, s_));
    UnpackArgs plain{};
    plain.err = ctx_->c.err_word;
    return apply_sparse_patches(a, 8 * width(a), Epi::Plain, 0, plain, dst, a.len);
}

vxg_status Planner::decode_into(const vxg_array& a, void* dst) {
    if (!is_primitive_dtype(a)) return set_error(VXG_ERR_MISMATCHED_TYPES, "expected a primitive dtype");
    const int w = width(a);
    if (w == 0) return set_error(VXG_ERR_NOT_IMPLEMENTED, "unsupported ptype");
    switch (a.encoding) {
    case VXG_ENC_PRIMITIVE: {
        const void* p;
        VXG_TRY(view_primitive(a, &p));
        if (p != dst && a.len)
            VXG_TRY(launch_copy_bytes(dst, p, a.len * w, s_));
        return VXG_OK;
    }
    case VXG_ENC_FL_BITPACKED:
        return decode_bitpacked(a, Epi::Plain, 0, UnpackArgs{}, dst);
    case VXG_ENC_FL_FOR: {
        // for/mod.rs:105-109 -> for/compress.rs:86-98
        const vxg_array* enc = child(a, 0);
        if (!enc) return set_error(VXG_ERR_INVALID_ARGUMENT, "FoRArray is missing encoded child array");
        if (!ptype_is_int(a.ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "FoR needs an integer ptype");
        if (enc->encoding == VXG_ENC_FL_BITPACKED && width(*enc) == w) {
            UnpackArgs ua{};
            ua.reference = a.meta.for_.reference;
            ua.shift = a.meta.for_.shift;
            return decode_bitpacked(*enc, Epi::For, 0, ua, dst);
        }
        VXG_TRY(decode_into(*enc, dst));
        return launch_for(w, dst, a.len, a.meta.for_.reference, a.meta.for_.shift, false, dst, s_);
    }
    case VXG_ENC_ZIGZAG: {
        const vxg_array* enc = child(a, 0);
        if (!enc) return set_error(VXG_ERR_INVALID_ARGUMENT, "ZigZagArray is missing encoded child");
        if (!ptype_is_signed(a.ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "ZigZag decodes to signed ints");
        if (enc->encoding == VXG_ENC_FL_BITPACKED && width(*enc) == w)
            return decode_bitpacked(*enc, Epi::ForZigZag, 0, UnpackArgs{}, dst);
        VXG_TRY(decode_into(*enc, dst));
        return launch_zigzag(w, dst, a.len, dst, s_);
    }
    case VXG_ENC_ALP:
        return decode_alp(a, dst);
    case VXG_ENC_ALP_RD:
        return decode_alprd(a, dst);
    case VXG_ENC_DICT:
        return decode_dict_primitive(a, dst);
    case VXG_ENC_FL_DELTA: {
        // delta/mod.rs:237 -> delta/compress.rs:100-166
        const vxg_array* bases = child(a, 0);
        const vxg_array* deltas = child(a, 1);
        if (!bases || !deltas) return set_error(VXG_ERR_INVALID_ARGUMENT, "DeltaArray needs bases and deltas");
        const int T = 8 * w, lanes = 1024 / T;
        const uint64_t nd = deltas->len;
        if (bases->len != (nd / 1024) * lanes + (nd % 1024 ? 1 : 0))
            return set_error(VXG_ERR_INVALID_ARGUMENT, "DeltaArray: bases.len() != expected_bases_len");
        if (a.meta.delta.offset >= 1024 || a.meta.delta.offset + a.len > nd)
            return set_error(VXG_ERR_INVALID_ARGUMENT, "DeltaArray: offset/len out of range");
        const void *pb, *pd;
        VXG_TRY(view_primitive(*bases, &pb));
        VXG_TRY(view_primitive(*deltas, &pd));
        return launch_delta(w, pb, pd, nd, a.meta.delta.offset, a.len, dst, s_);
    }
    case VXG_ENC_RUN_END: {
        // runend/array.rs:191-197 -> runend/compress.rs:95-148
        const vxg_array* ends = child(a, 0);
        const vxg_array* values = child(a, 1);
        if (!ends || !values) return set_error(VXG_ERR_INVALID_ARGUMENT, "RunEndArray needs ends and values");
        if (ends->len != values->len) return set_error(VXG_ERR_INVALID_ARGUMENT, "RunEnd ends/values length mismatch");
        RunEndChunk c{};
        c.out = dst;
        c.n_runs = ends->len;
        c.offset = a.meta.runend.offset;
        c.len = a.len;
        VXG_TRY(runend_column(*ends, a.len <= kRunEndShortRun * ends->len, c.ends));
        VXG_TRY(runend_column(*values, a.len <= kRunEndShortRun * ends->len, c.values));
        return launch_runend(w, c, ctx_->c.err_word, s_);
    }
    case VXG_ENC_SPARSE:
        return decode_sparse_values(a, dst);
    case VXG_ENC_CONSTANT: {
        uint8_t sc[16] = {0};
        if (!a.meta.constant.is_null) std::memcpy(sc, a.meta.constant.scalar, 16);
        return launch_fill(w, sc, a.len, dst, s_);
    }
    case VXG_ENC_CHUNKED:
        return decode_chunked_primitive(a, dst);
    default:
        return set_error(VXG_ERR_NOT_IMPLEMENTED,
                         "no GPU canonicalize for encoding id " + std::to_string(a.encoding));
    }
}

// Where does the validity of `a` come from?  kind: 0 = no nulls, 1 = all invalid,
// 2 = Bool child array `node` (canonical bitmap buffer 0).
vxg_status Planner::validity_source(const vxg_array& a, const vxg_array** node, int* kind) {
    *node = nullptr;
    *kind = 0;
    auto from_meta = [&](uint32_t child_idx) -> vxg_status {
        switch (a.validity) {
        case VXG_VALIDITY_NON_NULLABLE:
        case VXG_VALIDITY_ALL_VALID: return VXG_OK;
        case VXG_VALIDITY_ALL_INVALID: *kind = 1; return VXG_OK;
        default: {
            const vxg_array* v = child(a, child_idx);
            if (!v || v->dtype != VXG_DTYPE_BOOL)
                return set_error(VXG_ERR_INVALID_ARGUMENT, "validity child must be a Bool array");
            *node = v;
            *kind = v->encoding == VXG_ENC_BOOL ? 2 : 5;  // 5: compressed bools, decoded
            return VXG_OK;
        }
        }
    };
    switch (a.encoding) {
    case VXG_ENC_PRIMITIVE:
    case VXG_ENC_BOOL:
    case VXG_ENC_BYTE_BOOL: return from_meta(0);
    case VXG_ENC_RUN_END_BOOL: return from_meta(1);
    case VXG_ENC_FL_BITPACKED: return from_meta(a.meta.bitpacked.has_patches ? 1 : 0);
    case VXG_ENC_FL_DELTA: return from_meta(2);
    case VXG_ENC_RUN_END: return from_meta(2);
    case VXG_ENC_VARBIN: return from_meta(2);
    case VXG_ENC_VARBINVIEW: return from_meta(1 + a.meta.varbinview.n_buffers);
    case VXG_ENC_FL_FOR:
    case VXG_ENC_ZIGZAG:
    case VXG_ENC_ALP: return child(a, 0) ? validity_source(*child(a, 0), node, kind) : VXG_OK;
    case VXG_ENC_ALP_RD: return child(a, 0) ? validity_source(*child(a, 0), node, kind) : VXG_OK;
    case VXG_ENC_FSST: return child(a, 2) ? validity_source(*child(a, 2), node, kind) : VXG_OK;
    case VXG_ENC_CONSTANT: *kind = a.meta.constant.is_null ? 1 : 0; return VXG_OK;
    case VXG_ENC_DICT: {
        const vxg_array* v = child(a, 0);
        if (!v) return VXG_OK;
        // take(values, codes) carries values.validity().take(codes) (primitive/compute/take.rs:
        // 58-67, varbinview/compute.rs:68-76): gathered from the values' bitmap by code
        VXG_TRY(validity_source(*v, node, kind));
        if (*kind != 0) {
            *kind = 6;
            *node = &a;
        }
        return VXG_OK;
    }
    case VXG_ENC_SPARSE:
        // primitives: valid exactly at the indices when the fill is null; bools: always
        // (canonicalize_sparse_bools builds its validity from the indices alone,
        // sparse/flatten.rs:41-61)
        if (a.meta.sparse.fill_is_null || a.dtype == VXG_DTYPE_BOOL) { *kind = 3; *node = &a; }
        return VXG_OK;
    case VXG_ENC_CHUNKED: {
        for (uint32_t i = 1; i < a.n_children; i++) {
            const vxg_array* n2;
            int k2;
            VXG_TRY(validity_source(a.children[i], &n2, &k2));
            if (k2 != 0) { *kind = 4; *node = &a; return VXG_OK; }
        }
        return VXG_OK;
    }
    default: return VXG_OK;
    }
}

vxg_status Planner::validity_into(const vxg_array& a, void** bitmap) {
    const vxg_array* node;
    int kind;
    VXG_TRY(validity_source(a, &node, &kind));
    if (kind == 0) {  // no nulls: validity NULL (a caller-provided bitmap is left untouched)
        *bitmap = nullptr;
        return VXG_OK;
    }
    const uint64_t bytes = ((a.len + 31) / 32) * 4;
    if (!*bitmap) VXG_TRY(hip_check(hipMalloc(bitmap, bytes ? bytes : 4), "validity alloc"));
    VXG_TRY(launch_copy_bytes(*bitmap, nullptr, bytes ? bytes : 4, s_));
    if (kind == 1) return VXG_OK;
    if (kind == 2) {
        const vxg_buffer* b = buf(*node, 0);
        if (!b) return set_error(VXG_ERR_INVALID_ARGUMENT, "BoolArray without buffer");
        return launch_copy_bits(*bitmap, 0, static_cast<const uint8_t*>(b->ptr),
                                node->meta.boolean.first_byte_bit_offset, a.len, false, s_);
    }
    if (kind == 5) return bools_into(*node, *bitmap, 0);
    if (kind == 6) {  // Dict with nullable values: bit i = values_valid[codes[i]]
        const vxg_array* vals = child(a, 0);
        const vxg_array* codes = child(a, 1);
        if (!vals || !codes) return set_error(VXG_ERR_INVALID_ARGUMENT, "DictArray needs values and codes");
        if (!ptype_is_int(codes->ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "Dict codes must be integers");
        void* vbits = nullptr;
        VXG_TRY(temp(((vals->len + 31) / 32) * 4, &vbits));
        VXG_TRY(validity_into(*vals, &vbits));
        const void* pc;
        VXG_TRY(view_primitive(*codes, &pc));
        return launch_gather_bits(*bitmap, pc, width(*codes), false, a.len, static_cast<const uint8_t*>(vbits), vals->len,
                                  ctx_->c.err_word, s_);
    }
    if (kind == 3) {  // Sparse with null fill: valid exactly at the indices (flatten.rs:82-93)
        const vxg_array* idx = child(a, 0);
        const void* pi;
        VXG_TRY(view_primitive(*idx, &pi));
        return launch_set_bits_at(*bitmap, pi, width(*idx), ptype_is_signed(idx->ptype),
                                  a.meta.sparse.indices_offset, idx->len, a.len, s_);
    }
    // kind 4: chunked concatenation of chunk validities
    uint64_t off = 0;
    for (uint32_t i = 1; i < a.n_children; i++) {
        const vxg_array& c = a.children[i];
        const vxg_array* n2;
        int k2;
        VXG_TRY(validity_source(c, &n2, &k2));
        if (k2 == 0) {
            VXG_TRY(launch_copy_bits(*bitmap, off, nullptr, 0, c.len, true, s_));
        } else if (k2 == 2) {
            VXG_TRY(launch_copy_bits(*bitmap, off, static_cast<const uint8_t*>(n2->buffers[0].ptr),
                                     n2->meta.boolean.first_byte_bit_offset, c.len, false, s_));
        } else if (k2 == 5) {
            VXG_TRY(bools_into(*n2, *bitmap, off));
        } else if (k2 != 1) {
            void* sub = nullptr;
            VXG_TRY(temp(((c.len + 31) / 32) * 4, &sub));
            VXG_TRY(validity_into(c, &sub));
            VXG_TRY(launch_copy_bits(*bitmap, off, static_cast<const uint8_t*>(sub), 0, c.len, false, s_));
        }
        off += c.len;
    }
    return VXG_OK;
}

// ---- compute::take on compressed arrays (vortex-array/src/compute/take.rs:10-34) ---------
vxg_status Planner::take_patches(const vxg_array& sp, TakePatches& p) {
    if (sp.encoding != VXG_ENC_SPARSE) return set_error(VXG_ERR_INVALID_ARGUMENT, "Can't patch with a non-Sparse array");
    const vxg_array* idx = child(sp, 0);
    const vxg_array* val = child(sp, 1);
    if (!idx || !val || idx->len != val->len)
        return set_error(VXG_ERR_INVALID_ARGUMENT, "Sparse patches need indices and values of equal length");
    if (!ptype_is_int(idx->ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "Sparse indices must be integers");
    VXG_TRY(view_primitive(*idx, &p.idx));
    VXG_TRY(view_primitive(*val, &p.values));
    p.n = idx->len;
    p.off = sp.meta.sparse.indices_offset;
    p.iw = width(*idx);
    p.isg = ptype_is_signed(idx->ptype);
    return VXG_OK;
}

vxg_status Planner::take_values(const vxg_array& a, const void* idx, int iw, bool isg, uint64_t n, void* dst) {
    if (n == 0) return VXG_OK;
    auto via_canonical = [&]() -> vxg_status {  // canonicalize, then take the primitive
        const void* pv;
        VXG_TRY(view_primitive(a, &pv));
        return launch_take(width(a), pv, a.len, iw, isg, idx, n, dst, ctx_->c.err_word, s_);
    };
    const vxg_array* bp = nullptr;
    Epi epi = Epi::Plain;
    EpiParams ep{};
    TakePatches outer;
    auto fl_child = [&](const vxg_array* c) -> const vxg_array* {  // FoR(BitPacked) or BitPacked
        if (c && c->encoding == VXG_ENC_FL_FOR && child(*c, 0) && child(*c, 0)->encoding == VXG_ENC_FL_BITPACKED) {
            ep.reference = c->meta.for_.reference;
            ep.shift = c->meta.for_.shift;
            return child(*c, 0);
        }
        return c && c->encoding == VXG_ENC_FL_BITPACKED ? c : nullptr;
    };
    switch (a.encoding) {
    case VXG_ENC_FL_BITPACKED: bp = &a; break;  // bitpacking/compute/take.rs:21-125
    case VXG_ENC_FL_FOR:                          // for/compute.rs:39-48: take the child, keep the FoR
        bp = fl_child(&a);
        epi = Epi::For;
        break;
    case VXG_ENC_ZIGZAG:  // zigzag/compute.rs: take the encoded child, decode
        bp = fl_child(child(a, 0));
        epi = Epi::ForZigZag;
        break;
    case VXG_ENC_ALP: {  // alp/compute.rs: take the encoded child and the patches
        const bool f32 = a.ptype == VXG_F32;
        const unsigned e = a.meta.alp.e, f = a.meta.alp.f;
        if ((f32 && (e > 10 || f > 10)) || (!f32 && (a.ptype != VXG_F64 || e > 23 || f > 23))) return via_canonical();
        bp = fl_child(child(a, 0));
        epi = f32 ? Epi::AlpF32 : Epi::AlpF64;
        ep.alp_a = f32 ? double(kF10f[f]) : kF10d[f];
        ep.alp_b = f32 ? double(kIF10f[e]) : kIF10d[e];
        if (bp && a.meta.alp.has_patches) {
            if (!child(a, 1)) return set_error(VXG_ERR_INVALID_ARGUMENT, "ALPArray: patches child missing");
            VXG_TRY(take_patches(*child(a, 1), outer));
        }
        break;
    }
    case VXG_ENC_DICT: {  // dict/compute.rs:44-52: take the codes, then the values at them
        const vxg_array* values = child(a, 0);
        const vxg_array* codes = child(a, 1);
        if (!values || !codes || values->dtype != VXG_DTYPE_PRIMITIVE || !ptype_is_int(codes->ptype))
            return via_canonical();
        void* tc;
        VXG_TRY(temp(n * width(*codes), &tc));
        VXG_TRY(take_values(*codes, idx, iw, isg, n, tc));
        const void* pv;
        VXG_TRY(view_primitive(*values, &pv));
        return launch_take(width(*values), pv, values->len, width(*codes), false, tc, n, dst, ctx_->c.err_word, s_);
    }
    default: return via_canonical();
    }
    const int T = bp ? 8 * width(*bp) : 0;
    const bool t_ok = bp && (epi == Epi::AlpF32 ? T == 32 : epi == Epi::AlpF64 ? T == 64 : T == 8 * width(a));
    // bitpacking/compute/take.rs:23-31: many indices -> canonicalize and take the primitive
    if (!t_ok || bp->len != a.len || n * 8 > a.len) return via_canonical();
    const vxg_buffer* pb = buf(*bp, 0);
    const unsigned W = bp->meta.bitpacked.bit_width, off = bp->meta.bitpacked.offset;
    if (off > 1023) return set_error(VXG_ERR_INVALID_ARGUMENT, "Offset must be less than full block, i.e. 1024");
    if (W > unsigned(T)) return set_error(VXG_ERR_INVALID_ARGUMENT, "Unsupported bit width");
    const uint64_t nblk = (bp->len + off + 1023) / 1024, have = pb ? pb->len : 0;
    if (W > 0 && have != nblk * 128ull * W)  // bitpacking/mod.rs:80-88
        return set_error(VXG_ERR_INVALID_ARGUMENT, "Expected " + std::to_string(nblk * 128ull * W) +
                                                       " packed bytes, got " + std::to_string(have));
    TakePacked t{};
    t.packed = pb ? static_cast<const uint8_t*>(pb->ptr) : nullptr;
    t.W = W;
    t.offset = off;
    t.len = a.len;
    t.idx = idx;
    t.iw = iw;
    t.isg = isg;
    t.n = n;
    t.out = dst;
    t.ep = ep;
    t.outer = outer;
    t.err = ctx_->c.err_word;
    if (bp->meta.bitpacked.has_patches) {  // take.rs:127-200: patches of the taken positions
        if (!child(*bp, 0)) return set_error(VXG_ERR_INVALID_ARGUMENT, "BitPacked patches child missing");
        VXG_TRY(take_patches(*child(*bp, 0), t.inner));
    }
    return launch_take_packed(T, epi, t, s_);
}

vxg_status Planner::take(const vxg_array& a, const void* idx, int iw, bool isg, uint64_t n, vxg_canonical& out) {
    if (a.dtype != VXG_DTYPE_PRIMITIVE) return set_error(VXG_ERR_NOT_IMPLEMENTED, "take supports primitive arrays");
    out.kind = VXG_ENC_PRIMITIVE;
    out.len = n;
    out.dtype = a.dtype;
    out.ptype = a.ptype;
    out.values_bytes = n * width(a);
    if (!out.values)
        VXG_TRY(hip_check(hipMalloc(&out.values, out.values_bytes ? out.values_bytes : 16), "take values alloc"));
    VXG_TRY(take_values(a, idx, iw, isg, n, out.values));
    const vxg_array* node;
    int kind;
    VXG_TRY(validity_source(a, &node, &kind));
    if (kind == 0) {  // validity.take of NonNullable / AllValid: no nulls
        out.validity = nullptr;
        return VXG_OK;
    }
    void* src = nullptr;  // the array's validity, then taken at the indices
    VXG_TRY(temp(((a.len + 31) / 32) * 4, &src));
    VXG_TRY(validity_into(a, &src));
    const uint64_t bytes = ((n + 31) / 32) * 4;
    if (!out.validity) VXG_TRY(hip_check(hipMalloc(&out.validity, bytes ? bytes : 4), "take validity alloc"));
    return launch_gather_bits(out.validity, idx, iw, isg, n, static_cast<const uint8_t*>(src), a.len, ctx_->c.err_word,
                              s_);
}

// compute::filter (compute/filter.rs:23-52).  The predicate (any Bool encoding) becomes a bit
// buffer padded to whole u64 words; one sync reads the true count (the filtered length the
// reference's Array carries); the array is canonicalized into temporaries and compacted.
// Strings get a new single heap of the selected rows' bytes (VarBin/FSST filter, then
// varbin/flatten.rs), null rows as empty values.
vxg_status Planner::filter(const vxg_array& a, const vxg_array& pred, vxg_canonical& out) {
    if (pred.dtype != VXG_DTYPE_BOOL || pred.nullable)  // filter.rs:27-32
        return set_error(VXG_ERR_INVALID_ARGUMENT, "predicate must be non-nullable bool");
    if (pred.len != a.len)  // filter.rs:33-39
        return set_error(VXG_ERR_INVALID_ARGUMENT, "predicate.len() is " + std::to_string(pred.len) +
                                                       ", does not equal array.len() of " + std::to_string(a.len));
    const bool is_str = a.dtype == VXG_DTYPE_UTF8 || a.dtype == VXG_DTYPE_BINARY;
    if (!is_str && a.dtype != VXG_DTYPE_BOOL && a.dtype != VXG_DTYPE_PRIMITIVE)
        return set_error(VXG_ERR_NOT_IMPLEMENTED, "filter supports primitive, bool and utf8/binary dtypes");
    const uint64_t n = a.len, tiles = filter_tiles(n);
    void* mask;
    VXG_TRY(temp(((n + 63) / 64) * 8, &mask));
    VXG_TRY(launch_copy_bytes(mask, nullptr, ((n + 63) / 64) * 8, s_));
    VXG_TRY(bools_into(pred, mask, 0));
    void* toff;
    VXG_TRY(temp((tiles + 1) * 8, &toff));
    const uint64_t* m = static_cast<const uint64_t*>(mask);
    uint64_t* to = static_cast<uint64_t*>(toff);
    VXG_TRY(launch_filter_count(m, n, to, s_));
    uint64_t k = 0;
    VXG_TRY(hip_check(hipMemcpyAsync(&k, to + tiles, 8, hipMemcpyDeviceToHost, s_), "filter count readback"));
    VXG_TRY(hip_check(hipStreamSynchronize(s_), "filter count sync"));

    // canonical source in temporaries
    vxg_canonical src{};
    const vxg_array* vnode;
    int vkind;
    VXG_TRY(validity_source(a, &vnode, &vkind));
    if (vkind != 0) VXG_TRY(temp(((n + 31) / 32) * 4, &src.validity));
    std::vector<vxg_data_buffer> bufs;
    if (is_str) {
        uint64_t extent;
        VXG_TRY(string_layout(a, bufs, extent));
        VXG_TRY(temp(16 * n, &src.views));
        VXG_TRY(temp(extent + 16, &src.data));
        src.data_bytes = extent;
        src.data_buffers = bufs.data();
        src.n_data_buffers = src.data_buffers_cap = uint32_t(bufs.size());
    } else if (a.dtype == VXG_DTYPE_BOOL) {
        VXG_TRY(temp(((n + 31) / 32) * 4, &src.values));
    } else {
        VXG_TRY(temp(n * width(a), &src.values));
    }
    VXG_TRY(canonical(a, src));

    out.kind = src.kind;
    out.len = k;
    out.dtype = a.dtype;
    out.ptype = a.ptype;
    const uint64_t vbits = ((k + 31) / 32) * 4;
    if (src.validity) {  // validity.filter(predicate)
        if (!out.validity) VXG_TRY(hip_check(hipMalloc(&out.validity, vbits ? vbits : 4), "filter validity alloc"));
        VXG_TRY(launch_copy_bytes(out.validity, nullptr, vbits ? vbits : 4, s_));
        VXG_TRY(launch_filter_bits(m, n, to, static_cast<const uint8_t*>(src.validity), out.validity, s_));
    } else {
        out.validity = nullptr;
    }
    if (a.dtype == VXG_DTYPE_PRIMITIVE) {
        out.values_bytes = k * width(a);
        if (!out.values)
            VXG_TRY(hip_check(hipMalloc(&out.values, out.values_bytes ? out.values_bytes : 16), "filter values alloc"));
        return launch_filter_values(m, n, to, src.values, width(a), out.values, s_);
    }
    if (a.dtype == VXG_DTYPE_BOOL) {
        out.values_bytes = vbits;
        if (!out.values) VXG_TRY(hip_check(hipMalloc(&out.values, vbits ? vbits : 4), "filter bool alloc"));
        VXG_TRY(launch_copy_bytes(out.values, nullptr, vbits ? vbits : 4, s_));
        return launch_filter_bits(m, n, to, static_cast<const uint8_t*>(src.values), out.values, s_);
    }
    // strings: compact the views, then rebuild one heap of the selected rows
    if (!out.views) VXG_TRY(hip_check(hipMalloc(&out.views, k ? 16 * k : 16), "filter views alloc"));
    VXG_TRY(launch_filter_values(m, n, to, src.views, 16, out.views, s_));
    const uint64_t ktiles = filter_tiles(k);
    void* hoff;
    VXG_TRY(temp((ktiles + 1) * 8, &hoff));
    uint8_t* views = static_cast<uint8_t*>(out.views);
    const uint8_t* valid = static_cast<const uint8_t*>(out.validity);
    VXG_TRY(launch_view_heap_sizes(views, k, valid, static_cast<uint64_t*>(hoff), s_));
    uint64_t heap = 0;
    VXG_TRY(hip_check(hipMemcpyAsync(&heap, static_cast<uint64_t*>(hoff) + ktiles, 8, hipMemcpyDeviceToHost, s_),
                      "filter heap readback"));
    VXG_TRY(hip_check(hipStreamSynchronize(s_), "filter heap sync"));
    if (heap > 0xFFFFFFFFull) return set_error(VXG_ERR_INVALID_ARGUMENT, "filtered string heap exceeds u32 view offsets");
    if (out.data && out.data_bytes < heap)
        return set_error(VXG_ERR_INVALID_ARGUMENT, "caller-provided data holds " + std::to_string(out.data_bytes) +
                                                       " bytes, the filtered heap needs " + std::to_string(heap));
    if (!out.data) VXG_TRY(hip_check(hipMalloc(&out.data, heap + 16), "filter heap alloc"));
    out.data_bytes = heap;
    out.n_data_buffers = 1;
    if (out.data_buffers && out.data_buffers_cap >= 1) out.data_buffers[0] = vxg_data_buffer{0, heap};
    std::vector<const uint8_t*> bases(bufs.size());
    for (size_t i = 0; i < bufs.size(); ++i) bases[i] = static_cast<const uint8_t*>(src.data) + bufs[i].offset;
    void* dbases;
    VXG_TRY(temp(bases.size() * sizeof(void*) + 8, &dbases));
    if (!bases.empty())
        VXG_TRY(hip_check(hipMemcpyAsync(dbases, bases.data(), bases.size() * sizeof(void*), hipMemcpyHostToDevice, s_),
                          "filter buffer table upload"));
    VXG_TRY(launch_view_heap_build(views, k, valid, static_cast<uint64_t*>(hoff),
                                   static_cast<const uint8_t* const*>(dbases), uint32_t(bases.size()),
                                   static_cast<uint8_t*>(out.data), ctx_->c.err_word, s_));
    return hip_check(hipStreamSynchronize(s_), "filter sync");  // `bases` is read by the upload
}

// ---- bools: canonical BoolArray = LSB bit buffer (bool/mod.rs), from every Bool encoding ----
vxg_status Planner::bools_into(const vxg_array& a, void* bits, uint64_t off) {
    if (a.dtype != VXG_DTYPE_BOOL) return set_error(VXG_ERR_MISMATCHED_TYPES, "expected a Bool array");
    if (a.len == 0) return VXG_OK;
    switch (a.encoding) {
    case VXG_ENC_BOOL: {  // bool/mod.rs:25-28: bits from first_byte_bit_offset
        const vxg_buffer* b = buf(a, 0);
        const uint64_t fbo = a.meta.boolean.first_byte_bit_offset;
        if (!b || b->len * 8 < fbo + a.len) return set_error(VXG_ERR_INVALID_ARGUMENT, "BoolArray buffer too short");
        return launch_copy_bits(bits, off, static_cast<const uint8_t*>(b->ptr), fbo, a.len, false, s_);
    }
    case VXG_ENC_BYTE_BOOL: {  // bytebool/src/array.rs:138-146
        const vxg_buffer* b = buf(a, 0);
        if (!b || b->len < a.len) return set_error(VXG_ERR_INVALID_ARGUMENT, "ByteBoolArray buffer too short");
        return launch_bytebool(static_cast<const uint8_t*>(b->ptr), a.len, bits, off, s_);
    }
    case VXG_ENC_RUN_END_BOOL: {  // runend-bool/src/array.rs:152-163 -> compress.rs:46-93
        const vxg_array* e = child(a, 0);
        if (!e || e->len == 0) return set_error(VXG_ERR_INVALID_ARGUMENT, "Ends array must have at least one element");
        if (!ptype_is_unsigned(e->ptype))
            return set_error(VXG_ERR_INVALID_ARGUMENT, "Ends array must be an unsigned integer type");
        const void* pe;
        VXG_TRY(view_primitive(*e, &pe));
        return launch_runend_bool(pe, width(*e), e->len, a.meta.runendbool.offset, a.meta.runendbool.start != 0,
                                  a.len, bits, off, ctx_->c.err_word, s_);
    }
    case VXG_ENC_ROARING_BOOL: {  // roaring/src/boolean/mod.rs:127-147 (K16, roaring.hip)
        const vxg_buffer* b = buf(a, 0);
        if (!b) return set_error(VXG_ERR_INVALID_ARGUMENT, "RoaringBoolArray without buffer");
        return launch_roaring_bool(static_cast<const uint8_t*>(b->ptr), b->len, a.len, bits, off, ctx_->c.err_word, s_);
    }
    case VXG_ENC_CONSTANT:  // constant/canonical.rs:26-33: new_set / new_unset
        if (!a.meta.constant.is_null && a.meta.constant.scalar[0])
            return launch_copy_bits(bits, off, nullptr, 0, a.len, true, s_);
        return VXG_OK;
    case VXG_ENC_SPARSE: {  // sparse/flatten.rs:41-61 canonicalize_sparse_bools
        const vxg_array* idx = child(a, 0);
        const vxg_array* val = child(a, 1);
        if (!idx || !val || idx->len != val->len)
            return set_error(VXG_ERR_INVALID_ARGUMENT, "Sparse needs indices and values of equal length");
        if (!a.meta.sparse.fill_is_null && a.meta.sparse.fill[0])
            VXG_TRY(launch_copy_bits(bits, off, nullptr, 0, a.len, true, s_));
        if (idx->len == 0) return VXG_OK;
        void* vb;
        const uint64_t vbytes = ((val->len + 31) / 32) * 4;
        VXG_TRY(temp(vbytes, &vb));
        VXG_TRY(launch_copy_bytes(vb, nullptr, vbytes, s_));
        VXG_TRY(bools_into(*val, vb, 0));
        const void* pi;
        VXG_TRY(view_primitive(*idx, &pi));
        return launch_assign_bits_at(bits, off, pi, width(*idx), ptype_is_signed(idx->ptype),
                                     a.meta.sparse.indices_offset, idx->len, a.len, static_cast<const uint8_t*>(vb), s_);
    }
    case VXG_ENC_CHUNKED: {  // chunked/canonical.rs:154-163 pack_bools
        uint64_t o = 0;
        for (uint32_t i = 1; i < a.n_children; i++) {
            VXG_TRY(bools_into(a.children[i], bits, off + o));
            o += a.children[i].len;
        }
        if (o != a.len) return set_error(VXG_ERR_INVALID_ARGUMENT, "Chunked len != sum of chunk lens");
        return VXG_OK;
    }
    default:
        return set_error(VXG_ERR_NOT_IMPLEMENTED, "bool canonicalize for encoding id " + std::to_string(a.encoding));
    }
}

// ---- strings: VarBin, VarBinView, FSST, Dict(strings), Chunked (pack_views) -------------
// Every string canonical is a VarBinView (canonical.rs:56-63).  Its data buffers: one per
// VarBin / FSST leaf (the bytes buffer / the decoded heap), a Dict's are its values', a
// VarBinView input keeps its own, and a ChunkedArray concatenates its chunks' lists with each
// chunk's buffer_index rebased by the buffers before it (chunked/canonical.rs:194-236).
vxg_status Planner::string_buffer_count(const vxg_array& a, uint32_t& n) {
    switch (a.encoding) {
    case VXG_ENC_VARBIN:
    case VXG_ENC_FSST: n = 1; return VXG_OK;
    case VXG_ENC_VARBINVIEW: n = a.meta.varbinview.n_buffers; return VXG_OK;
    case VXG_ENC_DICT:
        if (a.n_children < 1) return set_error(VXG_ERR_INVALID_ARGUMENT, "DictArray needs values and codes");
        return string_buffer_count(a.children[0], n);
    case VXG_ENC_CHUNKED: {
        uint32_t t = 0;
        for (uint32_t i = 1; i < a.n_children; i++) {
            uint32_t k;
            VXG_TRY(string_buffer_count(a.children[i], k));
            t += k;
        }
        n = t;
        return VXG_OK;
    }
    default:
        return set_error(VXG_ERR_NOT_IMPLEMENTED, "string canonicalize for encoding id " + std::to_string(a.encoding));
    }
}

// Buffer lengths in order; FSST heap sizes (sum of uncompressed lengths) are device sums
// recorded in `fsst` as (slot, node) and resolved by string_layout with one readback.
vxg_status Planner::string_lens(const vxg_array& a, std::vector<uint64_t>& lens,
                                std::vector<std::pair<size_t, const vxg_array*>>& fsst) const {
    switch (a.encoding) {
    case VXG_ENC_VARBIN: {
        const vxg_array* bytes = child(a, 1);
        if (!bytes) return set_error(VXG_ERR_INVALID_ARGUMENT, "VarBinArray needs offsets and bytes");
        lens.push_back(bytes->len);
        return VXG_OK;
    }
    case VXG_ENC_VARBINVIEW:
        if (a.n_children < 1 + a.meta.varbinview.n_buffers)
            return set_error(VXG_ERR_INVALID_ARGUMENT, "VarBinViewArray: missing views/data buffers");
        for (uint32_t b = 0; b < a.meta.varbinview.n_buffers; b++) lens.push_back(a.children[1 + b].len);
        return VXG_OK;
    case VXG_ENC_FSST:
        if (!child(a, 3)) return set_error(VXG_ERR_INVALID_ARGUMENT, "FSST lengths child missing");
        fsst.emplace_back(lens.size(), &a);
        lens.push_back(0);
        return VXG_OK;
    case VXG_ENC_DICT:
        if (!child(a, 0)) return set_error(VXG_ERR_INVALID_ARGUMENT, "DictArray needs values and codes");
        return string_lens(a.children[0], lens, fsst);
    case VXG_ENC_CHUNKED:
        for (uint32_t i = 1; i < a.n_children; i++) VXG_TRY(string_lens(a.children[i], lens, fsst));
        return VXG_OK;
    default:
        return set_error(VXG_ERR_NOT_IMPLEMENTED, "string canonicalize for encoding id " + std::to_string(a.encoding));
    }
}

vxg_status Planner::string_layout(const vxg_array& a, std::vector<vxg_data_buffer>& bufs, uint64_t& extent) {
    std::vector<uint64_t> lens;
    std::vector<std::pair<size_t, const vxg_array*>> fsst;
    VXG_TRY(string_lens(a, lens, fsst));
    if (!fsst.empty()) {  // fsst/canonical.rs:29-42: heap size = sum of uncompressed lengths
        void* d;
        VXG_TRY(temp(8 * fsst.size(), &d));
        for (size_t k = 0; k < fsst.size(); k++) {
            const vxg_array& ul = *child(*fsst[k].second, 3);
            const void* pul;
            VXG_TRY(view_primitive(ul, &pul));
            VXG_TRY(launch_sum(pul, width(ul), ptype_is_signed(ul.ptype), ul.len, static_cast<uint64_t*>(d) + k, s_));
        }
        std::vector<uint64_t> h(fsst.size());
        VXG_TRY(hip_check(hipMemcpyAsync(h.data(), d, 8 * h.size(), hipMemcpyDeviceToHost, s_), "sum readback"));
        VXG_TRY(hip_check(hipStreamSynchronize(s_), "sum sync"));
        for (size_t k = 0; k < fsst.size(); k++) lens[fsst[k].first] = h[k];
    }
    bufs.resize(lens.size());
    uint64_t off = 0;
    for (size_t b = 0; b < lens.size(); b++) {
        bufs[b] = vxg_data_buffer{off, lens[b]};
        off = (off + lens[b] + 15) & ~15ull;
    }
    extent = lens.empty() ? 0 : bufs.back().offset + bufs.back().len;
    return VXG_OK;
}

// Canonical views of `a` into `views`, its data buffers into `data` at bufs[0..k), non-inlined
// views carrying buffer_index bidx + (buffer within a).  `validity`: a's LSB bitmap or NULL.
vxg_status Planner::strings_into(const vxg_array& a, uint8_t* views, uint8_t* data, const vxg_data_buffer* bufs,
                                 uint32_t bidx, const uint8_t* validity) {
    switch (a.encoding) {
    case VXG_ENC_VARBIN: {
        // varbin/flatten.rs:10-17: views over the whole bytes buffer (arrow-cast Utf8 -> Utf8View)
        const vxg_array* offs = child(a, 0);
        const vxg_array* bytes = child(a, 1);
        const void *po, *pb;
        VXG_TRY(view_primitive(*offs, &po));
        VXG_TRY(view_primitive(*bytes, &pb));
        uint8_t* heap = data + bufs[0].offset;
        if (bufs[0].len)
            VXG_TRY(launch_copy_bytes(heap, pb, bufs[0].len, s_));
        return launch_varbin_views(heap, bufs[0].len, width(*offs), po, a.len, validity, bidx, views, ctx_->c.err_word, s_);
    }
    case VXG_ENC_VARBINVIEW: {
        // already canonical: views (rebased) and buffers copied into the output layout
        const vxg_array* vw = child(a, 0);
        const void* pv;
        VXG_TRY(view_primitive(*vw, &pv));
        if (vw->len < 16 * a.len) return set_error(VXG_ERR_INVALID_ARGUMENT, "VarBinView views shorter than 16 * len");
        VXG_TRY(launch_views_rebase(static_cast<const uint8_t*>(pv), a.len, bidx, views, s_));
        for (uint32_t b = 0; b < a.meta.varbinview.n_buffers; b++) {
            const void* pb;
            VXG_TRY(view_primitive(a.children[1 + b], &pb));
            if (bufs[b].len)
                VXG_TRY(launch_copy_bytes(data + bufs[b].offset, pb, bufs[b].len, s_));
        }
        return VXG_OK;
    }
    case VXG_ENC_FSST: {
        // fsst/canonical.rs:7-57
        const vxg_array* sym = child(a, 0);
        const vxg_array* slen = child(a, 1);
        const vxg_array* codes = child(a, 2);
        const vxg_array* ulen = child(a, 3);
        if (!sym || !slen || !codes || !ulen || codes->encoding != VXG_ENC_VARBIN)
            return set_error(VXG_ERR_INVALID_ARGUMENT, "FSSTArray needs symbols, lengths, VarBin codes, lengths");
        const void *psym, *pslen, *pcb;
        VXG_TRY(view_primitive(*sym, &psym));
        VXG_TRY(view_primitive(*slen, &pslen));
        VXG_TRY(view_primitive(*child(*codes, 1), &pcb));
        FsstChunk f{};
        f.symbols = static_cast<const uint64_t*>(psym);
        f.sym_lens = static_cast<const uint8_t*>(pslen);
        f.n_symbols = unsigned(sym->len);
        f.codes = static_cast<const uint8_t*>(pcb);
        VXG_TRY(int_column(*child(*codes, 0), f.offs));  // read in place by the FSST kernels
        VXG_TRY(int_column(*ulen, f.lens));              // (packed columns stay packed)
        f.n = a.len;
        f.validity = validity;
        f.heap = data + bufs[0].offset;
        f.heap_len = bufs[0].len;
        f.views = views;
        f.bidx = bidx;
        if (fsst_batch_) {  // a chunk: decoded with the other FSST chunks
            fsst_batch_->push_back(f);
            return VXG_OK;
        }
        std::vector<FsstChunk> one{f};
        void* scratch;
        VXG_TRY(temp(fsst_batch_scratch_bytes(one.data(), 1), &scratch));
        return launch_fsst_batch(one, scratch, ctx_->c.err_word, s_, plan_);
    }
    case VXG_ENC_DICT: {
        // Dict over string values: take on the values' views (varbinview/compute.rs:68-76); the
        // values' buffers are the result's buffers, so they decode straight into the output
        const vxg_array* values = child(a, 0);
        const vxg_array* codes = child(a, 1);
        if (!values || !codes) return set_error(VXG_ERR_INVALID_ARGUMENT, "DictArray needs values and codes");
        const vxg_array* vn;
        int vk;
        VXG_TRY(validity_source(*values, &vn, &vk));
        void* vbits = nullptr;  // nullable values: their null rows get zero views before the take
        if (vk != 0) {
            VXG_TRY(temp(((values->len + 31) / 32) * 4, &vbits));
            VXG_TRY(validity_into(*values, &vbits));
        }
        void* vviews;
        VXG_TRY(temp(16 * values->len, &vviews));
        VXG_TRY(strings_into(*values, static_cast<uint8_t*>(vviews), data, bufs, bidx,
                             static_cast<const uint8_t*>(vbits)));
        if (codes->encoding == VXG_ENC_FL_BITPACKED && codes->meta.bitpacked.bit_width <= kDictFusedMaxW) {
            UnpackArgs ua{};
            ua.dict = vviews;
            ua.dict_len = values->len;
            return decode_bitpacked(*codes, Epi::Dict, 16, ua, views);
        }
        const void* pc;
        VXG_TRY(view_primitive(*codes, &pc));
        return launch_take(16, vviews, values->len, width(*codes), false, pc, a.len, views, ctx_->c.err_word, s_);
    }
    case VXG_ENC_CHUNKED: {
        // pack_views (chunked/canonical.rs:194-236): each chunk's views go to its slice of the
        // output, its buffers after the preceding chunks', buffer_index rebased accordingly.
        // Dict(VarBin values, BitPacked codes) chunks share launches: one batched
        // views-and-bytes launch for all their dictionaries, one grouped K1 gather.
        const uint64_t n = a.meta.chunked.nchunks;
        if (a.n_children != n + 1) return set_error(VXG_ERR_INVALID_ARGUMENT, "Chunked child count != nchunks + 1");
        auto dict_batchable = [&](const vxg_array& c) {
            if (c.encoding != VXG_ENC_DICT || c.n_children < 2) return false;
            const vxg_array& v = c.children[0];
            const vxg_array& k = c.children[1];
            return v.encoding == VXG_ENC_VARBIN && v.validity != VXG_VALIDITY_ARRAY &&
                   v.validity != VXG_VALIDITY_ALL_INVALID && v.n_children >= 2 &&
                   v.children[0].encoding == VXG_ENC_PRIMITIVE && v.children[1].encoding == VXG_ENC_PRIMITIVE &&
                   k.encoding == VXG_ENC_FL_BITPACKED && ptype_is_unsigned(k.ptype) && !k.nullable &&
                   k.meta.bitpacked.bit_width <= kDictFusedMaxW;
        };
        uint64_t dict_rows = 0;
        for (uint64_t i = 0; i < n; i++)
            if (dict_batchable(a.children[i + 1])) dict_rows += a.children[i + 1].children[0].len;
        uint8_t* dviews = nullptr;
        if (dict_rows) {
            void* t;
            VXG_TRY(temp(16 * dict_rows, &t));
            dviews = static_cast<uint8_t*>(t);
        }
        std::vector<VarBinChunk> dicts;
        std::vector<K1Job> jobs;
        std::vector<PatchJob> patches;
        std::vector<FsstChunk> fssts;
        uint64_t row = 0;
        uint32_t b = 0;
        for (uint64_t i = 0; i < n; i++) {
            const vxg_array& c = a.children[i + 1];
            if (c.dtype != a.dtype) return set_error(VXG_ERR_MISMATCHED_TYPES, "Chunks must have the ChunkedArray's dtype");
            uint32_t k;
            VXG_TRY(string_buffer_count(c, k));
            if (dict_batchable(c)) {
                const vxg_array& v = c.children[0];
                const void *po, *pb;
                VXG_TRY(view_primitive(v.children[0], &po));
                VXG_TRY(view_primitive(v.children[1], &pb));
                VarBinChunk d{};
                d.src = static_cast<const uint8_t*>(pb);
                d.dst = data + bufs[b].offset;
                d.offsets = po;
                d.views = dviews;
                d.bytes = bufs[b].len;
                d.n = v.len;
                d.offs_width = uint32_t(width(v.children[0]));
                d.bidx = bidx + b;
                // a plan batch with a small dictionary: K1g builds its views in LDS (no views
                // launch); otherwise the views are built into dviews first
                const vxg_array& codes = c.children[1];
                // also in an unbatched plan (its own K1g launch per column instead of a views
                // launch + K14: VXG_PLAN_VB_K1G=0 restores those)
                const bool vb = (defer(a) || (plan_ && plan_vb_k1g())) && v.len <= kGenVarBinDictMax && v.len > 0 &&
                                codes.len > 0 && !codes.meta.bitpacked.has_patches;
                if (!vb) dicts.push_back(d);
                UnpackArgs ua{};
                ua.dict = vb ? nullptr : dviews;
                ua.dict_len = v.len;
                dviews += 16 * v.len;
                k1_batch_ = &jobs;
                patch_batch_ = &patches;
                const size_t nj = jobs.size(), np = patches.size();
                const vxg_status st = decode_bitpacked(c.children[1], Epi::Dict, 16, ua, views + 16 * row);
                k1_batch_ = nullptr;
                patch_batch_ = nullptr;
                VXG_TRY(st);
                if (vb) {
                    if (jobs.size() != nj + 1 || patches.size() != np)
                        return set_error(VXG_ERR_INVALID_ARGUMENT, "internal: VarBin-dictionary job shape");
                    jobs.back().vb = true;
                    jobs.back().vbc = d;
                }
            } else {
                void* cv = nullptr;  // the chunk's own validity (null views are all-zero)
                const vxg_array* vn;
                int vk;
                VXG_TRY(validity_source(c, &vn, &vk));
                if (vk != 0) {
                    VXG_TRY(temp(((c.len + 31) / 32) * 4, &cv));
                    VXG_TRY(validity_into(c, &cv));
                }
                if (c.encoding == VXG_ENC_FSST) fsst_batch_ = &fssts;
                const vxg_status st =
                    strings_into(c, views + 16 * row, data, bufs + b, bidx + b, static_cast<const uint8_t*>(cv));
                fsst_batch_ = nullptr;
                VXG_TRY(st);
            }
            row += c.len;
            b += k;
        }
        if (row != a.len) return set_error(VXG_ERR_INVALID_ARGUMENT, "Chunked len != sum of chunk lens");
        if (!fssts.empty() && defer(a)) {  // a plan's root: decoded at the batch's flush
            batch_->fssts.insert(batch_->fssts.end(), fssts.begin(), fssts.end());
        } else if (!fssts.empty()) {
            void* scratch;
            VXG_TRY(temp(fsst_batch_scratch_bytes(fssts.data(), fssts.size()), &scratch));
            VXG_TRY(launch_fsst_batch(fssts, scratch, ctx_->c.err_word, s_, plan_));
        }
        if (defer(a) && patches.empty()) {  // a plan's root: launched with the other arrays' jobs (PlanBatch)
            batch_->dicts.insert(batch_->dicts.end(), dicts.begin(), dicts.end());
            batch_->jobs.insert(batch_->jobs.end(), jobs.begin(), jobs.end());
            return VXG_OK;
        }
        VXG_TRY(launch_varbin_dicts(dicts, ctx_->c.err_word, s_, plan_));
        VXG_TRY(launch_k1_jobs(jobs, ctx_->c.err_word, s_, plan_));
        for (const PatchJob& p : patches) VXG_TRY(apply_sparse_patches(*p.sp, p.T, p.epi, p.vw, p.a, p.dst, p.out_len));
        return VXG_OK;
    }
    default:
        return set_error(VXG_ERR_NOT_IMPLEMENTED, "string canonicalize for encoding id " + std::to_string(a.encoding));
    }
}

vxg_status Planner::string_canonical(const vxg_array& a, vxg_canonical& out) {
    out.kind = VXG_ENC_VARBINVIEW;
    out.len = a.len;
    out.dtype = a.dtype;
    uint32_t nb;
    VXG_TRY(string_buffer_count(a, nb));
    std::vector<vxg_data_buffer> bufs;
    if (out.views && out.data) {
        // caller-allocated (sized with vxg_canonical_layout / _size): no device sum + sync on
        // the decode path
        if (nb == 1) {
            bufs.push_back(vxg_data_buffer{0, out.data_bytes});
        } else {
            if (!out.data_buffers || out.n_data_buffers != nb)
                return set_error(VXG_ERR_INVALID_ARGUMENT, "caller-provided data needs the vxg_canonical_layout buffer table (" +
                                                               std::to_string(nb) + " buffers)");
            bufs.assign(out.data_buffers, out.data_buffers + nb);
        }
    } else {
        uint64_t extent;
        VXG_TRY(string_layout(a, bufs, extent));
        if (nb > 1 && (!out.data_buffers || out.data_buffers_cap < nb))
            return set_error(VXG_ERR_INVALID_ARGUMENT, "data_buffers must have room for " + std::to_string(nb) + " buffers");
        if (!out.views) VXG_TRY(hip_check(hipMalloc(&out.views, a.len ? 16 * a.len : 16), "views alloc"));
        if (!out.data) VXG_TRY(hip_check(hipMalloc(&out.data, extent + 16), "data alloc"));
        out.data_bytes = extent;
    }
    out.n_data_buffers = nb;
    if (out.data_buffers && out.data_buffers_cap >= nb && out.data_buffers != bufs.data())
        std::copy(bufs.begin(), bufs.end(), out.data_buffers);
    VXG_TRY(validity_into(a, &out.validity));
    return strings_into(a, static_cast<uint8_t*>(out.views), static_cast<uint8_t*>(out.data), bufs.data(), 0,
                        static_cast<const uint8_t*>(out.validity));
}

vxg_status Planner::canonical_size(const vxg_array& a, uint64_t& vb, uint64_t& db) {
    vb = db = 0;
    if (a.dtype == VXG_DTYPE_PRIMITIVE) {
        vb = a.len * width(a);
        return VXG_OK;
    }
    if (a.dtype == VXG_DTYPE_BOOL) {  // whole 32-bit words
        vb = ((a.len + 31) / 32) * 4;
        return VXG_OK;
    }
    if (a.dtype != VXG_DTYPE_UTF8 && a.dtype != VXG_DTYPE_BINARY)
        return set_error(VXG_ERR_NOT_IMPLEMENTED, "canonical size for this dtype");
    vb = a.len * 16;
    std::vector<vxg_data_buffer> bufs;
    return string_layout(a, bufs, db);
}

vxg_status Planner::canonical(const vxg_array& a, vxg_canonical& out) {
    root_ = &a;
    out.len = a.len;
    out.dtype = a.dtype;
    out.ptype = a.ptype;
    if (a.dtype == VXG_DTYPE_UTF8 || a.dtype == VXG_DTYPE_BINARY) return string_canonical(a, out);
    if (a.dtype == VXG_DTYPE_BOOL) {  // Canonical::Bool: LSB bit buffer + validity
        out.kind = VXG_ENC_BOOL;
        out.values_bytes = ((a.len + 31) / 32) * 4;
        if (!out.values)
            VXG_TRY(hip_check(hipMalloc(&out.values, out.values_bytes ? out.values_bytes : 4), "bool values alloc"));
        if (out.values_bytes)
            VXG_TRY(launch_copy_bytes(out.values, nullptr, out.values_bytes, s_));
        VXG_TRY(bools_into(a, out.values, 0));
        return validity_into(a, &out.validity);
    }
    if (a.dtype != VXG_DTYPE_PRIMITIVE)
        return set_error(VXG_ERR_NOT_IMPLEMENTED, "canonicalize supports primitive, bool and utf8/binary dtypes");
    out.kind = VXG_ENC_PRIMITIVE;
    out.values_bytes = a.len * width(a);
    if (!out.values)
        VXG_TRY(hip_check(hipMalloc(&out.values, out.values_bytes ? out.values_bytes : 16), "values alloc"));
    VXG_TRY(decode_into(a, out.values));
    return validity_into(a, &out.validity);
}

}  // namespace

// ===================================================================================
// C ABI
// ===================================================================================
// The device error word's bits -> the VortexError variant each one stands for.
static vxg_status status_of_err_word(uint32_t err) {
    if (err & kErrTakeOOB) return set_error(VXG_ERR_OUT_OF_BOUNDS, "take: index out of bounds");
    if (err & kErrPatchOOB) return set_error(VXG_ERR_OUT_OF_BOUNDS, "patch index out of bounds");
    if (err & kErrPatchOrder) return set_error(VXG_ERR_INVALID_ARGUMENT, "patch indices are not sorted");
    if (err & kErrRunEnd) return set_error(VXG_ERR_INVALID_ARGUMENT, "RunEnd ends do not cover the array");
    if (err & kErrFsst) return set_error(VXG_ERR_INVALID_ARGUMENT, "FSST codes do not decode to uncompressed_lengths");
    if (err & kErrRoaring) return set_error(VXG_ERR_INVALID_SERDE, "RoaringBool buffer is not a croaring Native bitmap");
    if (err & kErrVarBin) return set_error(VXG_ERR_INVALID_ARGUMENT, "VarBin offsets out of range of the bytes");
    if (err & kErrPlanSync)
        return set_error(VXG_ERR_ASSERTION_FAILED, "plan launch: in-grid pre-pass records never published "
                                                   "(overlapping replays of one plan?)");
    return set_error(VXG_ERR_ASSERTION_FAILED, "unknown device error bit");
}

extern "C" {

int vxg_abi_version(void) { return VXG_ABI_VERSION; }

const char* vxg_last_error(void) { return g_last_error.c_str(); }

vxg_status vxg_open(int device, vxg_ctx** out) {
    if (!out) return set_error(VXG_ERR_INVALID_ARGUMENT, "null out");
    int n = 0;
    VXG_TRY(hip_check(hipGetDeviceCount(&n), "hipGetDeviceCount"));
    if (device < 0 || device >= n) return set_error(VXG_ERR_INVALID_ARGUMENT, "no such device");
    VXG_TRY(hip_check(hipSetDevice(device), "hipSetDevice"));
    auto* c = new vxg_ctx();
    c->c.device = device;
    c->c.opt = default_options();
    hipError_t e = hipMalloc(&c->c.err_word, 16);
    if (e == hipSuccess) e = hipMemset(c->c.err_word, 0, 16);
    if (e == hipSuccess) {
        // Planner temporaries come from the device's stream-ordered pool; keep freed blocks
        // cached instead of returning them to the driver at every synchronisation (the default
        // threshold 0 made each canonicalize re-map its temporaries: ~25 us of host time).
        hipMemPool_t pool;
        uint64_t keep = ~0ull;
        if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess)
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
    if (e == hipSuccess) e = fsst_diag_init();  // (a synchronous copy: never inside a plan's capture)
    if (e != hipSuccess) {
        vxg_close(c);
        return hip_check(e, "context setup");
    }
    *out = c;
    return VXG_OK;
}

vxg_status vxg_set_option(vxg_ctx* ctx, int option, int64_t value) {
    if (!ctx) return set_error(VXG_ERR_INVALID_ARGUMENT, "null vxg_ctx");
    Options& o = ctx->c.opt;
    switch (option) {
    case VXG_OPT_K1W_MIN_GROUPS:
        if (value < 0 || value > (int64_t(1) << 31)) return set_error(VXG_ERR_INVALID_ARGUMENT, "K1W_MIN_GROUPS out of range");
        o.k1w_min_groups = value;
        return VXG_OK;
    case VXG_OPT_K1W_BPW:
        if (value < 0 || value > 32) return set_error(VXG_ERR_INVALID_ARGUMENT, "K1W_BPW must be in [0, 32]");
        o.k1w_bpw = value;
        return VXG_OK;
    case VXG_OPT_K1_WAVE:
        if (value < -1 || value > 2) return set_error(VXG_ERR_INVALID_ARGUMENT, "K1_WAVE must be -1, 0, 1 or 2");
        o.k1_wave = value;
        return VXG_OK;
    }
    return set_error(VXG_ERR_INVALID_ARGUMENT, "unknown option " + std::to_string(option));
}

vxg_status vxg_get_option(vxg_ctx* ctx, int option, int64_t* value) {
    if (!ctx || !value) return set_error(VXG_ERR_INVALID_ARGUMENT, "null argument");
    const Options& o = ctx->c.opt;
    switch (option) {
    case VXG_OPT_K1W_MIN_GROUPS: *value = o.k1w_min_groups; return VXG_OK;
    case VXG_OPT_K1W_BPW: *value = o.k1w_bpw; return VXG_OK;
    case VXG_OPT_K1_WAVE: *value = o.k1_wave; return VXG_OK;
    }
    return set_error(VXG_ERR_INVALID_ARGUMENT, "unknown option " + std::to_string(option));
}

vxg_status vxg_get_launch_stats(vxg_ctx* ctx, vxg_launch_stats* out, int reset) {
    if (!ctx || !out) return set_error(VXG_ERR_INVALID_ARGUMENT, "null argument");
    std::lock_guard<std::mutex> lk(ctx->c.mu);
    const LaunchStats& st = ctx->c.st;
    *out = vxg_launch_stats{};
    out->k1w_launches = st.k1w_launches;
    out->k1w_last_groups = st.k1w_last_groups;
    out->k1w_last_bpw = st.k1w_last_bpw;
    out->k1w_min_bpw = st.k1w_min_bpw;
    out->k1w_max_bpw = st.k1w_max_bpw;
    out->k1w_last_bpw_max = st.k1w_last_bpw_max;
    if (reset) ctx->c.st = LaunchStats{};
    return VXG_OK;
}

vxg_status vxg_close(vxg_ctx* ctx) {
    if (!ctx) return VXG_OK;
    if (g_cur_ctx == &ctx->c) g_cur_ctx = nullptr;
    (void)hipSetDevice(ctx->c.device);
    (void)hipDeviceSynchronize();
    if (ctx->c.err_word) (void)hipFree(ctx->c.err_word);
    delete ctx;
    return VXG_OK;
}

vxg_status vxg_alloc(vxg_ctx* ctx, uint64_t bytes, void** dptr) {
    VXG_TRY(use_device(ctx));
    return hip_check(hipMalloc(dptr, bytes ? bytes : 16), "hipMalloc");
}

vxg_status vxg_free(vxg_ctx* ctx, void* dptr) {
    VXG_TRY(use_device(ctx));
    return hip_check(hipFree(dptr), "hipFree");
}

vxg_status vxg_host_alloc(vxg_ctx* ctx, uint64_t bytes, void** hptr) {
    VXG_TRY(use_device(ctx));
    return hip_check(hipHostMalloc(hptr, bytes ? bytes : 16, hipHostMallocDefault), "hipHostMalloc");
}

vxg_status vxg_host_free(vxg_ctx* ctx, void* hptr) {
    VXG_TRY(use_device(ctx));
    return hip_check(hipHostFree(hptr), "hipHostFree");
}

vxg_status vxg_memcpy_h2d(vxg_ctx* ctx, void* dst, const void* src, uint64_t bytes, void* stream) {
    VXG_TRY(use_device(ctx));
    return hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, S(stream)), "h2d");
}

vxg_status vxg_memcpy_d2h(vxg_ctx* ctx, void* dst, const void* src, uint64_t bytes, void* stream) {
    VXG_TRY(use_device(ctx));
    return hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, S(stream)), "d2h");
}

vxg_status vxg_memcpy_d2d(vxg_ctx* ctx, void* dst, const void* src, uint64_t bytes, void* stream) {
    VXG_TRY(use_device(ctx));
    return hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, S(stream)), "d2d");
}

vxg_status vxg_stream_sync(vxg_ctx* ctx, void* stream) {
    VXG_TRY(use_device(ctx));
    VXG_TRY(hip_check(hipStreamSynchronize(S(stream)), "hipStreamSynchronize"));
    uint32_t err = 0;
    VXG_TRY(hip_check(hipMemcpy(&err, ctx->c.err_word, 4, hipMemcpyDeviceToHost), "error word readback"));
    if (err) {
        VXG_TRY(hip_check(hipMemset(ctx->c.err_word, 0, 4), "error word reset"));
        return status_of_err_word(err);
    }
    return VXG_OK;
}

vxg_status vxg_canonical_size(vxg_ctx* ctx, const vxg_array* a, uint64_t* values_bytes, uint64_t* data_bytes) {
    VXG_TRY(use_device(ctx));
    if (!a) return set_error(VXG_ERR_INVALID_ARGUMENT, "null array");
    Planner p(ctx, nullptr);
    uint64_t vb = 0, db = 0;
    VXG_TRY(p.canonical_size(*a, vb, db));
    if (values_bytes) *values_bytes = vb;
    if (data_bytes) *data_bytes = db;
    return VXG_OK;
}

vxg_status vxg_canonical_layout(vxg_ctx* ctx, const vxg_array* a, uint64_t* values_bytes, uint64_t* data_bytes,
                                vxg_data_buffer* bufs, uint32_t cap, uint32_t* n_bufs) {
    VXG_TRY(use_device(ctx));
    if (!a) return set_error(VXG_ERR_INVALID_ARGUMENT, "null array");
    Planner p(ctx, nullptr);
    uint64_t vb = 0, db = 0;
    uint32_t n = 0;
    if (a->dtype == VXG_DTYPE_UTF8 || a->dtype == VXG_DTYPE_BINARY) {
        std::vector<vxg_data_buffer> v;
        VXG_TRY(p.string_layout(*a, v, db));
        vb = 16 * a->len;
        n = uint32_t(v.size());
        if (bufs && cap < n) return set_error(VXG_ERR_INVALID_ARGUMENT, "buffer table too small");
        if (bufs) std::copy(v.begin(), v.end(), bufs);
    } else {
        VXG_TRY(p.canonical_size(*a, vb, db));
    }
    if (values_bytes) *values_bytes = vb;
    if (data_bytes) *data_bytes = db;
    if (n_bufs) *n_bufs = n;
    return VXG_OK;
}

vxg_status vxg_canonicalize(vxg_ctx* ctx, const vxg_array* a, vxg_canonical* out, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!a || !out) return set_error(VXG_ERR_INVALID_ARGUMENT, "null array/out");
    Planner p(ctx, S(stream));
    return p.canonical(*a, *out);
}

// ---- prepared canonicalize --------------------------------------------------------------
}  // extern "C"

// Bytes a canonicalize of `a` moves (every buffer of the tree read once + the canonical
// output written): the plan's branch-balancing weight.
static uint64_t tree_bytes(const vxg_array& a) {
    uint64_t b = 0;
    for (uint32_t i = 0; i < a.n_buffers; i++) b += a.buffers[i].len;
    for (uint32_t i = 0; i < a.n_children; i++) b += tree_bytes(a.children[i]);
    return b;
}

// Encoding that decides an array's decode kernel: the first non-Chunked node of its tree.
static uint16_t leading_encoding(const vxg_array& a) {
    return a.encoding == VXG_ENC_CHUNKED && a.n_children ? leading_encoding(a.children[0]) : a.encoding;
}

// Branch-balancing weight: estimated device time ~ bytes moved / the kernel's measured fraction
// of the HBM roofline (round 3, each lineitem column alone, profiles/r03_c5_columns_w1.jsonl):
// FSST 0.45, string dictionaries (16-byte views) 0.55, short-run RunEnd 0.34, other decodes ~0.7.
static uint64_t plan_cost(const vxg_array& a) {
    const bool str = a.dtype == VXG_DTYPE_UTF8 || a.dtype == VXG_DTYPE_BINARY;
    const uint64_t out = a.dtype == VXG_DTYPE_BOOL ? a.len / 8 : a.len * (str ? 16 : ptype_width(a.ptype));
    const uint64_t bytes = tree_bytes(a) + out;
    const uint16_t e = leading_encoding(a);
    const uint64_t pct = e == VXG_ENC_FSST ? 45 : e == VXG_ENC_RUN_END ? 34 : str ? 55 : 70;
    return bytes * 100 / pct;
}

// Parallel graph branches of a plan (VXG_PLAN_BRANCHES overrides, 1..16; 0 = unset).
static uint32_t plan_branches_env() {
    static const uint32_t nb = [] {
        const char* e = std::getenv("VXG_PLAN_BRANCHES");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return v >= 1 && v <= 16 ? uint32_t(v) : 0u;
    }();
    return nb;
}

// Plan batching (PlanBatch + K1g).  Whether it pays depends on the table (round 4: C5 per GPU at
// 8 / 4 GPUs measured 0.060 / 0.095 ms batched vs 0.120 / 0.131 unbatched, but 0.200 vs 0.180 at
// 2 GPUs; mixing batched and unbatched arrays was slower than either).  So VXG_PLAN_MEASURE
// records the plan both ways (unbatched on 2 graph branches, batched on 1) and keeps one by
// vxg_plan_select (3 interleaved timed replays each after one warm-up).  The knob
// VXG_PLAN_BATCH (read at every create) is a diagnostic: "0" unbatched, "1" batched, "mixed"
// (arrays whose output is <= VXG_PLAN_BATCH_MAX_BYTES batched, the others not), unset = measured.
// "s" batches only the string-dictionary columns (one K1g launch for all of them on a branch
// of its own, the other columns unbatched).
enum class BatchMode { Auto, Off, On, Mixed, Strings };
static BatchMode plan_batch_mode() {
    const char* e = std::getenv("VXG_PLAN_BATCH");
    if (!e || !*e) return BatchMode::Auto;
    if (e[0] == '0') return BatchMode::Off;
    if (e[0] == '1') return BatchMode::On;
    if (e[0] == 'm') return BatchMode::Mixed;
    if (e[0] == 's') return BatchMode::Strings;
    return BatchMode::Auto;
}
// A string column whose leading encoding is Dict (C5's four Dict(VarBin) columns).
static bool dict_string_column(const vxg_array& a) {
    const bool str = a.dtype == VXG_DTYPE_UTF8 || a.dtype == VXG_DTYPE_BINARY;
    if (!str) return false;
    if (a.encoding == VXG_ENC_CHUNKED) {
        for (uint32_t i = 1; i < a.n_children; i++)
            if (a.children[i].encoding != VXG_ENC_DICT) return false;
        return a.n_children > 1;
    }
    return a.encoding == VXG_ENC_DICT;
}
static uint64_t env_bytes(const char* name, uint64_t dflt) {
    const char* e = std::getenv(name);
    return e ? uint64_t(std::strtoull(e, nullptr, 10)) : dflt;
}
static uint64_t plan_batch_max_bytes() { return env_bytes("VXG_PLAN_BATCH_MAX_BYTES", uint64_t(64) << 20); }
// vxg_plan_create without VXG_PLAN_MEASURE records one candidate: batched.  (Round 4 kept
// unbatched plans above 400 MB of output: then every small-enough numeric column went to K1g's
// runtime-width body.  With K1g limited to groups below 20 MiB and the FSST decode inside the
// K1g launch, batched measured faster at every C5 size in round 5: 1 GPU 0.272 vs 0.289 ms,
// 2-GPU shard 0.145 vs 0.173, 4 0.072 vs 0.125, 8 0.042 vs 0.104.)

static uint64_t canonical_out_bytes(const vxg_array& a) {
    const bool str = a.dtype == VXG_DTYPE_UTF8 || a.dtype == VXG_DTYPE_BINARY;
    return a.dtype == VXG_DTYPE_BOOL ? a.len / 8 : a.len * (str ? 16 : ptype_width(a.ptype));
}

// A batched plan's fused FSST+K1g launch with the in-grid pre-pass (fsst.hip): its arguments live
// here so that every replay can give it a new record tag (FsstFusedArgs::tag).
struct FusedNode {
    FsstFusedArgs fa;
    const GenChunk* gtab;
    uint32_t gn, dict_off;
    bool dict_lds;
    uint32_t* err;
    uint64_t gpe;
    void* args[7];
    hipGraphNode_t node = nullptr;
    hipKernelNodeParams p{};
    explicit FusedNode(void** a) {
        fa = *static_cast<const FsstFusedArgs*>(a[0]);
        gtab = *static_cast<const GenChunk* const*>(a[1]);
        gn = *static_cast<const uint32_t*>(a[2]);
        dict_off = *static_cast<const uint32_t*>(a[3]);
        dict_lds = *static_cast<const bool*>(a[4]);
        err = *static_cast<uint32_t* const*>(a[5]);
        gpe = *static_cast<const uint64_t*>(a[6]);
        void* const mine[7] = {&fa, &gtab, &gn, &dict_off, &dict_lds, &err, &gpe};
        std::copy(mine, mine + 7, args);
    }
};

struct vxg_plan {
    vxg_ctx* ctx = nullptr;
    std::vector<std::unique_ptr<FusedNode>> fused;  // in-grid pre-pass launches (tag per replay)
    uint64_t launches = 0;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    DevTables store;  // the recorded launches' temporaries and device chunk tables
    // A recorded graph that is one short chain of kernels (a sharded scan after batching:
    // FSST pre-pass -> decode -> K1g) replays as direct launches of its kernel nodes: one stream,
    // no graph-to-graph dependency (a graph replay boundary cost ~14 us on the C5 shard).
    std::vector<hipKernelNodeParams> direct;
    bool batched = false;  // recorded with a PlanBatch (diagnostics)
    uint32_t branches = 0;
    vxg_plan_info info{};  // filled by vxg_plan_create_ex
};

// Direct replay of short kernel chains (VXG_PLAN_DIRECT=0 disables; at most
// VXG_PLAN_DIRECT_MAX nodes, default 16: C5's 1-GPU batched chain is 9 kernels, 0.2745 ms per
// step as a graph vs 0.2719 direct).  Read at every plan recording.
static size_t plan_direct_max() {
    const char* e = std::getenv("VXG_PLAN_DIRECT_MAX");
    return e ? size_t(std::strtoull(e, nullptr, 10)) : size_t(16);
}
static bool plan_direct_enabled() {
    const char* e = std::getenv("VXG_PLAN_DIRECT");
    return !(e && e[0] == '0');
}

// The kernel nodes of `g` in order if g is a chain of <= plan_direct_max() kernel nodes, else empty.
static std::vector<hipKernelNodeParams> kernel_chain(hipGraph_t g) {
    std::vector<hipKernelNodeParams> out;
    size_t nn = 0;
    if (hipGraphGetNodes(g, nullptr, &nn) != hipSuccess || nn == 0 || nn > plan_direct_max()) return out;
    std::vector<hipGraphNode_t> nodes(nn);
    if (hipGraphGetNodes(g, nodes.data(), &nn) != hipSuccess) return out;
    std::vector<hipGraphNode_t> dep(nn, nullptr);
    size_t roots = 0, root = 0;
    for (size_t i = 0; i < nn; i++) {
        hipGraphNodeType t{};
        if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess || t != hipGraphNodeTypeKernel) {
            if (std::getenv("VXG_PLAN_DEBUG")) std::fprintf(stderr, "plan: node %zu of %zu has type %d\n", i, nn, int(t));
            return out;
        }
        size_t nd = 0;
        if (hipGraphNodeGetDependencies(nodes[i], nullptr, &nd) != hipSuccess || nd > 1) return out;
        if (nd == 1 && hipGraphNodeGetDependencies(nodes[i], &dep[i], &nd) != hipSuccess) return out;
        if (nd == 0) {
            roots++;
            root = i;
        }
    }
    if (roots != 1) return out;
    std::vector<size_t> order{root};
    while (order.size() < nn) {  // the unique node depending on the last one
        size_t next = nn, cnt = 0;
        for (size_t i = 0; i < nn; i++)
            if (dep[i] == nodes[order.back()]) {
                next = i;
                cnt++;
            }
        if (cnt != 1) return out;
        order.push_back(next);
    }
    for (size_t i : order) {
        hipKernelNodeParams p{};
        if (hipGraphKernelNodeGetParams(nodes[i], &p) != hipSuccess || p.extra || !p.kernelParams || !p.func) {
            out.clear();
            return out;
        }
        out.push_back(p);
    }
    return out;
}

// The plan's fused launches with an in-grid pre-pass: arguments copied into the plan (the direct
// chain's entry repointed at them; graph replays set them on the executable graph).
static vxg_status bind_fused_nodes(vxg_plan* pl, hipGraph_t g) {
    size_t nn = 0;
    if (hipGraphGetNodes(g, nullptr, &nn) != hipSuccess) return set_error(VXG_ERR_ASSERTION_FAILED, "graph nodes");
    std::vector<hipGraphNode_t> nodes(nn);
    if (nn && hipGraphGetNodes(g, nodes.data(), &nn) != hipSuccess) return set_error(VXG_ERR_ASSERTION_FAILED, "graph nodes");
    for (hipGraphNode_t nd : nodes) {
        hipGraphNodeType t{};
        if (hipGraphNodeGetType(nd, &t) != hipSuccess || t != hipGraphNodeTypeKernel) continue;
        hipKernelNodeParams p{};
        if (hipGraphKernelNodeGetParams(nd, &p) != hipSuccess || !p.kernelParams || !is_fsst_fused_kernel(p.func)) continue;
        if (static_cast<const FsstFusedArgs*>(p.kernelParams[0])->prepass == 0) continue;
        auto f = std::make_unique<FusedNode>(p.kernelParams);
        f->node = nd;
        f->p = p;
        f->p.kernelParams = f->args;
        for (hipKernelNodeParams& d : pl->direct)
            if (d.func == p.func) d.kernelParams = f->args;  // (one fused launch per plan)
        pl->fused.push_back(std::move(f));
    }
    return VXG_OK;
}

// Record one candidate plan: arrays with batched[i] defer their deferrable launches into one
// PlanBatch flushed at the end; `branches` parallel graph branches (arrays spread longest-first).
static vxg_status record_plan(vxg_ctx* ctx, const vxg_array* arrays, vxg_canonical* outs, uint32_t n,
                              const std::vector<bool>& batched, uint32_t branches, vxg_plan** plan) {
    *plan = nullptr;
    const bool batching = std::find(batched.begin(), batched.end(), true) != batched.end();
    // Record on an origin stream forked into `branches` streams: the arrays are independent, so
    // their launches become parallel graph branches (the graph runs them on several hardware
    // queues, overlapping the ramp and drain of the many small kernels of a chunked scan), joined
    // back into the origin stream.  The batched arrays' deferrable launches (K1 decodes, RunEnd
    // expansions, dictionary views of chunked columns) go to one more branch -- or, with one
    // branch, follow the arrays on it (a single-stream graph) -- recorded after every array.
    const bool own = batching && branches > 1;
    const uint32_t nb = (n < branches ? (n ? n : 1) : branches) + (own ? 1 : 0);
    const uint32_t na = own ? nb - 1 : nb;  // branches the arrays are spread over
    PlanBatch batch;
    hipStream_t cs;
    VXG_TRY(hip_check(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking), "plan stream"));
    std::vector<hipStream_t> br(nb, nullptr);
    std::vector<hipEvent_t> ev(nb + 1, nullptr);
    vxg_status st = VXG_OK;
    for (uint32_t b = 0; b < nb && st == VXG_OK; b++)
        st = hip_check(hipStreamCreateWithFlags(&br[b], hipStreamNonBlocking), "plan branch stream");
    for (uint32_t b = 0; b <= nb && st == VXG_OK; b++)
        st = hip_check(hipEventCreateWithFlags(&ev[b], hipEventDisableTiming), "plan event");
    auto* pl = new vxg_plan();
    pl->ctx = ctx;
    pl->batched = batching;
    pl->branches = na;
    if (st == VXG_OK) st = hip_check(hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
    if (st == VXG_OK) {
        st = hip_check(hipEventRecord(ev[nb], cs), "fork");
        for (uint32_t b = 0; b < nb && st == VXG_OK; b++)
            st = hip_check(hipStreamWaitEvent(br[b], ev[nb], 0), "fork wait");
        // longest-processing-time-first: arrays in decreasing order of the bytes their decode
        // moves, each onto the branch with the least work so far, so one heavy column (C5's
        // l_comment) does not queue behind others on its branch
        std::vector<uint32_t> order(n);
        std::vector<uint64_t> cost(n), load(na, 0);
        for (uint32_t i = 0; i < n; i++) {
            order[i] = i;
            cost[i] = plan_cost(arrays[i]);
        }
        std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return cost[x] > cost[y]; });
        for (uint32_t k = 0; k < n && st == VXG_OK; k++) {
            const uint32_t i = order[k];
            const uint32_t b = uint32_t(std::min_element(load.begin(), load.end()) - load.begin());
            if (!(own && batched[i])) load[b] += cost[i];  // (a batched array's launches run on the batch branch)
            Planner p(ctx, br[b], &pl->store, batched[i] ? &batch : nullptr);
            st = p.canonical(arrays[i], outs[i]);
        }
        // A batch on its own branch waits for every array branch first: deferred
        // launches read what those branches wrote -- a chunked FSST column's per-chunk validity
        // bitmaps, a Dict chunk's decoded values -- and nothing else orders the two streams.
        for (uint32_t b = 0; own && b < na && st == VXG_OK; b++) {
            st = hip_check(hipEventRecord(ev[b], br[b]), "batch join");
            if (st == VXG_OK) st = hip_check(hipStreamWaitEvent(br[nb - 1], ev[b], 0), "batch join wait");
        }
        if (batching && st == VXG_OK) st = flush_plan_batch(batch, ctx->c.err_word, br[nb - 1], &pl->store);
        for (uint32_t b = 0; b < nb && st == VXG_OK; b++) {
            st = hip_check(hipEventRecord(ev[b], br[b]), "join");
            if (st == VXG_OK) st = hip_check(hipStreamWaitEvent(cs, ev[b], 0), "join wait");
        }
        hipGraph_t g = nullptr;
        const hipError_t e = hipStreamEndCapture(cs, &g);
        if (st == VXG_OK) st = hip_check(e, "hipStreamEndCapture");
        pl->graph = g;
        if (st == VXG_OK && std::getenv("VXG_PLAN_DOT")) {  // diagnostics: PREFIX_<n>.dot per recorded graph
            static int cnt = 0;
            const std::string path = std::string(std::getenv("VXG_PLAN_DOT")) + "_" + std::to_string(cnt++) + ".dot";
            (void)hipGraphDebugDotPrint(g, path.c_str(), 0);
        }
        if (st == VXG_OK)
            st = hip_check(hipGraphInstantiate(&pl->exec, g, nullptr, nullptr, 0), "hipGraphInstantiate");
        if (st == VXG_OK) st = pl->store.upload();  // device chunk tables, once for all replays
        if (st == VXG_OK && plan_direct_enabled()) pl->direct = kernel_chain(g);
        if (st == VXG_OK) st = bind_fused_nodes(pl, g);
    }
    for (hipEvent_t e : ev)
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t b : br)
        if (b) (void)hipStreamDestroy(b);
    (void)hipStreamDestroy(cs);
    if (st == VXG_OK) *plan = pl;
    else vxg_plan_destroy(pl);
    return st;
}

// Median device time of `reps` interleaved replays of each candidate (after one warm-up each).
static vxg_status time_plans(const std::vector<vxg_plan*>& cands, int reps, std::vector<float>* ms) {
    hipStream_t s;
    VXG_TRY(hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "plan timing stream"));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    vxg_status st = hip_check(hipEventCreate(&e0), "plan timing event");
    if (st == VXG_OK) st = hip_check(hipEventCreate(&e1), "plan timing event");
    std::vector<std::vector<float>> t(cands.size());
    for (vxg_plan* p : cands)
        if (st == VXG_OK) st = vxg_plan_launch(p, s);
    for (int r = 0; r < reps && st == VXG_OK; r++) {
        for (size_t c = 0; c < cands.size() && st == VXG_OK; c++) {
            st = hip_check(hipEventRecord(e0, s), "plan timing");
            if (st == VXG_OK) st = vxg_plan_launch(cands[c], s);
            if (st == VXG_OK) st = hip_check(hipEventRecord(e1, s), "plan timing");
            if (st == VXG_OK) st = hip_check(hipEventSynchronize(e1), "plan timing");
            float x = 0;
            if (st == VXG_OK) st = hip_check(hipEventElapsedTime(&x, e0, e1), "plan timing");
            t[c].push_back(x);
        }
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    ms->clear();
    for (auto& v : t) {
        std::sort(v.begin(), v.end());
        ms->push_back(v.empty() ? 0.f : v[v.size() / 2]);
    }
    return st;
}

// Graph nodes + dependency edges: what a replay pays beyond its kernels (each cross-branch edge
// is a queue synchronisation; a direct chain replays with no graph at all).
static uint32_t graph_cost(hipGraph_t g) {
    size_t nn = 0, ne = 0;
    if (!g || hipGraphGetNodes(g, nullptr, &nn) != hipSuccess) return 0;
    if (hipGraphGetEdges(g, nullptr, nullptr, &ne) != hipSuccess) ne = 0;
    return uint32_t(nn + ne);
}

extern "C" {

uint32_t vxg_plan_select(const float* ms, const uint32_t* cost, uint32_t n, uint32_t* selection) {
    uint32_t sel = VXG_PLAN_SEL_SINGLE, best = 0;
    if (n > 1 && !ms) {  // unmeasured: the smallest graph
        sel = VXG_PLAN_SEL_UNMEASURED;
        for (uint32_t c = 1; c < n; c++)
            if (cost && cost[c] < cost[best]) best = c;
    } else if (n > 1) {
        uint32_t fastest = 0;
        for (uint32_t c = 1; c < n; c++)
            if (ms[c] < ms[fastest]) fastest = c;
        best = fastest;
        sel = VXG_PLAN_SEL_FASTER;
        // candidates within 3 % of the fastest are equal: the smallest graph among them, the
        // lowest index on equal cost
        for (uint32_t c = 0; c < n; c++) {
            if (c == fastest || !(ms[c] <= ms[fastest] * 1.03f)) continue;
            sel = VXG_PLAN_SEL_TIE_COST;
            if (!cost) continue;
            if (cost[c] < cost[best] || (cost[c] == cost[best] && c < best)) best = c;
        }
    }
    if (selection) *selection = sel;
    return best;
}

vxg_status vxg_plan_create(vxg_ctx* ctx, const vxg_array* arrays, vxg_canonical* outs, uint32_t n, vxg_plan** plan) {
    return vxg_plan_create_ex(ctx, arrays, outs, n, 0, plan);
}

vxg_status vxg_plan_create_ex(vxg_ctx* ctx, const vxg_array* arrays, vxg_canonical* outs, uint32_t n,
                              uint32_t flags, vxg_plan** plan) {
    const auto t0 = std::chrono::steady_clock::now();
    VXG_TRY(use_device(ctx));
    if (!plan || (n && (!arrays || !outs))) return set_error(VXG_ERR_INVALID_ARGUMENT, "null plan/arrays/outs");
    if (flags & ~uint32_t(VXG_PLAN_MEASURE)) return set_error(VXG_ERR_INVALID_ARGUMENT, "unknown plan flags");
    *plan = nullptr;
    for (uint32_t i = 0; i < n; i++) {  // nothing may allocate or synchronise while recording
        const vxg_array& a = arrays[i];
        const vxg_canonical& o = outs[i];
        const bool str = a.dtype == VXG_DTYPE_UTF8 || a.dtype == VXG_DTYPE_BINARY;
        if (str ? (!o.views || !o.data) : !o.values)
            return set_error(VXG_ERR_INVALID_ARGUMENT, "a plan needs caller-allocated outputs");
        if (a.nullable && !o.validity)
            return set_error(VXG_ERR_INVALID_ARGUMENT, "a plan needs caller-allocated validity for nullable arrays");
    }
    // candidates: (batched mask, branches); 2 branches unbatched (C5 at 1 GPU 322.6 us/replay vs
    // 362 with 1 and 348 with 3), 1 batched (each cross-branch edge costs a replay several
    // microseconds of queue synchronisation: C5 shard 82 -> 68 us)
    const uint32_t env_br = plan_branches_env();
    const std::vector<bool> none(n, false), all(n, true);
    std::vector<bool> mixed(n);
    for (uint32_t i = 0; i < n; i++) mixed[i] = canonical_out_bytes(arrays[i]) <= plan_batch_max_bytes();
    std::vector<std::pair<std::vector<bool>, uint32_t>> cand;
    const bool measure = (flags & VXG_PLAN_MEASURE) != 0;
    switch (plan_batch_mode()) {
    case BatchMode::Off: cand.emplace_back(none, env_br ? env_br : 2u); break;
    case BatchMode::On: cand.emplace_back(all, env_br ? env_br : 1u); break;
    case BatchMode::Mixed: cand.emplace_back(mixed, env_br ? env_br : 2u); break;
    case BatchMode::Strings: {
        std::vector<bool> strs(n);
        for (uint32_t i = 0; i < n; i++) strs[i] = dict_string_column(arrays[i]);
        cand.emplace_back(strs, env_br ? env_br : 2u);
        break;
    }
    case BatchMode::Auto:
        if (measure) {
            cand.emplace_back(none, env_br ? env_br : 2u);
            if (n) cand.emplace_back(all, env_br ? env_br : 1u);
        } else {
            cand.emplace_back(all, env_br ? env_br : 1u);
        }
        break;
    }
    std::vector<vxg_plan*> plans;
    vxg_status st = VXG_OK;
    for (const auto& [mask, branches] : cand) {
        vxg_plan* p = nullptr;
        st = record_plan(ctx, arrays, outs, n, mask, branches, &p);
        if (st != VXG_OK) break;
        plans.push_back(p);
    }
    size_t best = 0;
    uint32_t selection = VXG_PLAN_SEL_SINGLE;
    std::vector<float> ms(plans.size(), 0.f);
    std::vector<uint32_t> cost(plans.size(), 0);
    for (size_t c = 0; c < plans.size(); c++) cost[c] = graph_cost(plans[c]->graph);
    if (st == VXG_OK && measure && plans.size() > 1) {
        // the candidates read the inputs now: every upload the caller enqueued (any stream) first
        st = hip_check(hipDeviceSynchronize(), "plan create: device synchronize");
        uint32_t pending = 0;  // an error of the caller's earlier work: theirs to sync, not ours
        if (st == VXG_OK)
            st = hip_check(hipMemcpy(&pending, ctx->c.err_word, 4, hipMemcpyDeviceToHost), "error word readback");
        if (st == VXG_OK && pending) {
            best = vxg_plan_select(nullptr, cost.data(), uint32_t(plans.size()), &selection);
        } else if (st == VXG_OK) {
            st = time_plans(plans, 3, &ms);
            if (st == VXG_OK) best = vxg_plan_select(ms.data(), cost.data(), uint32_t(plans.size()), &selection);
            if (st == VXG_OK) {  // errors the measured runs found belong to create, not the next sync
                uint32_t err = 0;
                st = hip_check(hipMemcpy(&err, ctx->c.err_word, 4, hipMemcpyDeviceToHost), "error word readback");
                if (st == VXG_OK && err) {
                    st = hip_check(hipMemset(ctx->c.err_word, 0, 4), "error word reset");
                    if (st == VXG_OK) st = status_of_err_word(err);
                }
            }
        }
        if (std::getenv("VXG_PLAN_DEBUG"))
            for (size_t c = 0; c < ms.size(); c++)
                std::fprintf(stderr, "plan candidate %zu (%s, %u branches, %zu kernel-chain nodes): %.4f ms%s\n", c,
                             plans[c]->batched ? "batched" : "unbatched", cand[c].second, plans[c]->direct.size(),
                             ms[c], c == best ? "  <- kept" : "");
    }
    if (st == VXG_OK && !plans.empty()) {
        vxg_plan_info& in = plans[best]->info;
        in.batched = plans[best]->batched;
        in.branches = plans[best]->branches;
        in.direct_nodes = uint32_t(plans[best]->direct.size());
        in.n_candidates = uint32_t(std::min<size_t>(plans.size(), 2));
        for (size_t c = 0; c < plans.size() && c < 2; c++) {
            in.candidate_batched[c] = plans[c]->batched;
            in.candidate_ms[c] = ms[c];
        }
        in.selection = selection;
        for (size_t c = 0; c < plans.size() && c < 2; c++) in.candidate_cost[c] = cost[c];
        in.create_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    for (size_t c = 0; c < plans.size(); c++)
        if (st != VXG_OK || c != best) vxg_plan_destroy(plans[c]);
    if (st == VXG_OK && !plans.empty()) *plan = plans[best];
    return st;
}

vxg_status vxg_plan_get_info(const vxg_plan* plan, vxg_plan_info* info) {
    if (!plan || !info) return set_error(VXG_ERR_INVALID_ARGUMENT, "null plan/info");
    *info = plan->info;
    return VXG_OK;
}

vxg_status vxg_plan_launch(vxg_plan* plan, void* stream) {
    if (!plan || !plan->exec) return set_error(VXG_ERR_INVALID_ARGUMENT, "null plan");
    VXG_TRY(use_device(plan->ctx));
    // a new record tag per launch for the in-grid pre-pass (the previous launch's records carry
    // the previous tag)
    const uint32_t tag = uint32_t(++plan->launches % 65535u) + 1u;
    for (auto& f : plan->fused) f->fa.tag = tag;
    if (!plan->direct.empty()) {
        for (const hipKernelNodeParams& p : plan->direct)
            VXG_TRY(hip_check(hipLaunchKernel(p.func, p.gridDim, p.blockDim, p.kernelParams, p.sharedMemBytes, S(stream)),
                              "plan kernel"));
        return VXG_OK;
    }
    for (auto& f : plan->fused)
        VXG_TRY(hip_check(hipGraphExecKernelNodeSetParams(plan->exec, f->node, &f->p), "plan fused launch tag"));
    return hip_check(hipGraphLaunch(plan->exec, S(stream)), "hipGraphLaunch");
}

vxg_status vxg_plan_destroy(vxg_plan* plan) {
    if (!plan) return VXG_OK;
    if (plan->ctx) (void)hipSetDevice(plan->ctx->c.device);
    if (plan->exec) (void)hipGraphExecDestroy(plan->exec);
    if (plan->graph) (void)hipGraphDestroy(plan->graph);
    if (!plan->store.allocs.empty()) (void)hipDeviceSynchronize();  // no replay may still use them
    for (void* p : plan->store.allocs) (void)hipFree(p);
    delete plan;
    return VXG_OK;
}

static int unsigned_T(int ptype) { return 8 * ptype_width(ptype); }

vxg_status vxg_bitunpack(vxg_ctx* ctx, int ptype, unsigned bit_width, unsigned offset, uint64_t len,
                         const void* packed, uint64_t packed_bytes, void* out, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_int(ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "BitPacked needs an integer ptype");
    return bitunpack_common(ctx, unsigned_T(ptype), bit_width, offset, len, packed, packed_bytes, Epi::Plain, 0,
                            UnpackArgs{}, out, stream);
}

vxg_status vxg_bitunpack_for(vxg_ctx* ctx, int ptype, unsigned bit_width, unsigned offset, uint64_t len,
                             const void* packed, uint64_t packed_bytes, uint64_t reference, unsigned shift,
                             int zigzag, void* out, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_int(ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "FoR needs an integer ptype");
    UnpackArgs a{};
    a.reference = reference;
    a.shift = shift;
    return bitunpack_common(ctx, unsigned_T(ptype), bit_width, offset, len, packed, packed_bytes,
                            zigzag ? Epi::ForZigZag : Epi::For, 0, a, out, stream);
}

vxg_status vxg_bitunpack_alp(vxg_ctx* ctx, int float_ptype, unsigned bit_width, unsigned offset, uint64_t len,
                             const void* packed, uint64_t packed_bytes, uint64_t for_reference,
                             unsigned for_shift, unsigned e, unsigned f, void* out, void* stream) {
    VXG_TRY(use_device(ctx));
    const bool f32 = float_ptype == VXG_F32;
    if (!f32 && float_ptype != VXG_F64) return set_error(VXG_ERR_MISMATCHED_TYPES, "ALP decodes to f32/f64");
    if ((f32 && (e > 10 || f > 10)) || (!f32 && (e > 23 || f > 23)))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "ALP exponents out of range");
    UnpackArgs a{};
    a.reference = for_reference;
    a.shift = for_shift;
    a.alp_a = f32 ? double(kF10f[f]) : kF10d[f];
    a.alp_b = f32 ? double(kIF10f[e]) : kIF10d[e];
    return bitunpack_common(ctx, f32 ? 32 : 64, bit_width, offset, len, packed, packed_bytes,
                            f32 ? Epi::AlpF32 : Epi::AlpF64, 0, a, out, stream);
}

vxg_status vxg_bitunpack_dict(vxg_ctx* ctx, int codes_ptype, unsigned bit_width, unsigned offset, uint64_t len,
                              const void* packed, uint64_t packed_bytes, const void* dict_values,
                              uint64_t dict_len, unsigned value_width, void* out, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_unsigned(codes_ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "Dict codes must be unsigned");
    if (bit_width > unsigned(kDictFusedMaxW))
        return set_error(VXG_ERR_NOT_IMPLEMENTED, "fused dict decode supports code widths <= 16");
    UnpackArgs a{};
    a.dict = dict_values;
    a.dict_len = dict_len;
    return bitunpack_common(ctx, unsigned_T(codes_ptype), bit_width, offset, len, packed, packed_bytes, Epi::Dict,
                            int(value_width), a, out, stream);
}

vxg_status vxg_bitunpack_dict_chunks(vxg_ctx* ctx, int codes_ptype, unsigned bit_width, unsigned value_width,
                                     const vxg_dict_chunk* chunks_host, uint32_t n_chunks, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_unsigned(codes_ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "Dict codes must be unsigned");
    if (bit_width > unsigned(kDictFusedMaxW))
        return set_error(VXG_ERR_NOT_IMPLEMENTED, "fused dict decode supports code widths <= 16");
    std::vector<K1Job> jobs(n_chunks);
    for (uint32_t i = 0; i < n_chunks; i++) {
        const vxg_dict_chunk& c = chunks_host[i];
        if (c.n_blocks != (c.len + 1023) / 1024)
            return set_error(VXG_ERR_INVALID_ARGUMENT, "chunk n_blocks != ceil(len/1024)");
        UnpackArgs a{};
        a.dict = c.dict_values;
        a.dict_len = c.dict_len;
        VXG_TRY(make_k1_job(unsigned_T(codes_ptype), bit_width, 0, c.len, c.packed, c.n_blocks * 128ull * bit_width,
                            Epi::Dict, int(value_width), a, c.out, jobs[i]));
    }
    return launch_k1_jobs(jobs, ctx->c.err_word, S(stream));
}

vxg_status vxg_patch(vxg_ctx* ctx, int ptype, void* out, uint64_t out_len, int indices_ptype, const void* indices,
                     uint64_t indices_offset, const void* values, uint64_t n_patches, void* stream) {
    VXG_TRY(use_device(ctx));
    const int w = ptype_width(ptype);
    if (!w || !ptype_is_int(indices_ptype)) return set_error(VXG_ERR_INVALID_ARGUMENT, "bad ptype");
    UnpackArgs a{};
    a.err = ctx->c.err_word;
    IntCol ic{};
    ic.p = indices;
    ic.width = ptype_width(indices_ptype);
    ic.sgn = ptype_is_signed(indices_ptype);
    return launch_patch(0, ic, Epi::Plain, 8 * w, out, out_len, indices_offset, values, n_patches, a, S(stream));
}

vxg_status vxg_for_decode(vxg_ctx* ctx, int ptype, const void* in, uint64_t n, uint64_t reference,
                          unsigned shift, void* out, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_int(ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "FoR needs an integer ptype");
    return launch_for(ptype_width(ptype), in, n, reference, shift, false, out, S(stream));
}

vxg_status vxg_zigzag_decode(vxg_ctx* ctx, int out_ptype, const void* in, uint64_t n, void* out, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_signed(out_ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "ZigZag decodes to signed ints");
    return launch_zigzag(ptype_width(out_ptype), in, n, out, S(stream));
}

vxg_status vxg_alp_decode(vxg_ctx* ctx, int float_ptype, const void* encoded, uint64_t n, unsigned e, unsigned f,
                          void* out, void* stream) {
    VXG_TRY(use_device(ctx));
    const bool f32 = float_ptype == VXG_F32;
    if ((f32 && (e > 10 || f > 10)) || (!f32 && (e > 23 || f > 23)))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "ALP exponents out of range");
    return launch_alp(float_ptype, encoded, n, f32 ? double(kF10f[f]) : kF10d[f],
                      f32 ? double(kIF10f[e]) : kIF10d[e], out, S(stream));
}

vxg_status vxg_alprd_decode(vxg_ctx* ctx, int float_ptype, const uint16_t* left_codes, const uint16_t* dict_host,
                            unsigned dict_len, unsigned right_bw, const void* right, uint64_t n,
                            const uint64_t* exc_pos, const uint16_t* exc_vals, uint64_t n_exc, void* out,
                            void* stream) {
    VXG_TRY(use_device(ctx));
    if (dict_len > 8) return set_error(VXG_ERR_INVALID_ARGUMENT, "ALP-RD dictionary holds at most 8 entries");
    return launch_alprd(float_ptype, left_codes, dict_host, dict_len, right_bw, right, n, exc_pos, 8, false, 0,
                        exc_vals, n_exc, out, ctx->c.err_word, S(stream));
}

vxg_status vxg_take(vxg_ctx* ctx, unsigned value_width, const void* values, uint64_t n_values, int codes_ptype,
                    const void* codes, uint64_t n, void* out, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_unsigned(codes_ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "take indices must be unsigned");
    return launch_take(int(value_width), values, n_values, ptype_width(codes_ptype), ptype_is_signed(codes_ptype), codes, n, out,
                       ctx->c.err_word, S(stream));
}

vxg_status vxg_delta_decode(vxg_ctx* ctx, int ptype, const void* bases, uint64_t n_bases, const void* deltas,
                            uint64_t n_deltas, uint64_t offset, uint64_t len, void* out, void* stream) {
    VXG_TRY(use_device(ctx));
    const int w = ptype_width(ptype);
    if (!ptype_is_unsigned(ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "Delta decodes unsigned ints");
    const uint64_t lanes = 1024 / (8 * w);
    if (n_bases != (n_deltas / 1024) * lanes + (n_deltas % 1024 ? 1 : 0))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "DeltaArray: bases.len() != expected_bases_len");
    if (offset + len > n_deltas) return set_error(VXG_ERR_INVALID_ARGUMENT, "offset + len > deltas len");
    return launch_delta(w, bases, deltas, n_deltas, offset, len, out, S(stream));
}

vxg_status vxg_runend_decode(vxg_ctx* ctx, unsigned value_width, const void* values, int ends_ptype,
                             const void* ends, uint64_t n_runs, uint64_t offset, uint64_t len, void* out,
                             void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_int(ends_ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "RunEnd ends must be integers");
    RunEndChunk c{};
    c.ends.p = ends;
    c.ends.width = ptype_width(ends_ptype);
    c.ends.sgn = ptype_is_signed(ends_ptype);
    c.values.p = values;
    c.values.width = int(value_width);
    c.out = out;
    c.n_runs = n_runs;
    c.offset = offset;
    c.len = len;
    return launch_runend(int(value_width), c, ctx->c.err_word, S(stream));
}

vxg_status vxg_take_array(vxg_ctx* ctx, const vxg_array* a, int indices_ptype, const void* indices,
                          uint64_t n_indices, vxg_canonical* out, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!a || !out || (n_indices && !indices)) return set_error(VXG_ERR_INVALID_ARGUMENT, "null array/indices/out");
    if (!ptype_is_int(indices_ptype)) return set_error(VXG_ERR_INVALID_ARGUMENT, "take indices must be integers");
    Planner p(ctx, S(stream));
    return p.take(*a, indices, ptype_width(indices_ptype), ptype_is_signed(indices_ptype), n_indices, *out);
}

// ---- encoders on the GPU (encode_gpu.hip, fl_pack_impl.hpp) ----------------------------
vxg_status vxg_compute_int_stats(vxg_ctx* ctx, int ptype, const void* values, uint64_t n, vxg_int_stats* out,
                                 void* stream) {
    VXG_TRY(use_device(ctx));
    if (!out || (n && !values)) return set_error(VXG_ERR_INVALID_ARGUMENT, "null values/out");
    if (!ptype_is_int(ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "integer statistics need an integer ptype");
    IntStats st{};
    VXG_TRY(launch_int_stats(ptype_width(ptype), ptype_is_signed(ptype), values, n, &st, S(stream)));
    std::memset(out, 0, sizeof(*out));
    out->n = st.n;
    out->min_bits = st.min_bits;
    out->max_bits = st.max_bits;
    out->trailing_zeros = st.trailing_zeros;
    std::memcpy(out->bit_width_freq, st.bit_width_freq, sizeof(out->bit_width_freq));
    return VXG_OK;
}

static vxg_status pack_common(vxg_ctx* ctx, int ptype, bool for_, uint64_t reference, unsigned shift,
                              unsigned bit_width, const void* values, uint64_t n, void* packed, uint64_t packed_bytes,
                              void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_int(ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "bitpack needs an integer ptype");
    const int T = 8 * ptype_width(ptype);
    if (bit_width >= unsigned(T))  // bitpack_encode (bitpacking/compress.rs:22-30)
        return set_error(VXG_ERR_INVALID_ARGUMENT,
                         "Cannot pack -- specified bit width is greater than or equal to raw bit width");
    const uint64_t want = ((n + 1023) / 1024) * 128ull * bit_width;
    if (packed_bytes != want)
        return set_error(VXG_ERR_INVALID_ARGUMENT, "packed buffer must hold " + std::to_string(want) + " bytes");
    if (bit_width == 0 || n == 0) return VXG_OK;  // bit width 0: an empty buffer (compress.rs:86-88)
    if (!values || !packed) return set_error(VXG_ERR_INVALID_ARGUMENT, "null values/packed");
    if (reinterpret_cast<uintptr_t>(packed) & 15) return set_error(VXG_ERR_INVALID_ARGUMENT, "packed must be 16-byte aligned");
    if (reinterpret_cast<uintptr_t>(values) % uint64_t(ptype_width(ptype)))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "values must be aligned to the value width");
    const bool sgn = ptype_is_signed(ptype);
    switch (T) {
    case 8: return fl_pack_8(int(bit_width), for_, reference, shift, sgn, values, n, packed, S(stream));
    case 16: return fl_pack_16(int(bit_width), for_, reference, shift, sgn, values, n, packed, S(stream));
    case 32: return fl_pack_32(int(bit_width), for_, reference, shift, sgn, values, n, packed, S(stream));
    default: return fl_pack_64(int(bit_width), for_, reference, shift, sgn, values, n, packed, S(stream));
    }
}

vxg_status vxg_bitpack(vxg_ctx* ctx, int ptype, unsigned bit_width, const void* values, uint64_t n, void* packed,
                       uint64_t packed_bytes, void* stream) {
    return pack_common(ctx, ptype, false, 0, 0, bit_width, values, n, packed, packed_bytes, stream);
}

vxg_status vxg_for_bitpack(vxg_ctx* ctx, int ptype, uint64_t reference, unsigned shift, unsigned bit_width,
                           const void* values, uint64_t n, void* packed, uint64_t packed_bytes, void* stream) {
    if (shift >= unsigned(8 * ptype_width(ptype))) return set_error(VXG_ERR_INVALID_ARGUMENT, "FoR shift out of range");
    return pack_common(ctx, ptype, true, reference, shift, bit_width, values, n, packed, packed_bytes, stream);
}

vxg_status vxg_for_encode(vxg_ctx* ctx, int ptype, const void* values, uint64_t n, uint64_t reference, unsigned shift,
                          void* out, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_int(ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "FoR needs an integer ptype");
    if (shift >= unsigned(8 * ptype_width(ptype))) return set_error(VXG_ERR_INVALID_ARGUMENT, "FoR shift out of range");
    if (n && (!values || !out)) return set_error(VXG_ERR_INVALID_ARGUMENT, "null values/out");
    if (n == 0) return VXG_OK;
    return launch_for_encode(ptype_width(ptype), ptype_is_signed(ptype), values, n, reference, shift, out, S(stream));
}

vxg_status vxg_gather_patches(vxg_ctx* ctx, int ptype, unsigned bit_width, const void* values, uint64_t n,
                              uint64_t* indices, void* patch_values, uint64_t cap, uint64_t* n_patches, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!n_patches || (n && !values) || (cap && (!indices || !patch_values)))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "null argument");
    if (!ptype_is_int(ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "patches need an integer ptype");
    return launch_gather_patches_gpu(ptype_width(ptype), bit_width, values, n, indices, patch_values, cap, n_patches,
                                     S(stream));
}

vxg_status vxg_alp_encode(vxg_ctx* ctx, int float_ptype, const void* values, uint64_t n, uint8_t* e, uint8_t* f,
                          void* encoded, uint64_t* patch_indices, void* patch_values, uint64_t cap,
                          uint64_t* n_patches, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!e || !f || !n_patches || (n && (!values || !encoded)) || (cap && (!patch_indices || !patch_values)))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "null argument");
    return launch_alp_encode(float_ptype, values, n, e, f, encoded, patch_indices, patch_values, cap, n_patches,
                             S(stream));
}

vxg_status vxg_fsst_compress(vxg_ctx* ctx, const uint64_t* symbols, const uint8_t* symbol_lengths, uint32_t n_symbols,
                             int offsets_ptype, const void* offsets, const uint8_t* bytes, uint64_t bytes_len,
                             const uint8_t* validity, uint64_t n, uint8_t* codes, uint64_t codes_cap,
                             int32_t* code_offsets, int32_t* uncompressed_lengths, uint64_t* codes_len, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!codes_len || !code_offsets || (n_symbols && (!symbols || !symbol_lengths)) ||
        (n && (!offsets || !uncompressed_lengths)) || (bytes_len && !bytes) || (codes_cap && !codes))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "null argument");
    if (!ptype_is_int(offsets_ptype)) return set_error(VXG_ERR_MISMATCHED_TYPES, "VarBin offsets must be integers");
    return launch_fsst_compress(symbols, symbol_lengths, n_symbols, ptype_width(offsets_ptype),
                                ptype_is_signed(offsets_ptype), offsets, bytes, bytes_len, validity, n, codes, codes_cap,
                                code_offsets, uncompressed_lengths, codes_len, S(stream));
}

vxg_status vxg_filter_array(vxg_ctx* ctx, const vxg_array* a, const vxg_array* predicate, vxg_canonical* out,
                            void* stream) {
    VXG_TRY(use_device(ctx));
    if (!a || !predicate || !out) return set_error(VXG_ERR_INVALID_ARGUMENT, "null array/predicate/out");
    vxg_status st;
    {
        Planner p(ctx, S(stream));
        st = p.filter(*a, *predicate, *out);
    }
    if (st != VXG_OK) return st;
    // synchronous like the reference's compute::filter: every output is complete on return
    return hip_check(hipStreamSynchronize(S(stream)), "filter sync");
}

vxg_status vxg_runend_bool_decode(vxg_ctx* ctx, int ends_ptype, const void* ends, uint64_t n_runs, uint64_t offset,
                                  int start, uint64_t len, void* out_bits, uint64_t out_bit_offset, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_unsigned(ends_ptype))
        return set_error(VXG_ERR_INVALID_ARGUMENT, "Ends array must be an unsigned integer type");
    if (len && !out_bits) return set_error(VXG_ERR_INVALID_ARGUMENT, "null output");
    return launch_runend_bool(ends, ptype_width(ends_ptype), n_runs, offset, start != 0, len, out_bits,
                              out_bit_offset, ctx->c.err_word, S(stream));
}

vxg_status vxg_bytebool_to_bits(vxg_ctx* ctx, const uint8_t* bytes, uint64_t n, void* out_bits,
                                uint64_t out_bit_offset, void* stream) {
    VXG_TRY(use_device(ctx));
    if (n && (!bytes || !out_bits)) return set_error(VXG_ERR_INVALID_ARGUMENT, "null input/output");
    return launch_bytebool(bytes, n, out_bits, out_bit_offset, S(stream));
}

uint64_t vxg_fsst_scratch_bytes(uint64_t n) { return fsst_scratch_bytes(n); }

vxg_status vxg_fsst_decode(vxg_ctx* ctx, const uint64_t* symbols, const uint8_t* sym_lens, unsigned n_symbols,
                           const uint8_t* code_bytes, int offs_ptype, const void* code_offsets, int lens_ptype,
                           const void* lens, uint64_t n, const uint8_t* validity, void* scratch, uint8_t* heap,
                           uint8_t* views, void* stream) {
    VXG_TRY(use_device(ctx));
    if (!ptype_is_int(offs_ptype) || !ptype_is_int(lens_ptype))
        return set_error(VXG_ERR_MISMATCHED_TYPES, "FSST offsets/lengths must be integers");
    FsstChunk f{};
    f.symbols = symbols;
    f.sym_lens = sym_lens;
    f.n_symbols = n_symbols;
    f.codes = code_bytes;
    f.offs.p = code_offsets;
    f.offs.width = ptype_width(offs_ptype);
    f.offs.sgn = ptype_is_signed(offs_ptype);
    f.lens.p = lens;
    f.lens.width = ptype_width(lens_ptype);
    f.lens.sgn = ptype_is_signed(lens_ptype);
    f.n = n;
    f.validity = validity;
    f.heap = heap;
    f.views = views;
    std::vector<FsstChunk> one{f};
    return launch_fsst_batch(one, scratch, ctx->c.err_word, S(stream));
}

vxg_status vxg_fill(vxg_ctx* ctx, unsigned value_width, const void* scalar_host, uint64_t n, void* out,
                    void* stream) {
    VXG_TRY(use_device(ctx));
    uint8_t sc[16] = {0};
    if (value_width > 16) return set_error(VXG_ERR_INVALID_ARGUMENT, "value width > 16");
    std::memcpy(sc, scalar_host, value_width);
    return launch_fill(int(value_width), sc, n, out, S(stream));
}

}  // extern "C"
