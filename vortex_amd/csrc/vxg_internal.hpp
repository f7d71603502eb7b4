// vxg_internal.hpp — shared internals of the MI355X decode engine (not part of the C ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/vortex_gpu.h"

namespace vxg {

// FastLanes FL_ORDER (fastlanes 0.1.8).
__host__ __device__ constexpr int fl_order(int i) {
    constexpr int o[8] = {0, 4, 2, 6, 1, 5, 3, 7};
    return o[i];
}
// index(row, lane) = FL_ORDER[row/8]*16 + (row%8)*128 + lane
__host__ __device__ constexpr int fl_index(int row, int lane) {
    return fl_order(row / 8) * 16 + (row % 8) * 128 + lane;
}

// Address-space-qualified accesses through generic pointers.  A pointer read from memory (a
// plan's device chunk table, the FSST chunk of a tile) is generic to the compiler, which then
// emits FLAT instructions for it: those also count against the LDS wait counter (every LDS wait
// then waits for the outstanding flat loads and stores as well) and take the aperture check.
// gload / gstore: the pointer addresses global memory (chunk buffers, outputs); lds_load: LDS.
template <class T>
using gptr = __attribute__((address_space(1))) T*;
// (a 16-byte struct such as uint4 moves as a native vector: its copy constructor would bind a
// generic reference and bring the flat access back)
template <class T>
__device__ __forceinline__ T gload(const T* p) {
    if constexpr (sizeof(T) == 16 && !std::is_scalar_v<T>) {
        using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
        const u32x4 x = *(gptr<const u32x4>)p;
        T r;
        __builtin_memcpy(&r, &x, 16);
        return r;
    } else {
        return *(gptr<const T>)p;
    }
}
template <class T>
__device__ __forceinline__ void gstore(T* p, const T& v) {
    if constexpr (sizeof(T) == 16 && !std::is_scalar_v<T>) {
        using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
        u32x4 x;
        __builtin_memcpy(&x, &v, 16);
        *(gptr<u32x4>)p = x;
    } else {
        *(gptr<T>)p = v;
    }
}
template <class T>
__device__ __forceinline__ T lds_load(const T* p) {
    if constexpr (sizeof(T) == 16 && !std::is_scalar_v<T>) {
        using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
        const u32x4 x = *(__attribute__((address_space(3))) const u32x4*)p;
        T r;
        __builtin_memcpy(&r, &x, 16);
        return r;
    } else {
        return *(__attribute__((address_space(3))) const T*)p;
    }
}

// Non-temporal (streaming) store of one value to global memory: decoded outputs are written once
// and not re-read by the producing launch (uint4 via a native vector type; scalars directly).
template <typename V>
__device__ __forceinline__ void nt_store(V* p, const V& v) {
    if constexpr (sizeof(V) == 16) {
        using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
        u32x4 vv;
        __builtin_memcpy(&vv, &v, 16);
        __builtin_nontemporal_store(vv, (gptr<u32x4>)p);
    } else {
        __builtin_nontemporal_store(v, (gptr<V>)p);
    }
}

inline int ptype_width(int p) {
    switch (p) {
    case VXG_U8: case VXG_I8: return 1;
    case VXG_U16: case VXG_I16: case VXG_F16: return 2;
    case VXG_U32: case VXG_I32: case VXG_F32: return 4;
    case VXG_U64: case VXG_I64: case VXG_F64: return 8;
    default: return 0;
    }
}
inline bool ptype_is_int(int p) { return p >= VXG_U8 && p <= VXG_I64; }
inline bool ptype_is_signed(int p) { return p >= VXG_I8 && p <= VXG_I64; }
inline bool ptype_is_unsigned(int p) { return p >= VXG_U8 && p <= VXG_U64; }

// ALP exponent tables: encodings/alp/src/alp/mod.rs:255-351 (same literals => same bits).
extern const float kF10f[11];
extern const float kIF10f[11];
extern const double kF10d[24];
extern const double kIF10d[24];

// Device error word bits (set by kernels, read by vxg_check via vxg_stream_sync).
enum : uint32_t { kErrTakeOOB = 1u, kErrPatchOOB = 2u, kErrRunEnd = 4u, kErrFsst = 8u, kErrRoaring = 16u, kErrVarBin = 32u,
                  kErrPatchOrder = 64u, kErrPlanSync = 128u };

// Per-context launch options (vxg_set_option, include/vortex_gpu.h): they shape launches, never
// what a launch computes.  Defaults: the environment at vxg_open, else the values below.
struct Options {
    int64_t k1w_min_groups = 1024;  // VXG_OPT_K1W_MIN_GROUPS
    int64_t k1w_bpw = 0;            // VXG_OPT_K1W_BPW (0 = the rule)
    int64_t k1_wave = -1;           // VXG_OPT_K1_WAVE (-1 = VXG_K1_WAVE, read at every launch)
};
// What the context's launches looked like (vxg_get_launch_stats).
struct LaunchStats {
    uint64_t k1w_launches = 0, k1w_last_groups = 0;
    uint32_t k1w_last_bpw = 0, k1w_min_bpw = 0, k1w_max_bpw = 0, k1w_last_bpw_max = 0;
};

struct Ctx {
    int device = 0;
    uint32_t* err_word = nullptr;  // device
    Options opt;
    std::mutex mu;                 // guards st (launches may come from several host threads)
    LaunchStats st;
};
// The context of the entry point running on this host thread (set by every entry point that
// takes one, before it launches or records anything).
extern thread_local Ctx* g_cur_ctx;
Options default_options();  // the environment's, as vxg_open applies them
inline Options cur_options() { return g_cur_ctx ? g_cur_ctx->opt : default_options(); }
// FastLanes unpack kernel choice: 0 register-resident only, 1 by launch size, 2 K1w always.
inline int k1_wave_mode() {
    const int64_t o = cur_options().k1_wave;
    if (o >= 0) return int(o > 2 ? 2 : o);
    const char* e = std::getenv("VXG_K1_WAVE");
    if (!e) return 1;
    return e[0] == '0' ? 0 : (e[0] == 'f' ? 2 : 1);
}
void note_k1w_launch(uint32_t bpw, uint32_t bpw_max, uint64_t groups);

vxg_status set_error(vxg_status s, const std::string& msg);
vxg_status hip_check(hipError_t e, const char* what);

// ---- chunk tables beyond the kernel-argument limit --------------------------------------
// A launch's chunk table normally travels as the kernel argument (<= 4 KiB: no upload, no host
// sync).  While a vxg_plan is recorded, a launch may instead cover any number of chunks with a
// device-resident table ("ext"): its entries are built in a host mirror during recording and
// copied to the device once when the plan is finalised, so replays cost nothing extra.
struct DevTables {
    std::vector<void*> allocs;                                     // owned device memory
    std::vector<std::pair<void*, std::vector<uint8_t>>> uploads;   // (device, host mirror)
    // n zeroed entries: returns the host mirror (valid until upload()), *dev its device copy
    template <class E>
    vxg_status table(size_t n, E** host, const E** dev) {
        void* d = nullptr;
        const hipError_t e = hipMalloc(&d, n * sizeof(E) + 16);
        if (e != hipSuccess) return hip_check(e, "hipMalloc (plan chunk table)");
        allocs.push_back(d);
        uploads.emplace_back(d, std::vector<uint8_t>(n * sizeof(E), 0));
        *host = reinterpret_cast<E*>(uploads.back().second.data());
        *dev = static_cast<const E*>(d);
        return VXG_OK;
    }
    vxg_status upload() {
        for (auto& u : uploads) {
            const hipError_t e = hipMemcpy(u.first, u.second.data(), u.second.size(), hipMemcpyHostToDevice);
            if (e != hipSuccess) return hip_check(e, "plan chunk table upload");
        }
        uploads.clear();
        return VXG_OK;
    }
};

// Index of the entry of a device-resident table (sorted by its first workgroup, entry 0 first
// = 0) that covers workgroup g: every lane of the wave compares one entry per round (all loads
// in flight together) and the ballot counts give the index -- wave-uniform, no dependent chain.
// Four entries per lane per round, all four loads issued before any ballot: a table of up to 256
// entries (C5's 92-chunk columns) costs one memory round trip, not one per 64 entries.
template <class E, class Key>
__device__ __forceinline__ uint32_t ext_chunk_index(const E* __restrict__ ext, uint32_t n, uint64_t g, Key key) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t cnt = 0;
    for (uint32_t base = 0; base < n; base += 256) {
        uint64_t kv[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t i = base + 64u * uint32_t(k) + lane;
            kv[k] = uint64_t(key(ext[i < n ? i : n - 1]));  // clamped: no per-lane branch
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool le = base + 64u * uint32_t(k) + lane < n && kv[k] <= g;
            cnt += uint32_t(__popcll(__ballot(le)));
        }
    }
    return cnt ? cnt - 1 : 0;
}

// As ext_chunk_index, when the planner knows that every entry but the last spans `gpe`
// workgroups (a chunked column's equal chunks; 0 = unknown): entry g / gpe is taken directly and
// checked against its first workgroup and the next entry's -- both read in the round trip that
// also brings the entry's other fields -- so the lookup costs no dependent round trip of its own;
// any mismatch falls back to the wave-wide count.
template <class E, class Key>
__device__ __forceinline__ uint32_t ext_chunk_index_gpe(const E* __restrict__ ext, uint32_t n, uint64_t g, uint64_t gpe,
                                                        Key key) {
    if (gpe) {
        // (32-bit: grids and per-entry counts are < 2^32; readfirstlane keeps the index -- computed
        // on the vector ALU -- visibly uniform, so the entry is read with scalar loads)
        const uint32_t q = uint32_t(g) / uint32_t(gpe);
        const uint32_t ci = __builtin_amdgcn_readfirstlane(q < n - 1 ? q : n - 1);
        const uint64_t f0 = uint64_t(key(ext[ci]));
        const uint64_t f1 = ci + 1 < n ? uint64_t(key(ext[ci + 1])) : ~0ull;
        if (f0 <= g && g < f1) return ci;
    }
    return ext_chunk_index(ext, n, g, key);
}
// Host side: the common workgroup count of a table's entries (all but the last equal, the last
// not larger), else 0.  VXG_EXT_GPE=0 (read once) disables the direct lookup (A/B).
inline uint64_t common_groups(const uint64_t* counts, size_t n) {
    static const bool on = [] {
        const char* e = std::getenv("VXG_EXT_GPE");
        return !(e && e[0] == '0');
    }();
    if (!on || n == 0 || counts[0] == 0) return 0;
    for (size_t i = 1; i + 1 < n; i++)
        if (counts[i] != counts[0]) return 0;
    return counts[n - 1] <= counts[0] ? counts[0] : 0;
}

// ---- launchers implemented in the .hip translation units -----------------------------
// Epilogue kinds of the fused FastLanes unpack.
enum class Epi : int { Plain = 0, For = 1, ForZigZag = 2, AlpF32 = 3, AlpF64 = 4, Dict = 5 };

struct UnpackArgs {
    const uint8_t* packed;
    void* out;
    uint64_t n_blocks;   // FastLanes blocks covered by the launch
    uint32_t offset;     // values to skip in block 0 (<1024)
    uint64_t len;        // values to write
    uint64_t reference;  // FoR reference bits
    uint32_t shift;      // FoR shift
    double alp_a, alp_b; // F10[f], IF10[e] (f32 tables are converted exactly)
    const void* dict;    // Dict values
    uint64_t dict_len;
    uint32_t* err;
};

// One K1 "chunk": an independent BitPacked array (a whole array, or one chunk of a
// ChunkedArray decoded straight into its output slice) with its fused epilogue parameters.
struct ChunkDev {
    const uint8_t* packed;
    void* out;              // output of packed position `offset` (values [0, len))
    uint64_t n_blocks;      // FastLanes blocks covered (ceil((len + offset) / 1024))
    uint64_t len;           // values to write
    uint64_t first_group;   // first 32-block workgroup of this chunk in the launch
    uint64_t reference;     // FoR reference bits
    double alp_a, alp_b;    // ALP F10[f], IF10[e] (f32 tables converted exactly)
    const void* dict;       // Dict values
    uint64_t dict_len;
    uint32_t offset;        // values to skip in block 0 (< 1024)
    uint32_t shift;         // FoR shift
};
// Up to kArgChunks descriptors travel as the kernel argument (~2.8 KB kernarg); a recorded
// plan's launch may use a device table of any length instead (ext: device, host: its mirror,
// which the host-side launch code reads and completes before the upload).
constexpr int kArgChunks = 32;
struct ChunkTable;  // below IntCol

// T in {8,16,32,64} bits; value_width only used for Epi::Dict.  `groups` = total 32-block
// workgroups of the table (first_group filled in).
vxg_status launch_fl_unpack(int T, int W, Epi epi, int value_width, const ChunkTable& tab, uint64_t groups,
                            hipStream_t s);

// An integer column a consumer kernel (FSST, patch scatter) reads in place: a plain array of `width`-byte integers,
// or a patch-free [FoR](BitPacked) column of T = 8*width bits (T = 32/64) whose elements are
// unpacked where they are used (fastlanes unpack_single, bitpacking/compress.rs:295-306).
struct IntCol {
    const void* p;
    int width;           // bytes of the logical integer type (1, 2, 4, 8)
    bool sgn;
    bool packed;
    uint32_t W;          // packed: bit width
    uint32_t shift;      // packed: FoR shift
    uint32_t offset;     // packed: BitPacked slice offset (< 1024)
    uint64_t reference;  // packed: FoR reference (0 for a bare BitPacked column)
};
// Sparse patches written by the K1w launch of a single array (n = 0: none), after the
// workgroup's own block stores: each value is written as-is (sizeof(output element) bytes) --
// ALP's outer f32/f64 exceptions (alp/compress.rs:80-96).  Indices: 8-byte integers, plain or
// [FoR](BitPacked u64) with W > 0.
// The indices are ascending (the Patches invariant; sparse/mod.rs:132-144 resolves them in order).
struct PatchCol {
    IntCol idx;
    const void* vals;
    uint64_t n;
    uint64_t idx_off;    // SparseArray indices_offset
};

struct ChunkTable {
    ChunkDev c[kArgChunks];
    uint32_t n;
    uint32_t* err;
    const ChunkDev* ext;
    ChunkDev* host;
    PatchCol patch;      // kernel-argument tables with n == 1 only (launch_fl_unpack, K1w)
    uint32_t bpw;        // K1w: blocks per workgroup of this launch (0 = the width's maximum)
};

// Set (host side) by a kernel-argument K1w launch that was handed tab.patch, the only K1 path
// that writes patches; a caller that offered patches clears it first and runs the separate
// scatter when it stays false (no other path may silently drop them).
extern thread_local bool g_k1w_wrote_patches;

// A launch with fewer 32-block workgroups than this uses the row split (S = 4): default 1024
// (round 5: the C3 8-GPU shard's 32-chunk kernel-argument launch is exactly 512 workgroups of 32
// blocks, one per two CUs' worth of waves); VXG_SPLIT_BELOW overrides (read once).
inline uint64_t split_below_groups() {
    static const uint64_t v = [] {
        const char* e = std::getenv("VXG_SPLIT_BELOW");
        return e ? uint64_t(std::strtoull(e, nullptr, 10)) : uint64_t(1024);
    }();
    return v;
}
// Whether launch_fl_unpack takes K1w for a kernel-argument table of `groups32` 32-block workgroups.
bool k1_takes_wave(int T, int W, Epi epi, uint64_t groups32);

// Patch scatter with the same epilogue applied to the patch value.
vxg_status launch_patch(int val_width, const IntCol& indices, Epi epi, int T, void* out, uint64_t out_len,
                        uint64_t indices_offset, const void* values, uint64_t n, const UnpackArgs& ep,
                        hipStream_t s);

vxg_status launch_for(int width, const void* in, uint64_t n, uint64_t ref, unsigned shift,
                      bool zigzag, void* out, hipStream_t s);
vxg_status launch_zigzag(int width, const void* in, uint64_t n, void* out, hipStream_t s);
vxg_status launch_alp(int float_ptype, const void* enc, uint64_t n, double a, double b, void* out,
                      hipStream_t s);
vxg_status launch_take(int value_width, const void* values, uint64_t n_values, int code_width, bool code_signed,
                       const void* codes, uint64_t n, void* out, uint32_t* err, hipStream_t s);
vxg_status launch_alprd(int float_ptype, const uint16_t* left, const uint16_t* dict, unsigned dict_len,
                        unsigned right_bw, const void* right, uint64_t n, const void* exc_pos,
                        int pos_width, bool pos_signed, uint64_t pos_off, const uint16_t* exc,
                        uint64_t n_exc, void* out, uint32_t* err, hipStream_t s);
vxg_status launch_copy_bits(void* dst, uint64_t dst_off, const uint8_t* src, uint64_t src_off, uint64_t n,
                            bool set_all, hipStream_t s);
// Bool producers OR words into a zeroed LSB bit buffer at bit dst_off.
// K16 (roaring.hip): croaring Native bitmap (n bytes) -> len bits at bit `off`.
vxg_status launch_roaring_bool(const uint8_t* buf, uint64_t n, uint64_t len, void* bits, uint64_t off, uint32_t* err,
                               hipStream_t s);
vxg_status launch_runend_bool(const void* ends, int ew, uint64_t n_runs, uint64_t offset, bool start, uint64_t len,
                              void* dst, uint64_t dst_off, uint32_t* err, hipStream_t s);
vxg_status launch_bytebool(const uint8_t* src, uint64_t n, void* dst, uint64_t dst_off, hipStream_t s);
vxg_status launch_assign_bits_at(void* dst, uint64_t dst_off, const void* idx, int iw, bool isg, uint64_t ioff,
                                 uint64_t n, uint64_t len, const uint8_t* vals, hipStream_t s);
vxg_status launch_gather_bits(void* dst, const void* codes, int cw, bool csg, uint64_t n, const uint8_t* src,
                              uint64_t n_values, uint32_t* err, hipStream_t s);
vxg_status launch_set_bits_at(void* dst, const void* idx, int iw, bool isg, uint64_t off, uint64_t n,
                              uint64_t len, hipStream_t s);
vxg_status launch_sum(const void* p, int w, bool sg, uint64_t n, void* out_u64, hipStream_t s);
// K1 instantiation units (fl_inst.hip)
vxg_status fl_plain_8(int W, Epi epi, const ChunkTable& t, uint64_t g, hipStream_t s);
vxg_status fl_plain_16(int W, Epi epi, const ChunkTable& t, uint64_t g, hipStream_t s);
vxg_status fl_plain_32(int W, Epi epi, const ChunkTable& t, uint64_t g, hipStream_t s);
vxg_status fl_plain_64(int W, Epi epi, const ChunkTable& t, uint64_t g, hipStream_t s);
vxg_status fl_alp(int T, int W, Epi epi, const ChunkTable& t, uint64_t g, hipStream_t s);
// K14: Dict(codes=BitPacked) with 8/16-byte values, thread per output (dict_rows.hip)
vxg_status launch_dict_rows(int T, int W, int vw, const ChunkTable& tab, hipStream_t s);
#define VXG_DECL_DICT(VW) vxg_status fl_dict_##VW(int T, int W, const ChunkTable& t, uint64_t g, hipStream_t s);
VXG_DECL_DICT(1)
VXG_DECL_DICT(2)
VXG_DECL_DICT(4)
VXG_DECL_DICT(8)
VXG_DECL_DICT(16)
#undef VXG_DECL_DICT
constexpr int kDictFusedMaxW = 16;
vxg_status launch_delta(int width, const void* bases, const void* deltas, uint64_t n_deltas,
                        uint64_t offset, uint64_t len, void* out, hipStream_t s);
// Batched RunEnd expansion: many chunks' runs in one launch (chunk table as kernel argument).
// ends/values: plain buffers, or (short-run kernel only) patch-free [FoR](BitPacked) 32/64-bit
// columns read in place -- the runs kernel unpacks the elements it needs, so a
// RunEnd(ends=BitPacked, values=FoR(BitPacked)) chunk is ONE launch with no temporaries.
// values.width is the output width (1..16); a packed values column has width 4 or 8.
struct RunEndChunk {
    IntCol ends;
    IntCol values;
    void* out;
    uint64_t n_runs;
    uint64_t offset;
    uint64_t len;
    uint64_t first_group;  // first workgroup of this chunk in the launch
};
vxg_status launch_runend(int value_width, const RunEndChunk& chunk, uint32_t* err, hipStream_t s);
constexpr uint64_t kRunEndSpan = 4096;
constexpr int kRunEndArgChunks = 32;
struct RunEndTable {
    RunEndChunk c[kRunEndArgChunks];
    uint32_t n;
    uint32_t* err;
    const RunEndChunk* ext;  // device table of n entries (plans), or null
};
vxg_status launch_runend_chunks(int value_width, const RunEndTable& t, uint64_t groups, hipStream_t s);
// Thread-per-run form for chunks whose runs are short (first_group counts kBlock runs per group).
constexpr uint64_t kRunEndShortRun = 16;  // mean rows per run at or below which a chunk uses it
constexpr uint64_t kRunEndRunsPerGroup = 1024;  // four runs per thread of a 256-thread workgroup
vxg_status launch_runend_runs(int value_width, const RunEndTable& t, uint64_t groups, hipStream_t s);

// Batched VarBin -> views (+ copy of the bytes into the output's data buffer), e.g. the
// dictionaries of a chunked Dict(VarBin) string column.
struct VarBinChunk {
    const uint8_t* src;      // VarBin bytes
    uint8_t* dst;            // data buffer in the canonical output
    const void* offsets;
    uint8_t* views;          // 16 B per row
    uint64_t bytes;          // bytes to copy
    uint64_t n;              // rows
    uint64_t first_group;
    uint32_t offs_width;
    uint32_t bidx;
};
constexpr int kVarBinArgChunks = 48;
struct VarBinTable {
    VarBinChunk c[kVarBinArgChunks];
    uint32_t n;
    const VarBinChunk* ext;  // device table of n entries (plans), or null
    uint32_t* err;           // kErrVarBin: offsets not monotonic inside the bytes
};
vxg_status launch_varbin_chunks(const VarBinTable& t, uint64_t groups, hipStream_t s);

// dst[0, n) = src[0, n), or zeros when src is null (kernels.hip K10).
vxg_status launch_copy_bytes(void* dst, const void* src, uint64_t n, hipStream_t s);
vxg_status launch_fill(int value_width, const uint8_t* scalar16, uint64_t n, void* out,
                       hipStream_t s);
// One FSST -> VarBinView decode (a whole array or one chunk of a ChunkedArray).
struct FsstChunk {
    const uint64_t* symbols;
    const uint8_t* sym_lens;
    const uint8_t* codes;
    const uint8_t* validity;  // LSB bitmap or NULL
    uint8_t* heap;            // the chunk's data buffer
    uint8_t* views;           // 16 B per row
    IntCol offs;              // codes VarBin offsets (n + 1)
    IntCol lens;              // uncompressed lengths (n)
    uint64_t n;
    uint64_t heap_len;        // decoded bytes (sum of the lengths) if known, else 0: picks the LDS budget
    uint64_t first_tile;      // launch-local: first decode workgroup (a tile of 256 strings) /
    uint64_t first_scan;      //               first pre-pass workgroup
    uint32_t n_symbols;
    uint32_t bidx;            // buffer_index of non-inlined views
};
constexpr int kFsstArgChunks = 24;
struct FsstTable {
    FsstChunk c[kFsstArgChunks];
    uint32_t n;
    const FsstChunk* ext;  // device table of n entries (plans), or null
};
// Scratch for a set of chunks (tile prefixes + scan-block totals + tile code ends).
uint64_t fsst_scratch_bytes(uint64_t n);
uint64_t fsst_batch_scratch_bytes(const FsstChunk* chunks, size_t n_chunks);
// A batched plan's FSST group whose decode tiles run inside the plan's K1g launch
// (fsst_k1g_kernel, launch_fsst_k1g in k1g.hpp): its device table, pre-pass records and tile map.
struct FsstFusedArgs {
    const FsstChunk* ext;
    const int64_t* tp;          // tile prefixes
    const int64_t* bt;          // scan-block totals
    const int64_t* tc;          // tile code ends
    const uint32_t* wg_chunk;   // chunk of every decode tile
    uint64_t tiles;             // decode tiles
    uint64_t mix;               // first workgroups of the grid the tiles are spread over (set at launch)
    // In-grid pre-pass (round 6): the group's length pre-pass runs as the first `prepass`
    // workgroups of the fused launch (one per kFusedScanTiles tiles, chunk scan_chunk[w]) and
    // publishes tagged records (value | tag << 48) that the tiles wait for.  `tag` (1-65535,
    // never the zeroed records' 0) is set by vxg_plan_launch before every launch: a new tag per
    // launch.  prepass = 0: the separate pre-pass kernel.
    uint64_t prepass;
    uint64_t delay;             // K1g workgroups placed before the first decode tile
    const uint32_t* scan_chunk;
    uint32_t tag;
};
// The fused launch's kernel (fsst.hip): true if `func` is one of its instantiations, whose
// arguments are (FsstFusedArgs, const GenChunk*, uint32_t, uint32_t, bool, uint32_t*, uint64_t).
bool is_fsst_fused_kernel(const void* func);
struct FsstFused {
    bool valid = false;
    int oa = 0, la = 0;         // offsets / lengths accessor kinds
    FsstFusedArgs a{};
};
// Decode every chunk: grouped by accessor kinds, kFsstArgChunks per launch pair (pre-pass +
// decode; a recorded plan's group over a device table is one pair).  `scratch` >=
// fsst_batch_scratch_bytes.  With `fuse` (recording a batched plan), one group whose accessors
// the fused kernel covers gets only its pre-pass launched and is described in *fuse instead.
// The FSST decode's diagnostics mask (VXG_FSST_ABL, read once per process) into its __constant__;
// called by vxg_open.
hipError_t fsst_diag_init();
vxg_status launch_fsst_batch(std::vector<FsstChunk>& chunks, void* scratch, uint32_t* err, hipStream_t s,
                             DevTables* dt = nullptr, FsstFused* fuse = nullptr);
// Views carry `bidx` as the buffer_index of non-inlined rows.
vxg_status launch_varbin_views(const uint8_t* heap, uint64_t heap_len, int offs_width, const void* offsets, uint64_t n,
                               const uint8_t* validity, uint32_t bidx, uint8_t* views, uint32_t* err, hipStream_t s);
vxg_status launch_views_rebase(const uint8_t* src, uint64_t n, uint32_t add, uint8_t* dst, hipStream_t s);

}  // namespace vxg
