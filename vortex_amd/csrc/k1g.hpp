// k1g.hpp — K1g: one launch for many K1 decodes of DIFFERENT (T, W, epilogue) kernels.
//
// A recorded plan of a sharded scan (one GPU's chunk range of every column)
// holds many small BitPacked decodes, one K1 kernel variant per column; at 1/8 of TPC-H SF1 each
// is a 2-6 MB launch whose ramp/drain and graph edge cost more than its data.  K1g decodes every
// job of such a plan in ONE launch: the job's (T, W, epilogue, value width) travel in its table
// entry, the workgroup stages its blocks' packed words in LDS and each thread extracts output
// values with runtime shifts (fastlanes unpack_single addressing, bitpacking/compress.rs:
// 295-306), then applies the same epilogues as K1 (fl_unpack_impl.hpp).
#pragma once

#include "vxg_internal.hpp"

namespace vxg {

struct GenChunk {
    ChunkDev d;        // first_group = first workgroup of this job in the launch
    uint32_t kind;     // body index (gen_kind)
    uint32_t W;        // bit width
    uint32_t bpw;      // FastLanes blocks per workgroup
    uint32_t vb_offs_width;
    // Dict over a VarBin string dictionary (<= 1024 entries): every workgroup builds the
    // dictionary's 16-byte views in LDS (the K10 views launch disappears) and copies its share of
    // the dictionary bytes into the chunk's output data buffer (varbin_chunks_kernel's work)
    const uint8_t* vb_src;   // dictionary bytes
    const void* vb_offs;     // dictionary offsets (dict_len + 1)
    uint8_t* vb_dst;         // the chunk's output data buffer
    uint64_t vb_bytes;       // bytes to copy
    uint32_t vb_bidx;        // buffer_index of non-inlined views
    uint32_t pad;
    // RunEnd kinds: a short-run chunk (runend_runs.hpp) whose ends/values are read in place
    // (re.first_group unused: d.first_group is the job's first workgroup)
    RunEndChunk re;
};

// Body index of a (T, W, epilogue, value width) job, or -1 when K1g has no body for it
// (varbin_dict: Dict over a VarBin dictionary whose views K1g builds, value width 16).
int gen_kind(int T, int epi, int vw, bool varbin_dict = false);
// Body index of a short-run RunEnd expansion with `value_width`-byte values, or -1.
int gen_runs_kind(int value_width);
// Largest VarBin dictionary a K1g job builds in LDS.
constexpr uint64_t kGenVarBinDictMax = 1024;
// A VarBin dictionary's bytes, when at most this many and they fit the 16 KiB stage beside its
// views, are staged in LDS too: loaded in the same round trip as the offsets (a view needs both),
// instead of a second dependent round of byte loads.
constexpr uint64_t kGenVarBinHeapLds = 2048;
__host__ __device__ constexpr bool gen_vb_heap_lds(uint64_t dict_len, uint64_t bytes) {
    return bytes <= kGenVarBinHeapLds && 16 * dict_len + ((bytes + 15) & ~15ull) <= 16 * 1024;
}
// LDS of a Dict-over-VarBin job's dictionary stage: the views (+ the bytes when staged)
__host__ __device__ constexpr uint32_t gen_vb_stage_bytes(uint64_t dict_len, uint64_t bytes) {
    return uint32_t(16 * dict_len + (gen_vb_heap_lds(dict_len, bytes) ? ((bytes + 15) & ~15ull) : 0));
}
// Blocks per workgroup of a job (its packed words staged in <= 16 KiB of LDS).
uint32_t gen_bpw(int T, int W, uint32_t cap = 0);
// The blocks-per-workgroup cap of a K1g launch over `blocks` FastLanes blocks (VXG_K1G_BPW if
// set, else 8 when the launch keeps >= kGenWideMinGroups workgroups at 8, else 4)
uint32_t gen_bpw_cap(uint64_t blocks);
// ... of a Dict-over-VarBin job: 1 in a launch of such jobs alone, else gen_bpw's
// (VXG_K1G_VB_BPW overrides both).
uint32_t gen_vb_bpw(int T, int W, bool alone, uint32_t cap = 0);
// LDS a short-run RunEnd expansion of `value_width`-byte values needs.
uint32_t gen_runs_lds_bytes(int value_width);
// One launch over a device table of n jobs (first_group filled in).  `dict_lds` = every Dict
// job's dictionary fits the LDS stage (16 KiB, 16-byte aligned); packed_bytes / dict_bytes /
// runs_bytes = the largest packed stage (bpw * 128 * W), dictionary stage (staged dictionaries,
// VarBin views) and RunEnd expansion LDS of the launch's jobs.
// With `fuse` valid, the launch also decodes that FSST group's tiles (fsst.hip fsst_k1g_kernel;
// n = 0 is allowed then).
vxg_status launch_k1_generic(const GenChunk* ext, uint32_t n, uint64_t groups, bool dict_lds, uint32_t packed_bytes,
                             uint32_t dict_bytes, uint32_t runs_bytes, uint32_t* err, hipStream_t s,
                             uint64_t gpe = 0, const FsstFused* fuse = nullptr);
// The fused launch (fsst.hip): K1g jobs `ext` (n entries, `groups` workgroups, LDS `shm` with the
// dictionary stage at dict_off) beside `fuse`'s decode tiles.
vxg_status launch_fsst_k1g(const FsstFused& fuse, const GenChunk* ext, uint32_t n, uint64_t groups, uint32_t dict_off,
                           bool dict_lds, size_t shm, uint32_t* err, hipStream_t s, uint64_t gpe);

}  // namespace vxg
