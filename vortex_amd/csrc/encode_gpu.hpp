// encode_gpu.hpp — launchers of the GPU encoders (encode_gpu.hip, pack_inst.hip); C ABI in capi.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "vxg_internal.hpp"

namespace vxg {

struct IntStats {
    uint64_t n;
    uint64_t min_bits, max_bits;  // LE bits of the ptype (signed compare for signed ptypes)
    uint32_t trailing_zeros;      // min over values (stats/mod.rs:178-189); T when all are 0
    uint64_t bit_width_freq[65];  // values of each bit width 0..T (unsigned view)
};

// Synchronous: the statistics are read back into *out.
vxg_status launch_int_stats(int width, bool sgn, const void* v, uint64_t n, IntStats* out, hipStream_t s);
// K15 (pack_inst.hip, one unit per T): FastLanes pack of n values at bit width W (1 <= W < T), with
// the FoR transform (v - ref) >> shift (arithmetic if sgn) applied first when for_.
vxg_status fl_pack_8(int W, bool for_, uint64_t ref, unsigned shift, bool sgn, const void* v, uint64_t n, void* packed,
                     hipStream_t s);
vxg_status fl_pack_16(int W, bool for_, uint64_t ref, unsigned shift, bool sgn, const void* v, uint64_t n, void* packed,
                      hipStream_t s);
vxg_status fl_pack_32(int W, bool for_, uint64_t ref, unsigned shift, bool sgn, const void* v, uint64_t n, void* packed,
                      hipStream_t s);
vxg_status fl_pack_64(int W, bool for_, uint64_t ref, unsigned shift, bool sgn, const void* v, uint64_t n, void* packed,
                      hipStream_t s);
// FoR compress_primitive: out = (v - ref) >> shift (arithmetic if sgn), width-byte integers.
vxg_status launch_for_encode(int width, bool sgn, const void* v, uint64_t n, uint64_t ref, unsigned shift, void* out,
                             hipStream_t s);
// Synchronous (count read back): sorted indices + values of the elements wider than W bits.
vxg_status launch_gather_patches_gpu(int width, unsigned W, const void* v, uint64_t n, uint64_t* idx, void* vals,
                                     uint64_t cap, uint64_t* count, hipStream_t s);
// Synchronous: exponents, encoded ints (device), exceptions (device) and their count.
vxg_status launch_alp_encode(int float_ptype, const void* v, uint64_t n, uint8_t* e, uint8_t* f, void* enc,
                             uint64_t* idx, void* vals, uint64_t cap, uint64_t* count, hipStream_t s);

// K17 (fsst_encode.hip), synchronous: FSST-compress n strings (VarBin offsets of offs_width bytes
// + bytes, optional LSB validity) with a trained table into codes (i32 offsets, n + 1) and i32
// uncompressed lengths; *codes_len = code bytes written (at most codes_cap).
vxg_status launch_fsst_compress(const uint64_t* symbols, const uint8_t* sym_lens, uint32_t n_symbols, int offs_width,
                                bool offs_signed, const void* offsets, const uint8_t* bytes, uint64_t bytes_len,
                                const uint8_t* validity, uint64_t n, uint8_t* codes, uint64_t codes_cap,
                                int32_t* code_offsets, int32_t* ulens, uint64_t* codes_len, hipStream_t s);

}  // namespace vxg
