/*
 * vortex_enc.h — host-side encoders that produce Vortex encodings for the decode engine.
 *
 * The decode engine only canonicalizes; these restate the reference ENCODERS so that tests and
 * bench.py can synthesise arrays in exactly the layouts the reference writes (the encoder side
 * on GPU is SURVEY.md §8(f) row 4, "next").  All buffers are host memory, caller-allocated.
 * Each function cites the reference encoder it restates.
 */
#ifndef VORTEX_ENC_H
#define VORTEX_ENC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* bitpacking/compress.rs:82-137 bitpack_primitive.  Returns packed bytes = ceil(n/1024)*128*W. */
uint64_t vxe_bitpack(int ptype, unsigned bit_width, const void* values, uint64_t n, void* packed);

/* bitpacking/compress.rs:329-367 find_best_bit_width (exception cost = width + 4 bytes). */
unsigned vxe_best_bit_width(int ptype, const void* values, uint64_t n);
/* bitpacking/compress.rs:308-327 find_min_patchless_bit_width. */
unsigned vxe_min_patchless_bit_width(int ptype, const void* values, uint64_t n);

/* bitpacking/compress.rs:139-165 gather_patches: positions (u64) and values of every element
 * needing more than bit_width bits.  Returns count (writes at most `cap`). */
uint64_t vxe_gather_patches(int ptype, unsigned bit_width, const void* values, uint64_t n,
                            uint64_t* indices, void* patch_values, uint64_t cap);

/* for/compress.rs:13-85 for_compress: reference = min, shift = min trailing zeros
 * (stats/mod.rs:178-189).  encoded = (v - min) >> shift in the unsigned type.
 * Returns 0, or 1 if every value is 0 after shifting (reference emits a ConstantArray). */
int vxe_for_compress(int ptype, const void* values, uint64_t n, void* encoded,
                     uint64_t* reference, unsigned* shift);

/* delta/compress.rs:14-98 (unsigned ptypes).  bases: n/1024*LANES (+1 if remainder). */
void vxe_delta_compress(int ptype, const void* values, uint64_t n, void* bases, void* deltas);

/* zigzag 0.1.0 encode (zigzag/compress.rs:10-33); in_ptype signed. */
void vxe_zigzag_encode(int in_ptype, const void* values, uint64_t n, void* out);

/* alp/mod.rs:51-246 + alp/compress.rs:26-46: exponents search on a 32-value sample, encode,
 * patches (positions u64 + original values), patched slots filled with the first encodable
 * value.  Returns number of patches (writes at most cap). */
uint64_t vxe_alp_encode_f64(const double* values, uint64_t n, uint8_t* e, uint8_t* f,
                            int64_t* encoded, uint64_t* patch_idx, double* patch_vals, uint64_t cap);
uint64_t vxe_alp_encode_f32(const float* values, uint64_t n, uint8_t* e, uint8_t* f,
                            int32_t* encoded, uint64_t* patch_idx, float* patch_vals, uint64_t cap);

/* alp_rd/mod.rs:140-250 RDEncoder (deterministic tie-break: smaller left bits first).
 * dict: up to 8 u16; left: u16 codes; right: u32/u64 per float width; exceptions as
 * (pos u64, left bits u16).  Returns number of exceptions. */
uint64_t vxe_alprd_encode_f64(const double* values, uint64_t n, uint8_t* right_bit_width,
                              uint16_t* dict, uint8_t* dict_len, uint16_t* left, uint64_t* right,
                              uint64_t* exc_pos, uint16_t* exc, uint64_t cap);
uint64_t vxe_alprd_encode_f32(const float* values, uint64_t n, uint8_t* right_bit_width,
                              uint16_t* dict, uint8_t* dict_len, uint16_t* left, uint32_t* right,
                              uint64_t* exc_pos, uint16_t* exc, uint64_t cap);

/* dict/compress.rs:33-86 dict_encode_typed_primitive (non-nullable): codes u64 in order of
 * first appearance.  Returns number of distinct values written to `dict_values` (<= cap). */
uint64_t vxe_dict_encode(int value_width, const void* values, uint64_t n, uint64_t* codes,
                         void* dict_values, uint64_t cap);

/* runend/compress.rs:15-93 runend_encode: ends u64 (exclusive run ends), values.
 * Returns number of runs. */
uint64_t vxe_runend_encode(int value_width, const void* values, uint64_t n, uint64_t* ends,
                           void* run_values);

/* FSST (fsst-rs 0.4.3 is not vendored): a symbol-table trainer + greedy compressor that emits
 * streams in fsst-rs's code format (<=255 symbols of 1..8 bytes, code 255 = escape).  The
 * table differs from fsst-rs's trainer; decode semantics are identical. */
typedef struct vxe_fsst_table {
    uint64_t symbols[255];
    uint8_t lens[255];
    uint32_t n_symbols;
} vxe_fsst_table;
/* Train on strings given by (heap, offsets[n+1] i64). */
void vxe_fsst_train(const uint8_t* heap, const int64_t* offsets, uint64_t n, vxe_fsst_table* t);
/* Compress all strings; writes codes heap and code offsets (n+1, i32 like VarBinBuilder<i32>,
 * fsst/compress.rs:83-129).  Returns code bytes written, or UINT64_MAX if cap exceeded. */
uint64_t vxe_fsst_compress(const vxe_fsst_table* t, const uint8_t* heap, const int64_t* offsets,
                           uint64_t n, uint8_t* codes, uint64_t cap, int32_t* code_offsets);

/* roaring/src/boolean/compress.rs:7-14 roaring_bool_encode: Bitmap of the set positions of an LSB
 * bit buffer of len bits, run_optimize(), serialize::<Native>() (croaring 2.1.1, not vendored:
 * its published Native/portable format restated).  Returns the serialized size; bytes are
 * written only when it is <= cap. */
uint64_t vxe_roaring_bool_encode(const uint8_t* bits, uint64_t len, uint8_t* out, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* VORTEX_ENC_H */
