/*
 * vx_oracle.h — CPU restatement of the spiraldb/vortex canonicalize/decompress hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the HIP engine in vortex_amd/.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / CPU baseline — never as the thing measured or shipped.
 *
 * Every function cites the reference file:line it restates (paths under the reference
 * checkout, workspace 0.12.0).  Third-party arithmetic that is not vendored in the reference
 * (fastlanes 0.1.8, fsst-rs 0.4.3, zigzag 0.1.0, arrow-cast 53.2) is restated from the
 * crates' published algorithms; see DESIGN.md "Oracle" for what is pinned by reference
 * known-answer tests and what is "parity unpinned" (the FastLanes packed bit layout).
 *
 * Plain C11; no allocation inside the decoders (callers own every buffer).
 */
#ifndef VX_ORACLE_H
#define VX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* PType codes: vortex-dtype/src/ptype.rs:19-31 (and dtype.fbs enum PType). */
enum {
    VXO_U8 = 0, VXO_U16 = 1, VXO_U32 = 2, VXO_U64 = 3,
    VXO_I8 = 4, VXO_I16 = 5, VXO_I32 = 6, VXO_I64 = 7,
    VXO_F16 = 8, VXO_F32 = 9, VXO_F64 = 10
};

int vxo_ptype_width(int ptype); /* bytes */

/* ---- FastLanes (fastlanes 0.1.8) ---------------------------------- */
/* index(row, lane) of the FastLanes unified transposed layout, T = bits of the type. */
unsigned vxo_fl_index(unsigned T, unsigned row, unsigned lane);
/* transpose(i) used by Delta (fastlanes transpose.rs). */
unsigned vxo_fl_transpose(unsigned i);

/* One 1024-value block.  T in {8,16,32,64}; `packed` holds 128*W bytes; `vals` 1024 of T. */
void vxo_fl_pack_block(unsigned T, unsigned W, const void* vals, void* packed);
void vxo_fl_unpack_block(unsigned T, unsigned W, const void* packed, void* vals);
uint64_t vxo_fl_unpack_single(unsigned T, unsigned W, const void* packed, unsigned index);

/* bitpacking/compress.rs:82-137 bitpack_primitive (zero-padded last block).
 * ptype must be unsigned; returns bytes written = ceil(n/1024)*128*W. */
size_t vxo_bitpack(int ptype, unsigned W, const void* vals, size_t n, void* packed);

/* bitpacking/compress.rs:209-273 unpack_primitive: skip `offset` (<1024), keep `len`. */
int vxo_unpack(int ptype, unsigned W, unsigned offset, size_t len,
               const void* packed, size_t packed_bytes, void* out);

/* SparseArray::resolved_indices (array/sparse/mod.rs:132-144) + PrimitiveArray::patch
 * (array/primitive/mod.rs:168-185): out[idx[i] - indices_offset] = values[i]. */
int vxo_patch(int ptype, void* out, size_t out_len,
              int idx_ptype, const void* indices, uint64_t indices_offset,
              const void* values, size_t n_patches);

/* for/compress.rs:100-117 decompress_primitive: out = (v << shift) wrapping_add reference.
 * Works in place (in == out allowed).  `reference` is the little-endian bit pattern. */
void vxo_for_decode(int ptype, const void* in, size_t n, uint64_t reference, unsigned shift,
                    void* out);

/* delta/compress.rs:100-166 decompress_primitive + slice [offset, offset+len) (:111). */
int vxo_delta_decode(int ptype, const void* bases, size_t n_bases,
                     const void* deltas, size_t n_deltas, size_t offset, size_t len, void* out);

/* zigzag/compress.rs:35-57 (zigzag 0.1.0): i = (u >> 1) ^ -(u & 1). ptype = OUTPUT signed. */
void vxo_zigzag_decode(int out_ptype, const void* in, size_t n, void* out);

/* ---- ALP (encodings/alp/src/alp/mod.rs) ---------------------------------------------- */
extern const float  VXO_F10_F32[11];
extern const float  VXO_IF10_F32[11];
extern const double VXO_F10_F64[24];
extern const double VXO_IF10_F64[24];
/* alp/mod.rs:161-163 decode_single; alp/compress.rs:98-106 decompress_primitive. */
void vxo_alp_decode_f32(const int32_t* enc, size_t n, unsigned e, unsigned f, float* out);
void vxo_alp_decode_f64(const int64_t* enc, size_t n, unsigned e, unsigned f, double* out);

/* alp_rd/mod.rs:260-301 alp_rd_decode. left_parts are u16 codes into dict. */
void vxo_alprd_decode_f32(const uint16_t* left, const uint16_t* dict, unsigned right_bw,
                          const uint32_t* right, size_t n, const uint64_t* exc_pos,
                          const uint16_t* exc, size_t n_exc, float* out);
void vxo_alprd_decode_f64(const uint16_t* left, const uint16_t* dict, unsigned right_bw,
                          const uint64_t* right, size_t n, const uint64_t* exc_pos,
                          const uint16_t* exc, size_t n_exc, double* out);

/* ---- Dict / take ----------------------------------------------------------------------- */
/* dict/array.rs:68-73 -> compute/take.rs:10-34 -> primitive/compute/take.rs:58-67.
 * Returns -1 (OutOfBounds) if any code >= n_values. */
int vxo_take(int val_width, const void* values, size_t n_values,
             int code_ptype, const void* codes, size_t n, void* out);

/* ---- RunEnd ---------------------------------------------------------------------------- */
/* runend/compress.rs:115-148 runend_decode_primitive. */
int vxo_runend_decode(int val_width, const void* values, int ends_ptype, const void* ends,
                      size_t n_runs, size_t offset, size_t len, void* out);

/* ---- Bool encodings (canonical Bool = LSB bit buffer, arrow BooleanBuffer) -------------- */
/* encodings/runend-bool/src/compress.rs:46-93 runend_bool_decode_slice: ends' = min(end -
 * offset, len); run r holds value_at_index(r, start) = start ^ (r odd) for positions
 * [ends'[r-1], ends'[r]).  Writes len bits into out_bits (zeroed first, ceil(len/8) bytes).
 * Returns -1 if the ends are not non-decreasing or do not reach len. */
int vxo_runend_bool_decode(int ends_ptype, const void* ends, size_t n_runs, size_t offset, int start,
                           size_t len, uint8_t* out_bits);
/* runend-bool/src/compress.rs:16-41 runend_bool_encode_slice over an LSB bit buffer of len bits:
 * writes the u64 ends (room for len + 1) and *start; returns the number of ends. */
size_t vxo_runend_bool_encode(const uint8_t* bits, size_t len, uint64_t* ends, int* start);
/* bytebool/src/array.rs:138-146 into_canonical: one byte per bool -> bit (byte != 0). */
void vxo_bytebool_to_bits(const uint8_t* bytes, size_t n, uint8_t* out_bits);
/* roaring/src/boolean/mod.rs:69-72,127-147: Bitmap::deserialize::<Native> (croaring 2.1.1,
 * not vendored: restated from its published format) + to_bitset, len bits (positions >= len
 * dropped).  Returns 0, or -1 for a malformed serialization. */
int vxo_roaring_bool_decode(const uint8_t* buf, size_t n, size_t len, uint8_t* out_bits);

/* ---- Sparse / Constant canonical (array/sparse/flatten.rs:68-98; constant/canonical.rs) - */
void vxo_fill(int val_width, const void* scalar, size_t n, void* out);

/* ---- FSST (fsst-rs 0.4.3 Decompressor) ------------------------------ */
/* Decompress a code stream; returns number of bytes written.  `out` must have room for
 * 8*n_codes bytes (symbols are written as 8-byte words, like fsst-rs). */
size_t vxo_fsst_decompress(const uint64_t* symbols, const uint8_t* sym_lens,
                           const uint8_t* codes, size_t n_codes, uint8_t* out);

/* fsst/canonical.rs:7-57 + varbin/flatten.rs:10-17 (arrow-cast 53.2 Utf8->Utf8View,
 * SURVEY Appendix C).  code_offsets: n+1 entries (i32 or i64 via offs_ptype).
 * `validity` is an LSB bitmap or NULL (all valid).  Writes heap (returns heap bytes via
 * *heap_len) and 16-byte views.  heap needs room for sum(lens)+8. */
int vxo_fsst_canonicalize(const uint64_t* symbols, const uint8_t* sym_lens,
                          const uint8_t* code_bytes, int offs_ptype, const void* code_offsets,
                          int lens_ptype, const void* uncompressed_lens, size_t n,
                          const uint8_t* validity, uint8_t* heap, size_t* heap_len,
                          uint8_t* views);

/* arrow-cast 53.2 cast(Utf8 -> Utf8View) view construction (make_view), block 0. */
void vxo_make_views(const uint8_t* heap, const int64_t* offsets, size_t n,
                    const uint8_t* validity, uint32_t buffer_index, uint8_t* views);

/* pack_views (array/chunked/canonical.rs:214-231): add `buffers_offset` to the buffer_index
 * of every non-inlined view (len > 12); inlined views are left unchanged. */
void vxo_rebase_views(uint8_t* views, size_t n, uint32_t buffers_offset);

#ifdef __cplusplus
}
#endif
#endif /* VX_ORACLE_H */
