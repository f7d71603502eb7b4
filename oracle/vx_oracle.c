/*
 * vx_oracle.c — CPU restatement of the Vortex canonicalize/decompress hot path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline "port"); see vx_oracle.h.
 * Build: oracle/Makefile (gcc -O3 -march=native -ffp-contract=off, never -ffast-math: the ALP
 * decode is two IEEE round-to-nearest multiplies in a fixed order, alp/mod.rs:161-163).
 */
#include "vx_oracle.h"

#include <string.h>

int vxo_ptype_width(int p) {
    switch (p) {
    case VXO_U8: case VXO_I8: return 1;
    case VXO_U16: case VXO_I16: case VXO_F16: return 2;
    case VXO_U32: case VXO_I32: case VXO_F32: return 4;
    case VXO_U64: case VXO_I64: case VXO_F64: return 8;
    default: return 0;
    }
}

/* ======================================================================================
 * FastLanes 0.1.8 (crate not vendored in the reference; Cargo.lock:1515-1518).
 * Restated from the crate's published design:
 *   FL_ORDER = [0,4,2,6,1,5,3,7]
 *   index(row, lane) = FL_ORDER[row/8]*16 + (row%8)*128 + lane
 *   lane `l`, packed word `w` lives at packed[l + LANES*w]  (LANES = 1024/T)
 * Used by vortex at bitpacking/compress.rs:110,128,238,251,305 and delta/compress.rs:58,69,143,147.
 * ====================================================================================== */
static const unsigned FL_ORDER[8] = {0, 4, 2, 6, 1, 5, 3, 7};

unsigned vxo_fl_index(unsigned T, unsigned row, unsigned lane) {
    (void)T;
    return FL_ORDER[row / 8] * 16 + (row % 8) * 128 + lane;
}

unsigned vxo_fl_transpose(unsigned i) {
    /* fastlanes transpose(): lane*64 + FL_ORDER[order]*8 + row, lane=i%16, order=(i/16)%8,
     * row=i/128. */
    unsigned lane = i % 16, order = (i / 16) % 8, row = i / 128;
    return lane * 64 + FL_ORDER[order] * 8 + row;
}

static inline uint64_t mask_bits(unsigned bits) {
    return bits >= 64 ? ~(uint64_t)0 : (((uint64_t)1 << bits) - 1);
}

#define FL_DEFINE(TY, TBITS)                                                                 \
    static inline __attribute__((always_inline)) void fl_unpack_##TBITS(                    \
        unsigned W, const TY* restrict packed, TY* restrict out) {                          \
        enum { T = TBITS, LANES = 1024 / TBITS };                                            \
        if (W == 0) { memset(out, 0, 1024 * sizeof(TY)); return; }                           \
        if (W == T) {                                                                        \
            for (unsigned lane = 0; lane < LANES; lane++)                                    \
                for (unsigned row = 0; row < T; row++)                                       \
                    out[FL_ORDER[row / 8] * 16 + (row % 8) * 128 + lane] =                   \
                        packed[LANES * row + lane];                                          \
            return;                                                                          \
        }                                                                                    \
        const TY mask = (TY)mask_bits(W);                                                    \
        for (unsigned lane = 0; lane < LANES; lane++) {                                      \
            _Pragma("GCC unroll 64") for (unsigned row = 0; row < T; row++) {                \
                unsigned start = row * W, word = start / T, shift = start % T;               \
                TY v = (TY)(packed[LANES * word + lane] >> shift);                           \
                if (shift + W > T)                                                           \
                    v |= (TY)(packed[LANES * (word + 1) + lane] << (T - shift));             \
                out[FL_ORDER[row / 8] * 16 + (row % 8) * 128 + lane] = (TY)(v & mask);       \
            }                                                                                \
        }                                                                                    \
    }                                                                                        \
    static void fl_pack_##TBITS(unsigned W, const TY* restrict in, TY* restrict packed) {    \
        enum { T = TBITS, LANES = 1024 / TBITS };                                            \
        if (W == 0) return;                                                                  \
        if (W == T) {                                                                        \
            for (unsigned lane = 0; lane < LANES; lane++)                                    \
                for (unsigned row = 0; row < T; row++)                                       \
                    packed[LANES * row + lane] =                                             \
                        in[FL_ORDER[row / 8] * 16 + (row % 8) * 128 + lane];                 \
            return;                                                                          \
        }                                                                                    \
        const TY mask = (TY)mask_bits(W);                                                    \
        for (unsigned lane = 0; lane < LANES; lane++) {                                      \
            TY tmp = 0;                                                                      \
            for (unsigned row = 0; row < T; row++) {                                         \
                TY src = in[FL_ORDER[row / 8] * 16 + (row % 8) * 128 + lane] & mask;         \
                unsigned shift = (row * W) % T;                                              \
                if (row == 0) tmp = src; else tmp |= (TY)(src << shift);                     \
                unsigned cur = (row * W) / T, nxt = ((row + 1) * W) / T;                     \
                if (nxt > cur) {                                                             \
                    packed[LANES * cur + lane] = tmp;                                        \
                    unsigned rem = ((row + 1) * W) % T;                                      \
                    tmp = rem ? (TY)(src >> (W - rem)) : 0;                                  \
                }                                                                            \
            }                                                                                \
        }                                                                                    \
    }

FL_DEFINE(uint8_t, 8)
FL_DEFINE(uint16_t, 16)
FL_DEFINE(uint32_t, 32)
FL_DEFINE(uint64_t, 64)

void vxo_fl_pack_block(unsigned T, unsigned W, const void* vals, void* packed) {
    switch (T) {
    case 8: fl_pack_8(W, vals, packed); break;
    case 16: fl_pack_16(W, vals, packed); break;
    case 32: fl_pack_32(W, vals, packed); break;
    case 64: fl_pack_64(W, vals, packed); break;
    }
}

void vxo_fl_unpack_block(unsigned T, unsigned W, const void* packed, void* vals) {
    switch (T) {
    case 8: fl_unpack_8(W, packed, vals); break;
    case 16: fl_unpack_16(W, packed, vals); break;
    case 32: fl_unpack_32(W, packed, vals); break;
    case 64: fl_unpack_64(W, packed, vals); break;
    }
}

static uint64_t load_word(unsigned T, const void* p, size_t i) {
    switch (T) {
    case 8: return ((const uint8_t*)p)[i];
    case 16: return ((const uint16_t*)p)[i];
    case 32: return ((const uint32_t*)p)[i];
    default: return ((const uint64_t*)p)[i];
    }
}

uint64_t vxo_fl_unpack_single(unsigned T, unsigned W, const void* packed, unsigned index) {
    /* fastlanes unchecked_unpack_single; bitpacking/compress.rs:295-306 */
    const unsigned LANES = 1024 / T;
    if (W == 0) return 0;
    unsigned lane = index % LANES;
    unsigned s = index / 128;
    unsigned fl = (index - s * 128 - lane) / 16;
    unsigned row = FL_ORDER[fl] * 8 + s;
    if (W == T) return load_word(T, packed, (size_t)LANES * row + lane);
    unsigned start = row * W, word = start / T, shift = start % T;
    uint64_t v = load_word(T, packed, (size_t)LANES * word + lane) >> shift;
    if (shift + W > T) v |= load_word(T, packed, (size_t)LANES * (word + 1) + lane) << (T - shift);
    return v & mask_bits(W);
}

size_t vxo_bitpack(int ptype, unsigned W, const void* vals, size_t n, void* packed) {
    /* bitpacking/compress.rs:82-137 */
    const int bw = vxo_ptype_width(ptype);
    const unsigned T = 8u * (unsigned)bw;
    if (W == 0) return 0;
    const size_t nblk = (n + 1023) / 1024, full = n / 1024, blk_bytes = 128u * W;
    for (size_t b = 0; b < full; b++)
        vxo_fl_pack_block(T, W, (const uint8_t*)vals + b * 1024 * bw,
                          (uint8_t*)packed + b * blk_bytes);
    if (nblk != full) {
        uint64_t last[1024];
        memset(last, 0, sizeof last);
        memcpy(last, (const uint8_t*)vals + full * 1024 * bw, (n % 1024) * bw);
        vxo_fl_pack_block(T, W, last, (uint8_t*)packed + full * blk_bytes);
    }
    return nblk * blk_bytes;
}

int vxo_unpack(int ptype, unsigned W, unsigned offset, size_t len,
               const void* packed, size_t packed_bytes, void* out) {
    /* bitpacking/compress.rs:209-273 unpack_primitive */
    const int bw = vxo_ptype_width(ptype);
    const unsigned T = 8u * (unsigned)bw;
    if (W == 0) { memset(out, 0, len * bw); return 0; }                       /* :215-217 */
    const size_t nchunks = (offset + len + 1023) / 1024;                      /* :221 */
    const size_t blk_bytes = 128u * W;
    if (packed_bytes != nchunks * blk_bytes) return -1;                       /* :223-229 */
    uint64_t tmp[1024];
    size_t written = 0;
    for (size_t c = 0; c < nchunks && written < len; c++) {
        const uint8_t* src = (const uint8_t*)packed + c * blk_bytes;
        size_t skip = (c == 0) ? offset : 0;                                   /* :235-243 */
        size_t take = 1024 - skip;
        if (take > len - written) take = len - written;                        /* truncate :256 */
        if (skip == 0 && take == 1024) {
            vxo_fl_unpack_block(T, W, src, (uint8_t*)out + written * bw);      /* :246-253 */
        } else {
            vxo_fl_unpack_block(T, W, src, tmp);
            memcpy((uint8_t*)out + written * bw, (uint8_t*)tmp + skip * bw, take * bw);
        }
        written += take;
    }
    return 0;
}

int vxo_patch(int ptype, void* out, size_t out_len, int idx_ptype, const void* indices,
              uint64_t indices_offset, const void* values, size_t n) {
    /* sparse/mod.rs:132-144 resolved_indices: (idx as usize) - indices_offset;
     * primitive/mod.rs:168-185 patch: own_values[idx] = value. */
    const int bw = vxo_ptype_width(ptype);
    const int iw = vxo_ptype_width(idx_ptype);
    for (size_t i = 0; i < n; i++) {
        uint64_t idx = load_word(8u * iw, indices, i);
        if (idx_ptype >= VXO_I8 && idx_ptype <= VXO_I64 && iw < 8) {
            /* sign-extend signed index types */
            unsigned sh = 64 - 8 * iw;
            idx = (uint64_t)(((int64_t)(idx << sh)) >> sh);
        }
        idx -= indices_offset;
        if (idx >= out_len) return -1;
        memcpy((uint8_t*)out + idx * bw, (const uint8_t*)values + i * bw, bw);
    }
    return 0;
}

void vxo_for_decode(int ptype, const void* in, size_t n, uint64_t reference, unsigned shift,
                    void* out) {
    /* for/compress.rs:86-117: child reinterpreted to ptype (:89), (v << shift) wrapping_add
     * min.  Wrapping arithmetic is identical for signed and unsigned two's complement, so it
     * is computed on the unsigned bit pattern of the same width. */
    switch (vxo_ptype_width(ptype)) {
#define FOR_CASE(W, TY)                                                                      \
    case W: {                                                                                \
        const TY* a = in; TY* o = out; TY r = (TY)reference;                                 \
        for (size_t i = 0; i < n; i++) o[i] = (TY)((TY)(a[i] << shift) + r);                 \
    } break;
        FOR_CASE(1, uint8_t)
        FOR_CASE(2, uint16_t)
        FOR_CASE(4, uint32_t)
        FOR_CASE(8, uint64_t)
#undef FOR_CASE
    }
}

int vxo_delta_decode(int ptype, const void* bases, size_t n_bases, const void* deltas,
                     size_t n_deltas, size_t offset, size_t len, void* out) {
    /* delta/compress.rs:100-166 decompress_primitive; then slice(offset, offset+len) :111.
     * Full blocks: Delta::undelta (per lane running wrapping add in index(row,lane) order)
     * then Transpose::untranspose; remainder: scalar running sum from bases[last]. */
    const int bw = vxo_ptype_width(ptype);
    const unsigned T = 8u * (unsigned)bw, LANES = 1024 / T;
    const size_t nchunks = n_deltas / 1024, rem = n_deltas % 1024;
    if (n_bases != nchunks * LANES + (rem ? 1 : 0)) return -1;
    if (offset + len > n_deltas) return -1;
    uint64_t trans[1024], blk[1024];
    size_t written = 0;
#define DELTA_CASE(W, TY)                                                                    \
    case W: {                                                                                \
        const TY* B = bases; const TY* D = deltas; TY* O = out;                              \
        TY* tr = (TY*)trans; TY* bl = (TY*)blk;                                              \
        for (size_t c = 0; c < nchunks; c++) {                                               \
            size_t lo = c * 1024, hi = lo + 1024;                                            \
            if (hi <= offset || lo >= offset + len) continue;                                \
            const TY* d = D + lo;                                                            \
            for (unsigned lane = 0; lane < LANES; lane++) {                                  \
                TY prev = B[c * LANES + lane];                                               \
                for (unsigned row = 0; row < T; row++) {                                     \
                    unsigned idx = vxo_fl_index(T, row, lane);                               \
                    TY nx = (TY)(d[idx] + prev);                                             \
                    tr[idx] = nx; prev = nx;                                                 \
                }                                                                            \
            }                                                                                \
            for (unsigned i = 0; i < 1024; i++) bl[vxo_fl_transpose(i)] = tr[i];             \
            size_t s = offset > lo ? offset - lo : 0;                                        \
            size_t e = (offset + len < hi ? offset + len : hi) - lo;                         \
            memcpy(O + written, bl + s, (e - s) * sizeof(TY));                               \
            written += e - s;                                                                \
        }                                                                                    \
        if (rem) {                                                                           \
            TY base = B[nchunks * LANES];                                                    \
            for (size_t i = nchunks * 1024; i < n_deltas; i++) {                             \
                TY nx = (TY)(D[i] + base); base = nx;                                        \
                if (i >= offset && i < offset + len) O[written++] = nx;                      \
            }                                                                                \
        }                                                                                    \
    } break;
    switch (bw) {
        DELTA_CASE(1, uint8_t)
        DELTA_CASE(2, uint16_t)
        DELTA_CASE(4, uint32_t)
        DELTA_CASE(8, uint64_t)
    }
#undef DELTA_CASE
    return written == len ? 0 : -1;
}

void vxo_zigzag_decode(int out_ptype, const void* in, size_t n, void* out) {
    /* zigzag 0.1.0 decode: (n >> 1) ^ -((n & 1))  (zigzag/compress.rs:49-57) */
    switch (vxo_ptype_width(out_ptype)) {
#define ZZ_CASE(W, TY)                                                                       \
    case W: {                                                                                \
        const TY* a = in; TY* o = out;                                                       \
        for (size_t i = 0; i < n; i++) o[i] = (TY)((a[i] >> 1) ^ (TY)(0 - (a[i] & 1)));      \
    } break;
        ZZ_CASE(1, uint8_t)
        ZZ_CASE(2, uint16_t)
        ZZ_CASE(4, uint32_t)
        ZZ_CASE(8, uint64_t)
#undef ZZ_CASE
    }
}

/* ======================================================================================
 * ALP — encodings/alp/src/alp/mod.rs:255-351 (F10/IF10 tables), :161-163 decode_single.
 * ====================================================================================== */
const float VXO_F10_F32[11] = {1.0f, 10.0f, 100.0f, 1000.0f, 10000.0f, 100000.0f, 1000000.0f,
                               10000000.0f, 100000000.0f, 1000000000.0f, 10000000000.0f};
const float VXO_IF10_F32[11] = {1.0f, 0.1f, 0.01f, 0.001f, 0.0001f, 0.00001f, 0.000001f,
                                0.0000001f, 0.00000001f, 0.000000001f, 0.0000000001f};
const double VXO_F10_F64[24] = {
    1.0, 10.0, 100.0, 1000.0, 10000.0, 100000.0, 1000000.0, 10000000.0, 100000000.0,
    1000000000.0, 10000000000.0, 100000000000.0, 1000000000000.0, 10000000000000.0,
    100000000000000.0, 1000000000000000.0, 10000000000000000.0, 100000000000000000.0,
    1000000000000000000.0, 10000000000000000000.0, 100000000000000000000.0,
    1000000000000000000000.0, 10000000000000000000000.0, 100000000000000000000000.0};
const double VXO_IF10_F64[24] = {
    1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001, 0.00000001, 0.000000001,
    0.0000000001, 0.00000000001, 0.000000000001, 0.0000000000001, 0.00000000000001,
    0.000000000000001, 0.0000000000000001, 0.00000000000000001, 0.000000000000000001,
    0.0000000000000000001, 0.00000000000000000001, 0.000000000000000000001,
    0.0000000000000000000001, 0.00000000000000000000001};

void vxo_alp_decode_f32(const int32_t* enc, size_t n, unsigned e, unsigned f, float* out) {
    const float a = VXO_F10_F32[f], b = VXO_IF10_F32[e];
    for (size_t i = 0; i < n; i++) {
        float x = (float)enc[i] * a; /* SSE float: RN, no excess precision, no contraction */
        out[i] = x * b;
    }
}

void vxo_alp_decode_f64(const int64_t* enc, size_t n, unsigned e, unsigned f, double* out) {
    const double a = VXO_F10_F64[f], b = VXO_IF10_F64[e];
    for (size_t i = 0; i < n; i++) {
        double x = (double)enc[i] * a; /* SSE2 double: RN, no excess precision */
        out[i] = x * b;
    }
}

/* alp_rd/mod.rs:260-301 */
#define ALPRD_BODY(UT)                                                                       \
    for (size_t i = 0; i < n; i++) out_bits[i] = (UT)dict[left[i]];                          \
    for (size_t i = 0; i < n_exc; i++) out_bits[exc_pos[i]] = (UT)exc[i];                    \
    for (size_t i = 0; i < n; i++) out_bits[i] = (UT)((out_bits[i] << right_bw) | right[i]);

void vxo_alprd_decode_f32(const uint16_t* left, const uint16_t* dict, unsigned right_bw,
                          const uint32_t* right, size_t n, const uint64_t* exc_pos,
                          const uint16_t* exc, size_t n_exc, float* out) {
    uint32_t* out_bits = (uint32_t*)out;
    ALPRD_BODY(uint32_t)
}

void vxo_alprd_decode_f64(const uint16_t* left, const uint16_t* dict, unsigned right_bw,
                          const uint64_t* right, size_t n, const uint64_t* exc_pos,
                          const uint16_t* exc, size_t n_exc, double* out) {
    uint64_t* out_bits = (uint64_t*)out;
    ALPRD_BODY(uint64_t)
}

/* ======================================================================================
 * take — primitive/compute/take.rs:58-67 (indices as usize; OOB is a ComputeError/panic)
 * ====================================================================================== */
int vxo_take(int val_width, const void* values, size_t n_values, int code_ptype,
             const void* codes, size_t n, void* out) {
    const unsigned cw = 8u * (unsigned)vxo_ptype_width(code_ptype);
    for (size_t i = 0; i < n; i++) {
        uint64_t c = load_word(cw, codes, i);
        if (c >= n_values) return -1;
        memcpy((uint8_t*)out + i * val_width, (const uint8_t*)values + c * val_width, val_width);
    }
    return 0;
}

/* runend/compress.rs:115-148: trimmed = min(end - offset, length); repeat value. */
int vxo_runend_decode(int val_width, const void* values, int ends_ptype, const void* ends,
                      size_t n_runs, size_t offset, size_t len, void* out) {
    const unsigned ew = 8u * (unsigned)vxo_ptype_width(ends_ptype);
    size_t pos = 0;
    for (size_t r = 0; r < n_runs; r++) {
        uint64_t end = load_word(ew, ends, r) - (uint64_t)offset;
        if (end > len) end = len;
        if (end < pos) return -1; /* ends must be non-decreasing */
        for (; pos < end; pos++)
            memcpy((uint8_t*)out + pos * val_width, (const uint8_t*)values + r * val_width,
                   val_width);
    }
    return pos == len ? 0 : -1;
}

/* ======================================================================================
 * Bool encodings.  RunEndBool: encodings/runend-bool/src/compress.rs:46-93 (decode), :16-41
 * (encode, BooleanBuffer::set_slices = maximal runs of set bits); ByteBool:
 * encodings/bytebool/src/array.rs:138-146 (bytes reinterpreted as bools -> BooleanBuffer).
 * ====================================================================================== */
static int get_bit(const uint8_t* b, size_t i) { return (b[i >> 3] >> (i & 7)) & 1; }
static void put_bit(uint8_t* b, size_t i, int v) {
    if (v) b[i >> 3] |= (uint8_t)(1u << (i & 7));
}

int vxo_runend_bool_decode(int ends_ptype, const void* ends, size_t n_runs, size_t offset, int start,
                           size_t len, uint8_t* out_bits) {
    const unsigned ew = 8u * (unsigned)vxo_ptype_width(ends_ptype);
    memset(out_bits, 0, (len + 7) / 8);
    size_t pos = 0;
    for (size_t r = 0; r < n_runs; r++) {
        uint64_t end = load_word(ew, ends, r) - (uint64_t)offset; /* trimmed_ends */
        if (end > len) end = len;
        if (end < pos) return -1;
        const int v = (r % 2 == 0) ? (start != 0) : (start == 0); /* value_at_index */
        for (; pos < end; pos++) put_bit(out_bits, pos, v);
    }
    return pos == len ? 0 : -1;
}

size_t vxo_runend_bool_encode(const uint8_t* bits, size_t len, uint64_t* ends, int* start) {
    size_t n = 0, i = 0;
    /* first set slice */
    while (i < len && !get_bit(bits, i)) i++;
    if (i == len) { /* no set bits */
        ends[0] = len;
        *start = 0;
        return 1;
    }
    *start = i == 0;
    if (i != 0) ends[n++] = i;
    for (;;) {
        size_t e = i;
        while (e < len && get_bit(bits, e)) e++;
        ends[n++] = e; /* end of the set slice */
        i = e;
        while (i < len && !get_bit(bits, i)) i++;
        if (i == len) break;
        ends[n++] = i; /* start of the next set slice */
    }
    if (ends[n - 1] != len) ends[n++] = len;
    return n;
}

void vxo_bytebool_to_bits(const uint8_t* bytes, size_t n, uint8_t* out_bits) {
    memset(out_bits, 0, (n + 7) / 8);
    for (size_t i = 0; i < n; i++) put_bit(out_bits, i, bytes[i] != 0);
}

/* RoaringBool: croaring (2.1.1, not vendored) Native deserialization + to_bitset.  Byte 0 picks
 * the format: 1 = u32 cardinality + that many u32 values, 2 = the portable format (cookie 12346:
 * + u32 size, keys/cardinality-1 pairs, u32 offsets; cookie 12347 | (size-1) << 16: run-container
 * bitset, pairs, offsets when size >= 4).  Containers: run (bit set) = u16 n_runs + (start,
 * length-1) pairs; cardinality <= 4096 = sorted u16 values; else 1024 u64 bitset words. */
static uint32_t rd16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
static uint32_t rd32(const uint8_t* p) { return rd16(p) | (rd16(p + 2) << 16); }

int vxo_roaring_bool_decode(const uint8_t* buf, size_t n, size_t len, uint8_t* out_bits) {
    memset(out_bits, 0, (len + 7) / 8);
    if (n < 1) return -1;
    uint64_t card_total = 0;
    if (buf[0] == 1) {
        if (n < 5) return -1;
        const uint32_t card = rd32(buf + 1);
        if (5 + 4 * (uint64_t)card > n) return -1;
        for (uint32_t i = 0; i < card; i++) {
            const uint32_t v = rd32(buf + 5 + 4 * (size_t)i);
            if (v < len) put_bit(out_bits, v, 1);
        }
        return 0;
    }
    if (buf[0] != 2) return -1;
    const uint8_t* p = buf + 1;
    const size_t m = n - 1;
    if (m < 4) return -1;
    const uint32_t cookie = rd32(p);
    size_t size, pos;
    const uint8_t* runbits = NULL;
    int has_offsets;
    if ((cookie & 0xFFFF) == 12347) {
        size = (cookie >> 16) + 1;
        runbits = p + 4;
        pos = 4 + (size + 7) / 8;
        has_offsets = size >= 4;
    } else if (cookie == 12346) {
        if (m < 8) return -1;
        size = rd32(p + 4);
        pos = 8;
        has_offsets = 1;
    } else {
        return -1;
    }
    if (size > 65536 || pos + 4 * size > m) return -1;
    const uint8_t* desc = p + pos;
    pos += 4 * size;
    const uint8_t* offs = NULL;
    if (has_offsets) {
        if (pos + 4 * size > m) return -1;
        offs = p + pos;
        pos += 4 * size;
    }
    for (size_t k = 1; k < size; k++)
        if (rd16(desc + 4 * k) <= rd16(desc + 4 * (k - 1))) return -1; /* keys strictly increasing */
    for (size_t k = 0; k < size; k++) {
        const uint32_t key = rd16(desc + 4 * k), card = rd16(desc + 4 * k + 2) + 1;
        const int run = runbits && ((runbits[k / 8] >> (k % 8)) & 1);
        if (offs) pos = rd32(offs + 4 * k);
        if (pos > m) return -1;
        const uint8_t* c = p + pos;
        const uint64_t base = (uint64_t)key << 16;
        size_t bytes;
        if (run) {
            if (pos + 2 > m) return -1;
            const uint32_t nr = rd16(c);
            bytes = 2 + 4 * (size_t)nr;
            if (pos + bytes > m) return -1;
            uint64_t cnt = 0;
            for (uint32_t r = 0; r < nr; r++) {
                const uint32_t st = rd16(c + 2 + 4 * r), ln = rd16(c + 4 + 4 * r);
                if (st + ln > 65535) return -1; /* a run past its container */
                for (uint32_t x = st; x <= st + ln; x++) {
                    if (base + x < len) put_bit(out_bits, base + x, 1);
                    cnt++;
                }
            }
            card_total += cnt;
        } else if (card <= 4096) {
            bytes = 2 * (size_t)card;
            if (pos + bytes > m) return -1;
            for (uint32_t i = 0; i < card; i++) {
                const uint64_t v = base + rd16(c + 2 * i);
                if (v < len) put_bit(out_bits, v, 1);
            }
            card_total += card;
        } else {
            bytes = 8192;
            if (pos + bytes > m) return -1;
            for (uint32_t x = 0; x < 65536; x++)
                if ((c[x >> 3] >> (x & 7)) & 1) {
                    if (base + x < len) put_bit(out_bits, base + x, 1);
                    card_total++;
                }
        }
        pos += bytes;
    }
    (void)card_total;
    return 0;
}

void vxo_fill(int val_width, const void* scalar, size_t n, void* out) {
    for (size_t i = 0; i < n; i++) memcpy((uint8_t*)out + i * val_width, scalar, val_width);
}

/* ======================================================================================
 * FSST — fsst-rs 0.4.3 Decompressor::decompress (not vendored; Cargo.lock:1621-1624).
 * code 255 = escape: next byte literal; else copy sym_lens[c] bytes of symbols[c] (LE u64).
 * ====================================================================================== */
size_t vxo_fsst_decompress(const uint64_t* symbols, const uint8_t* sym_lens,
                           const uint8_t* codes, size_t n_codes, uint8_t* out) {
    size_t o = 0;
    for (size_t i = 0; i < n_codes; i++) {
        uint8_t c = codes[i];
        if (c == 255) {
            out[o++] = codes[++i];
        } else {
            memcpy(out + o, &symbols[c], 8); /* fsst-rs writes the whole 8-byte word */
            o += sym_lens[c];
        }
    }
    return o;
}

static int64_t load_off(int ptype, const void* p, size_t i) {
    switch (ptype) {
    case VXO_I32: return ((const int32_t*)p)[i];
    case VXO_U32: return ((const uint32_t*)p)[i];
    case VXO_I64: return ((const int64_t*)p)[i];
    case VXO_U64: return (int64_t)((const uint64_t*)p)[i];
    case VXO_U16: return ((const uint16_t*)p)[i];
    case VXO_I16: return ((const int16_t*)p)[i];
    case VXO_U8: return ((const uint8_t*)p)[i];
    case VXO_I8: return ((const int8_t*)p)[i];
    default: return 0;
    }
}

void vxo_make_views(const uint8_t* heap, const int64_t* offsets, size_t n,
                    const uint8_t* validity, uint32_t buffer_index, uint8_t* views) {
    /* arrow-array 53.2 make_view / GenericByteViewBuilder::append_null (null view == 0) */
    for (size_t i = 0; i < n; i++) {
        uint8_t* v = views + 16 * i;
        memset(v, 0, 16);
        if (validity && !((validity[i >> 3] >> (i & 7)) & 1)) continue;
        uint32_t start = (uint32_t)offsets[i];
        uint32_t len = (uint32_t)(offsets[i + 1] - offsets[i]);
        memcpy(v, &len, 4);
        if (len <= 12) {
            memcpy(v + 4, heap + start, len);
        } else {
            memcpy(v + 4, heap + start, 4);
            memcpy(v + 8, &buffer_index, 4);
            memcpy(v + 12, &start, 4);
        }
    }
}

int vxo_fsst_canonicalize(const uint64_t* symbols, const uint8_t* sym_lens,
                          const uint8_t* code_bytes, int offs_ptype, const void* code_offsets,
                          int lens_ptype, const void* ulens, size_t n,
                          const uint8_t* validity, uint8_t* heap, size_t* heap_len,
                          uint8_t* views) {
    /* fsst/canonical.rs:20-26: decompress sliced_bytes() = code_bytes[off[0]..off[n]] in bulk */
    int64_t first = load_off(offs_ptype, code_offsets, 0);
    int64_t last = load_off(offs_ptype, code_offsets, n);
    size_t hl = vxo_fsst_decompress(symbols, sym_lens, code_bytes + first,
                                    (size_t)(last - first), heap);
    /* canonical.rs:29-42: offsets = prefix sum of uncompressed lengths (read as i32 :37) */
    int64_t acc = 0;
    for (size_t i = 0; i < n; i++) {
        int64_t l = load_off(lens_ptype, ulens, i);
        int64_t o2[2] = {acc, acc + l};
        vxo_make_views(heap, o2, 1, NULL, 0, views + 16 * i);
        if (validity && !((validity[i >> 3] >> (i & 7)) & 1)) memset(views + 16 * i, 0, 16);
        acc += l;
    }
    if ((size_t)acc != hl) return -1;
    *heap_len = hl;
    return 0;
}

void vxo_rebase_views(uint8_t* views, size_t n, uint32_t buffers_offset) {
    /* chunked/canonical.rs:214-231: view.is_inlined() (len <= 12) -> copied as is, else
     * BinaryView::new_view(len, prefix, buffers_offset + buffer_index, offset) */
    for (size_t i = 0; i < n; i++) {
        uint8_t* v = views + 16 * i;
        uint32_t len, bi;
        memcpy(&len, v, 4);
        if (len <= 12) continue;
        memcpy(&bi, v + 8, 4);
        bi += buffers_offset;
        memcpy(v + 8, &bi, 4);
    }
}
