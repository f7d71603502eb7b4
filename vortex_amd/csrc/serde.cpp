// serde.cpp — host-side reader of Vortex files and IPC messages (include/vortex_file.h).
//
// Restates, without any flatbuffers/flexbuffers library (none in this image):
//   * vortex-serde/src/layouts/read/footer.rs:140-187  EOF (version u16 = 1, "VRTX"), the 32-byte
//     Postscript {schema_offset, footer_offset}, the Schema message and the Footer flatbuffer;
//   * layouts/read/layouts/{column,chunked,flat,inline_dtype}.rs  the layout tree (ids 3/2/1/4,
//     layouts/mod.rs:13-16; a Chunked layout's metadata byte says whether child 0 is the
//     row_offset metadata table);
//   * message_reader.rs:249-348  ArrayBufferReader: u32 length prefix, flatbuffer Message with a
//     Batch header {array, length, buffers[{offset, padding, compression}], buffer_size}, the
//     buffers split sequentially (len = next_offset - offset - padding);
//   * vortex-array/src/view.rs:45-172  ArrayView: encoding by u16 id, metadata bytes, optional
//     buffer_index, children whose dtype and length the parent encoding derives (the accessors
//     cited per encoding below);
//   * vortex-array/src/metadata.rs:35-47  metadata = serde structs serialized as flexbuffers
//     (structs -> maps keyed by field name, unit enum variants -> strings, PType -> lowercase
//     string (ptype.rs:19), Nullability -> bool (vortex-dtype/src/serde/serde.rs:7-24),
//     ScalarValue -> its primitive (vortex-scalar/src/serde/serde.rs:10-24)).
// Schemas: vortex-flatbuffers/flatbuffers/{vortex-serde/message.fbs, footer.fbs,
// vortex-array/array.fbs, vortex-dtype/dtype.fbs}.
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/vortex_file.h"

namespace vxg {
vxg_status set_error(vxg_status s, const std::string& msg);
}

namespace {

struct SerdeError : std::runtime_error {
    vxg_status st;
    SerdeError(vxg_status s, const std::string& m) : std::runtime_error(m), st(s) {}
};
[[noreturn]] void bad(const std::string& m) { throw SerdeError(VXG_ERR_INVALID_SERDE, m); }
[[noreturn]] void unsupported(const std::string& m) { throw SerdeError(VXG_ERR_NOT_IMPLEMENTED, m); }

template <class T> T rd(const uint8_t* buf, size_t len, size_t pos) {
    if (pos > len || len - pos < sizeof(T)) bad("read past the end of a buffer");
    T v;
    std::memcpy(&v, buf + pos, sizeof(T));
    return v;
}

// =========================================================================== flatbuffers
// Table: [soffset to vtable][fields]; vtable: [u16 vtable bytes][u16 table bytes][u16 field
// offsets...]; offsets to tables/vectors/strings are u32 relative to their own position.
struct FbTable {
    const uint8_t* buf = nullptr;
    size_t len = 0, pos = 0, vt = 0;
    uint16_t vt_size = 0;

    static FbTable at(const uint8_t* b, size_t n, size_t pos) {
        FbTable t;
        t.buf = b;
        t.len = n;
        t.pos = pos;
        const int64_t vt = int64_t(pos) - int64_t(rd<int32_t>(b, n, pos));
        if (vt < 0 || size_t(vt) + 4 > n) bad("flatbuffer vtable out of range");
        t.vt = size_t(vt);
        t.vt_size = rd<uint16_t>(b, n, t.vt);
        if (t.vt_size < 4 || (t.vt_size & 1) || t.vt + t.vt_size > n) bad("flatbuffer vtable malformed");
        return t;
    }
    static FbTable root(const uint8_t* b, size_t n) { return at(b, n, rd<uint32_t>(b, n, 0)); }

    uint16_t off(int field) const {
        const size_t o = 4 + 2 * size_t(field);
        return o + 2 <= vt_size ? rd<uint16_t>(buf, len, vt + o) : 0;
    }
    bool has(int field) const { return off(field) != 0; }
    template <class T> T get(int field, T def) const {
        const uint16_t o = off(field);
        return o ? rd<T>(buf, len, pos + o) : def;
    }
    size_t deref(int field) const {  // absolute position of the referenced object
        const size_t p = pos + off(field);
        const size_t t = p + rd<uint32_t>(buf, len, p);
        if (t >= len) bad("flatbuffer offset out of range");
        return t;
    }
    bool table(int field, FbTable* out) const {
        if (!has(field)) return false;
        *out = at(buf, len, deref(field));
        return true;
    }
    // vector: element count + position of element 0
    bool vector(int field, size_t elem, uint32_t* n, size_t* data) const {
        if (!has(field)) return false;
        const size_t v = deref(field);
        *n = rd<uint32_t>(buf, len, v);
        *data = v + 4;
        if (*data + uint64_t(*n) * elem > len) bad("flatbuffer vector out of range");
        return true;
    }
    FbTable vec_table(size_t data, uint32_t i) const {
        const size_t p = data + 4 * size_t(i);
        return at(buf, len, p + rd<uint32_t>(buf, len, p));
    }
    std::string vec_string(size_t data, uint32_t i) const {
        const size_t p = data + 4 * size_t(i);
        const size_t s = p + rd<uint32_t>(buf, len, p);
        const uint32_t n = rd<uint32_t>(buf, len, s);
        if (s + 4 + uint64_t(n) > len) bad("flatbuffer string out of range");
        return std::string(reinterpret_cast<const char*>(buf + s + 4), n);
    }
    std::string string(int field) const {
        uint32_t n;
        size_t d;
        if (!vector(field, 1, &n, &d)) return std::string();
        return std::string(reinterpret_cast<const char*>(buf + d), n);
    }
};

// =========================================================================== flexbuffers
// A value = (slot position, slot byte width, packed type).  Inline scalars live in the slot;
// everything else is an unsigned offset back from the slot to the object, whose element byte
// width is the packed type's low 2 bits.  Vectors/maps carry a size prefix (and maps the keys
// vector offset + its byte width before that); untyped vectors/maps are followed by one packed
// type byte per element.
enum FlexType : uint8_t {
    FX_NULL = 0, FX_INT = 1, FX_UINT = 2, FX_FLOAT = 3, FX_KEY = 4, FX_STRING = 5, FX_IND_INT = 6,
    FX_IND_UINT = 7, FX_IND_FLOAT = 8, FX_MAP = 9, FX_VECTOR = 10, FX_VEC_INT = 11, FX_VEC_UINT = 12,
    FX_VEC_FLOAT = 13, FX_VEC_KEY = 14, FX_VEC_STRING_DEPRECATED = 15, FX_VEC_INT2 = 16, FX_VEC_FLOAT4 = 24,
    FX_BLOB = 25, FX_BOOL = 26, FX_VEC_BOOL = 36
};

struct Flex {
    const uint8_t* buf = nullptr;
    size_t len = 0, pos = 0;
    uint8_t parent_width = 1, width = 1, type = FX_NULL;

    static Flex root(const uint8_t* b, size_t n) {
        if (n < 3) bad("flexbuffer too short");
        Flex f;
        f.buf = b;
        f.len = n;
        f.parent_width = b[n - 1];
        const uint8_t packed = b[n - 2];
        if (f.parent_width != 1 && f.parent_width != 2 && f.parent_width != 4 && f.parent_width != 8)
            bad("flexbuffer root width");
        if (n < 2 + size_t(f.parent_width)) bad("flexbuffer root out of range");
        f.pos = n - 2 - f.parent_width;
        f.width = uint8_t(1u << (packed & 3));
        f.type = packed >> 2;
        return f;
    }
    uint64_t ru(size_t p, int w) const {
        switch (w) {
        case 1: return rd<uint8_t>(buf, len, p);
        case 2: return rd<uint16_t>(buf, len, p);
        case 4: return rd<uint32_t>(buf, len, p);
        case 8: return rd<uint64_t>(buf, len, p);
        default: bad("flexbuffer width");
        }
    }
    int64_t ri(size_t p, int w) const {
        switch (w) {
        case 1: return rd<int8_t>(buf, len, p);
        case 2: return rd<int16_t>(buf, len, p);
        case 4: return rd<int32_t>(buf, len, p);
        case 8: return rd<int64_t>(buf, len, p);
        default: bad("flexbuffer width");
        }
    }
    double rf(size_t p, int w) const {
        if (w == 4) return rd<float>(buf, len, p);
        if (w == 8) return rd<double>(buf, len, p);
        bad("flexbuffer float width");
    }
    size_t target() const {
        const uint64_t o = ru(pos, parent_width);
        if (o > pos) bad("flexbuffer offset out of range");
        return pos - size_t(o);
    }
    bool is_null() const { return type == FX_NULL; }
    bool is_int_like() const {
        return type == FX_INT || type == FX_UINT || type == FX_BOOL || type == FX_IND_INT || type == FX_IND_UINT;
    }
    int64_t as_i64() const {
        switch (type) {
        case FX_INT: return ri(pos, parent_width);
        case FX_UINT: case FX_BOOL: return int64_t(ru(pos, parent_width));
        case FX_IND_INT: return ri(target(), width);
        case FX_IND_UINT: return int64_t(ru(target(), width));
        case FX_FLOAT: return int64_t(rf(pos, parent_width));
        case FX_IND_FLOAT: return int64_t(rf(target(), width));
        default: bad("flexbuffer value is not a number");
        }
    }
    uint64_t as_u64() const {
        if (type == FX_UINT || type == FX_BOOL) return ru(pos, parent_width);
        if (type == FX_IND_UINT) return ru(target(), width);
        return uint64_t(as_i64());
    }
    double as_f64() const {
        if (type == FX_FLOAT) return rf(pos, parent_width);
        if (type == FX_IND_FLOAT) return rf(target(), width);
        if (type == FX_UINT || type == FX_IND_UINT) return double(as_u64());
        return double(as_i64());
    }
    bool as_bool() const {
        if (type != FX_BOOL && !is_int_like()) bad("flexbuffer value is not a bool");
        return as_u64() != 0;
    }
    std::string as_string() const {
        if (type == FX_KEY) {
            const size_t t = target();
            size_t e = t;
            while (e < len && buf[e]) e++;
            if (e >= len) bad("flexbuffer key not terminated");
            return std::string(reinterpret_cast<const char*>(buf + t), e - t);
        }
        if (type != FX_STRING && type != FX_BLOB) bad("flexbuffer value is not a string");
        const size_t t = target();
        if (t < width) bad("flexbuffer string size out of range");
        const uint64_t n = ru(t - width, width);
        if (t + n > len) bad("flexbuffer string out of range");
        return std::string(reinterpret_cast<const char*>(buf + t), size_t(n));
    }
    bool is_vector() const {
        return type == FX_MAP || type == FX_VECTOR || (type >= FX_VEC_INT && type <= FX_VEC_FLOAT4) ||
               type == FX_VEC_BOOL;
    }
    uint64_t size() const {
        if (type >= FX_VEC_INT2 && type <= FX_VEC_FLOAT4) return uint64_t((type - FX_VEC_INT2) / 3 + 2);
        if (!is_vector()) bad("flexbuffer value is not a vector");
        const size_t t = target();
        if (t < width) bad("flexbuffer vector size out of range");
        return ru(t - width, width);
    }
    Flex at(uint64_t i) const {
        const uint64_t n = size();
        if (i >= n) bad("flexbuffer index out of range");
        const size_t t = target();
        Flex e;
        e.buf = buf;
        e.len = len;
        e.pos = t + size_t(i) * width;
        e.parent_width = width;
        e.width = width;
        if (type == FX_MAP || type == FX_VECTOR) {
            const uint8_t packed = uint8_t(ru(t + size_t(n) * width + size_t(i), 1));
            e.type = packed >> 2;
            e.width = uint8_t(1u << (packed & 3));
        } else if (type == FX_VEC_BOOL) {
            e.type = FX_BOOL;
        } else if (type == FX_VEC_KEY) {
            e.type = FX_KEY;
            e.width = 1;
        } else if (type >= FX_VEC_INT2) {
            e.type = uint8_t(FX_INT + (type - FX_VEC_INT2) % 3);
        } else {
            e.type = uint8_t(FX_INT + (type - FX_VEC_INT));
        }
        if (e.pos + e.parent_width > len) bad("flexbuffer element out of range");
        return e;
    }
    // map lookup (linear: maps here have a handful of keys)
    bool get(const char* key, Flex* out) const {
        if (type != FX_MAP) bad("flexbuffer value is not a map");
        const size_t t = target();
        if (t < 3 * size_t(width)) bad("flexbuffer map prefix out of range");
        const size_t kslot = t - 3 * size_t(width);
        const uint64_t koff = ru(kslot, width);
        if (koff > kslot) bad("flexbuffer map keys out of range");
        const size_t keys = kslot - size_t(koff);
        const int kw = int(ru(t - 2 * size_t(width), width));
        const uint64_t n = size();
        for (uint64_t i = 0; i < n; i++) {
            const size_t slot = keys + size_t(i) * kw;
            const uint64_t o = ru(slot, kw);
            if (o > slot) bad("flexbuffer key offset out of range");
            const size_t k = slot - size_t(o);
            size_t e = k;
            while (e < len && buf[e]) e++;
            if (e >= len) bad("flexbuffer key not terminated");
            if (e - k == std::strlen(key) && std::memcmp(buf + k, key, e - k) == 0) {
                *out = at(i);
                return true;
            }
        }
        return false;
    }
    Flex req(const char* key) const {
        Flex f;
        if (!get(key, &f)) bad(std::string("metadata field missing: ") + key);
        return f;
    }
};

// =========================================================================== dtypes
struct DType {
    enum Kind { Null, Bool, Prim, Utf8, Binary, Struct, List, Ext } kind = Null;
    int ptype = 0;
    bool nullable = false;
    std::vector<std::string> names;
    std::vector<DType> fields;
    std::string ext_id;
    std::vector<uint8_t> ext_meta;

    static DType prim(int p, bool n) { DType d; d.kind = Prim; d.ptype = p; d.nullable = n; return d; }
    DType with_nullable(bool n) const { DType d = *this; d.nullable = n; return d; }
    uint8_t vxg_dtype() const {
        switch (kind) {
        case Null: return VXG_DTYPE_NULL;
        case Bool: return VXG_DTYPE_BOOL;
        case Prim: return VXG_DTYPE_PRIMITIVE;
        case Utf8: return VXG_DTYPE_UTF8;
        case Binary: return VXG_DTYPE_BINARY;
        default: unsupported("struct/list/extension dtypes are not canonicalized by the engine");
        }
    }
};
const DType kBoolNN = [] { DType d; d.kind = DType::Bool; return d; }();  // Validity::DTYPE
const DType kBytes = DType::prim(VXG_U8, false);                          // DType::BYTES
const DType kIdx = DType::prim(VXG_U64, false);                           // DType::IDX

int unsigned_of(int p) {
    switch (p) {
    case VXG_I8: return VXG_U8;
    case VXG_I16: return VXG_U16;
    case VXG_I32: return VXG_U32;
    case VXG_I64: return VXG_U64;
    default: return p;
    }
}
bool is_signed_int(int p) { return p >= VXG_I8 && p <= VXG_I64; }
int ptype_width(int p) {
    static const int w[11] = {1, 2, 4, 8, 1, 2, 4, 8, 2, 4, 8};
    return p >= 0 && p < 11 ? w[p] : 0;
}

// dtype.fbs: DType {type_type, type}; union Type {Null=1, Bool, Primitive, Decimal, Utf8, Binary,
// Struct_, List, Extension}  (vortex-dtype/src/serde/flatbuffers/mod.rs:13-101)
DType parse_fb_dtype(const FbTable& t, int depth = 0) {
    if (depth > 64) bad("dtype nesting too deep");
    DType d;
    const uint8_t ty = t.get<uint8_t>(0, 0);
    FbTable v;
    const bool has = t.table(1, &v);
    if (!has && ty != 0) bad("DType union value missing");
    switch (ty) {
    case 1: d.kind = DType::Null; d.nullable = true; break;
    case 2: d.kind = DType::Bool; d.nullable = v.get<uint8_t>(0, 0) != 0; break;
    case 3: {
        d.kind = DType::Prim;
        d.ptype = v.get<uint8_t>(0, 0);
        if (d.ptype > VXG_F64) bad("unknown PType");
        d.nullable = v.get<uint8_t>(1, 0) != 0;
        break;
    }
    case 4: unsupported("Decimal dtype");
    case 5: d.kind = DType::Utf8; d.nullable = v.get<uint8_t>(0, 0) != 0; break;
    case 6: d.kind = DType::Binary; d.nullable = v.get<uint8_t>(0, 0) != 0; break;
    case 7: {
        d.kind = DType::Struct;
        uint32_t nn = 0, nd = 0;
        size_t dn = 0, dd = 0;
        if (!v.vector(0, 4, &nn, &dn)) bad("failed to parse struct names from flatbuffer");
        if (!v.vector(1, 4, &nd, &dd)) bad("failed to parse struct dtypes from flatbuffer");
        if (nn != nd) bad("struct names/dtypes length mismatch");
        for (uint32_t i = 0; i < nn; i++) {
            d.names.push_back(v.vec_string(dn, i));
            d.fields.push_back(parse_fb_dtype(v.vec_table(dd, i), depth + 1));
        }
        d.nullable = v.get<uint8_t>(2, 0) != 0;
        break;
    }
    case 8: {
        d.kind = DType::List;
        FbTable e;
        if (!v.table(0, &e)) bad("failed to parse list element type from flatbuffer");
        d.fields.push_back(parse_fb_dtype(e, depth + 1));
        d.nullable = v.get<uint8_t>(1, 0) != 0;
        break;
    }
    case 9: {
        d.kind = DType::Ext;
        if (!v.has(0)) bad("failed to parse extension id from flatbuffer");
        d.ext_id = v.string(0);
        uint32_t n;
        size_t p;
        if (v.vector(1, 1, &n, &p)) d.ext_meta.assign(v.buf + p, v.buf + p + n);
        d.nullable = v.get<uint8_t>(2, 0) != 0;
        break;
    }
    default: bad("Unknown DType variant");
    }
    return d;
}

int parse_ptype_name(const std::string& s) {  // PType serde: rename_all = "lowercase"
    static const char* n[11] = {"u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64", "f16", "f32", "f64"};
    for (int i = 0; i < 11; i++)
        if (s == n[i]) return i;
    bad("unknown PType '" + s + "'");
}

// serde DType (derive; ExtensionMetadata.storage_dtype, extension/mod.rs:19-21): unit variant
// -> string, newtype/tuple variants -> {"Variant": value | [values]}
DType parse_serde_dtype(const Flex& f) {
    DType d;
    if (f.type == FX_STRING || f.type == FX_KEY) {
        if (f.as_string() == "Null") { d.kind = DType::Null; d.nullable = true; return d; }
        bad("unknown DType variant");
    }
    if (f.type != FX_MAP || f.size() != 1) bad("DType must be a one-entry map");
    Flex v;
    if (f.get("Bool", &v)) { d.kind = DType::Bool; d.nullable = v.as_bool(); return d; }
    if (f.get("Utf8", &v)) { d.kind = DType::Utf8; d.nullable = v.as_bool(); return d; }
    if (f.get("Binary", &v)) { d.kind = DType::Binary; d.nullable = v.as_bool(); return d; }
    if (f.get("Primitive", &v)) {
        if (v.size() != 2) bad("Primitive dtype needs (ptype, nullability)");
        return DType::prim(parse_ptype_name(v.at(0).as_string()), v.at(1).as_bool());
    }
    unsupported("extension storage dtype other than Bool/Primitive/Utf8/Binary");
}

uint8_t parse_validity(const Flex& m) {  // ValidityMetadata, validity.rs:25-30
    const std::string s = m.req("validity").as_string();
    if (s == "NonNullable") return VXG_VALIDITY_NON_NULLABLE;
    if (s == "AllValid") return VXG_VALIDITY_ALL_VALID;
    if (s == "AllInvalid") return VXG_VALIDITY_ALL_INVALID;
    if (s == "Array") return VXG_VALIDITY_ARRAY;
    bad("unknown ValidityMetadata '" + s + "'");
}

// ScalarValue (vortex-scalar/src/serde/serde.rs) cast to `dt` (value.rs:14-16: primitive values
// may arrive narrower than the dtype; they are cast on read) -> LE bytes.  Returns is_null.
bool scalar_bytes(const Flex& v, const DType& dt, uint8_t out[16]) {
    std::memset(out, 0, 16);
    if (v.is_null()) return true;
    if (dt.kind == DType::Bool) {
        out[0] = v.as_bool() ? 1 : 0;
        return false;
    }
    if (dt.kind != DType::Prim) unsupported("non-primitive scalar values");
    const int p = dt.ptype;
    if (p == VXG_F32) {
        const float x = float(v.as_f64());
        std::memcpy(out, &x, 4);
    } else if (p == VXG_F64) {
        const double x = v.as_f64();
        std::memcpy(out, &x, 8);
    } else {
        // integers (and f16, whose PValue serializes as its u16 bits): two's complement bits
        uint64_t bits;
        if (v.type == FX_FLOAT || v.type == FX_IND_FLOAT) bits = uint64_t(int64_t(v.as_f64()));
        else if (v.type == FX_INT || v.type == FX_IND_INT) bits = uint64_t(v.as_i64());
        else bits = v.as_u64();
        std::memcpy(out, &bits, size_t(ptype_width(p)));
    }
    return false;
}

// =========================================================================== arrays
struct Pool {
    std::deque<std::unique_ptr<vxg_array[]>> nodes;
    std::deque<std::unique_ptr<vxg_buffer[]>> bufs;
    vxg_array* alloc_nodes(size_t n) {
        nodes.emplace_back(new vxg_array[n]());
        return nodes.back().get();
    }
    vxg_buffer* alloc_buf() {
        bufs.emplace_back(new vxg_buffer[1]());
        return bufs.back().get();
    }
};

struct BatchBuffers {
    std::vector<uint64_t> off, len;  // file offsets and lengths of the message's buffers
};

struct Builder {
    const uint8_t* file;      // host bytes (for values the reader must read: chunk offsets)
    uint64_t file_len;
    const BatchBuffers* bb;
    const uint8_t* region;    // caller's copy of the file bytes
    uint64_t region_off;
    uint64_t region_len;
    Pool* pool;

    Flex meta(const FbTable& a, bool required) const {
        uint32_t n;
        size_t p;
        if (!a.vector(3, 1, &n, &p)) {
            if (required) bad("Array requires metadata bytes");
            return Flex{};
        }
        return Flex::root(a.buf + p, n);
    }

    void set_buffer(const FbTable& a, vxg_array& o) const {
        if (!a.has(1)) return;  // buffer_index = null
        const uint64_t i = a.get<uint64_t>(1, 0);
        if (i >= bb->off.size()) bad("buffer_index out of range");
        // every buffer must lie inside the caller's region (chunk messages of a malformed file
        // need not be in ascending, non-overlapping order)
        if (bb->off[i] < region_off || bb->len[i] > region_len || bb->off[i] - region_off > region_len - bb->len[i])
            bad("buffer lies outside the region copied to the device");
        vxg_buffer* b = pool->alloc_buf();
        b->ptr = reinterpret_cast<const void*>(reinterpret_cast<uintptr_t>(region) + uintptr_t(bb->off[i] - region_off));
        b->len = bb->len[i];
        o.buffers = b;
        o.n_buffers = 1;
    }

    // children of `a` with the (dtype, len) the parent's accessors give them
    struct Kid { DType dt; uint64_t len; };
    void children(const FbTable& a, const std::vector<Kid>& kids, vxg_array& o, int depth) const {
        uint32_t n = 0;
        size_t d = 0;
        a.vector(5, 4, &n, &d);
        if (n != kids.size())
            bad("encoding " + std::to_string(o.encoding) + " expects " + std::to_string(kids.size()) +
                " children, the message holds " + std::to_string(n));
        if (!n) return;
        vxg_array* c = pool->alloc_nodes(n);
        for (uint32_t i = 0; i < n; i++) build(a.vec_table(d, i), kids[i].dt, kids[i].len, c[i], depth + 1);
        o.children = c;
        o.n_children = n;
    }

    uint64_t host_u64(const vxg_array& prim, uint64_t i) const {
        if (prim.encoding != VXG_ENC_PRIMITIVE || prim.n_buffers != 1 || prim.ptype != VXG_U64)
            unsupported("chunk_offsets must be a canonical u64 PrimitiveArray");
        const uint64_t fo =
            uint64_t(reinterpret_cast<uintptr_t>(prim.buffers[0].ptr) - reinterpret_cast<uintptr_t>(region)) + region_off;
        if ((i + 1) * 8 > prim.buffers[0].len || fo + (i + 1) * 8 > file_len) bad("chunk_offsets out of range");
        uint64_t v;
        std::memcpy(&v, file + fo + i * 8, 8);
        return v;
    }

    void build(const FbTable& a, const DType& dt, uint64_t len, vxg_array& o, int depth) const {
        if (depth > 64) bad("array nesting too deep");
        const uint16_t enc = a.get<uint16_t>(2, 0);
        if (dt.kind == DType::Ext) {  // ExtensionArray: its storage (extension/mod.rs:41-46)
            if (enc != 7) unsupported("extension dtype with encoding " + std::to_string(enc));
            const DType storage = parse_serde_dtype(meta(a, true).req("storage_dtype"));
            uint32_t n = 0;
            size_t d = 0;
            a.vector(5, 4, &n, &d);
            if (n != 1) bad("ExtensionArray must have one storage child");
            build(a.vec_table(d, 0), storage, len, o, depth + 1);
            return;
        }
        std::memset(&o, 0, sizeof(o));
        o.encoding = enc;
        o.dtype = dt.vxg_dtype();
        o.ptype = uint8_t(dt.kind == DType::Prim ? dt.ptype : VXG_U8);
        o.nullable = dt.nullable;
        o.len = len;
        set_buffer(a, o);
        const DType validity_dt = kBoolNN;
        auto need_prim = [&](const char* what) {
            if (dt.kind != DType::Prim) bad(std::string(what) + " requires a primitive dtype");
        };
        switch (enc) {
        case VXG_ENC_PRIMITIVE: {  // array/primitive/mod.rs:33-35, 93-101
            const Flex m = meta(a, true);
            o.validity = parse_validity(m);
            std::vector<Kid> k;
            if (o.validity == VXG_VALIDITY_ARRAY) k.push_back({validity_dt, len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_BOOL: {  // array/bool/mod.rs:25-56
            const Flex m = meta(a, true);
            o.validity = parse_validity(m);
            o.meta.boolean.first_byte_bit_offset = uint8_t(m.req("first_byte_bit_offset").as_u64());
            std::vector<Kid> k;
            if (o.validity == VXG_VALIDITY_ARRAY) k.push_back({validity_dt, len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_BYTE_BOOL: {  // encodings/bytebool/src/array.rs:20-36
            const Flex m = meta(a, true);
            o.validity = parse_validity(m);
            std::vector<Kid> k;
            if (o.validity == VXG_VALIDITY_ARRAY) k.push_back({validity_dt, len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_VARBIN: {  // array/varbin/mod.rs:35-39, 87-125
            const Flex m = meta(a, true);
            o.validity = parse_validity(m);
            const int op = parse_ptype_name(m.req("offsets_ptype").as_string());
            const uint64_t bl = m.req("bytes_len").as_u64();
            o.meta.varbin.offsets_ptype = uint8_t(op);
            o.meta.varbin.bytes_len = bl;
            std::vector<Kid> k = {{DType::prim(op, false), len + 1}, {kBytes, bl}};
            if (o.validity == VXG_VALIDITY_ARRAY) k.push_back({validity_dt, len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_VARBINVIEW: {  // array/varbinview/mod.rs:179-186, 303-360
            const Flex m = meta(a, true);
            o.validity = parse_validity(m);
            const Flex bl = m.req("buffer_lens");
            const uint64_t nb = bl.size();
            o.meta.varbinview.n_buffers = uint32_t(nb);
            std::vector<Kid> k = {{kBytes, len * 16}};
            for (uint64_t i = 0; i < nb; i++) k.push_back({kBytes, bl.at(i).as_u64()});
            if (o.validity == VXG_VALIDITY_ARRAY) k.push_back({validity_dt, len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_SPARSE: {  // array/sparse/mod.rs:24-29, 96-110
            const Flex m = meta(a, true);
            const uint64_t il = m.req("indices_len").as_u64();
            o.meta.sparse.indices_offset = m.req("indices_offset").as_u64();
            o.meta.sparse.indices_len = il;
            o.meta.sparse.fill_is_null = scalar_bytes(m.req("fill_value"), dt, o.meta.sparse.fill);
            children(a, {{kIdx, il}, {dt, il}}, o, depth);
            break;
        }
        case VXG_ENC_CONSTANT: {  // array/constant/mod.rs:21-24
            const Flex m = meta(a, true);
            o.meta.constant.is_null = scalar_bytes(m.req("scalar_value"), dt, o.meta.constant.scalar);
            children(a, {}, o, depth);
            break;
        }
        case VXG_ENC_CHUNKED: {  // array/chunked/mod.rs:34-36, 82-104
            const Flex m = meta(a, true);
            const uint64_t nc = m.req("nchunks").as_u64();
            o.meta.chunked.nchunks = nc;
            uint32_t n = 0;
            size_t d = 0;
            a.vector(5, 4, &n, &d);
            if (n != nc + 1) bad("ChunkedArray child count != nchunks + 1");
            vxg_array* c = pool->alloc_nodes(n);
            build(a.vec_table(d, 0), kIdx, nc + 1, c[0], depth + 1);
            for (uint64_t i = 0; i < nc; i++) {
                const uint64_t s = host_u64(c[0], i), e = host_u64(c[0], i + 1);
                if (e < s) bad("chunk offsets not ascending");
                build(a.vec_table(d, uint32_t(i + 1)), dt, e - s, c[i + 1], depth + 1);
            }
            o.children = c;
            o.n_children = n;
            break;
        }
        case VXG_ENC_ALP: {  // encodings/alp/src/alp/array.rs:19-24, 86-129
            need_prim("ALP");
            const Flex m = meta(a, true);
            const Flex ex = m.req("exponents");
            o.meta.alp.e = uint8_t(ex.req("e").as_u64());
            o.meta.alp.f = uint8_t(ex.req("f").as_u64());
            const int ep = dt.ptype == VXG_F32 ? VXG_I32 : dt.ptype == VXG_F64 ? VXG_I64 : -1;
            if (ep < 0) bad("ALP dtype must be f32 or f64");
            uint32_t n = 0;
            size_t d = 0;
            a.vector(5, 4, &n, &d);
            o.meta.alp.has_patches = n > 1;
            std::vector<Kid> k = {{DType::prim(ep, dt.nullable), len}};
            if (n > 1) k.push_back({dt.with_nullable(true), len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_ALP_RD: {  // encodings/alp/src/alp_rd/array.rs:15-24, 115-166
            need_prim("ALPRD");
            const Flex m = meta(a, true);
            o.meta.alprd.right_bit_width = uint8_t(m.req("right_bit_width").as_u64());
            o.meta.alprd.dict_len = uint8_t(m.req("dict_len").as_u64());
            const Flex dict = m.req("dict");
            if (dict.size() != 8) bad("ALPRD dict must hold 8 entries");
            for (int i = 0; i < 8; i++) o.meta.alprd.dict[i] = uint16_t(dict.at(i).as_u64());
            const int lp = parse_ptype_name(m.req("left_parts_ptype").as_string());
            o.meta.alprd.left_parts_ptype = uint8_t(lp);
            const bool exc = m.req("has_exceptions").as_bool();
            o.meta.alprd.has_exceptions = exc;
            std::vector<Kid> k = {{DType::prim(lp, dt.nullable), len},
                                  {DType::prim(dt.ptype == VXG_F32 ? VXG_U32 : VXG_U64, false), len}};
            if (exc) k.push_back({DType::prim(lp, true), len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_DICT: {  // encodings/dict/src/array.rs:21-25, 50-64
            const Flex m = meta(a, true);
            const int cp = parse_ptype_name(m.req("codes_ptype").as_string());
            const uint64_t vl = m.req("values_len").as_u64();
            o.meta.dict.codes_ptype = uint8_t(cp);
            o.meta.dict.values_len = vl;
            children(a, {{dt, vl}, {DType::prim(cp, false), len}}, o, depth);
            break;
        }
        case VXG_ENC_FL_BITPACKED: {  // encodings/fastlanes/src/bitpacking/mod.rs:24-30, 158-187
            need_prim("BitPacked");
            const Flex m = meta(a, true);
            o.validity = parse_validity(m);
            o.meta.bitpacked.bit_width = uint8_t(m.req("bit_width").as_u64());
            o.meta.bitpacked.offset = uint16_t(m.req("offset").as_u64());
            const bool hp = m.req("has_patches").as_bool();
            o.meta.bitpacked.has_patches = hp;
            std::vector<Kid> k;
            if (hp) k.push_back({dt.with_nullable(true), len});
            if (o.validity == VXG_VALIDITY_ARRAY) k.push_back({validity_dt, len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_FL_DELTA: {  // encodings/fastlanes/src/delta/mod.rs:20-25, 159-205
            need_prim("Delta");
            const Flex m = meta(a, true);
            o.validity = parse_validity(m);
            const uint64_t dl = m.req("deltas_len").as_u64();
            o.meta.delta.deltas_len = dl;
            o.meta.delta.offset = uint16_t(m.req("offset").as_u64());
            const uint64_t lanes = 1024 / (8 * uint64_t(ptype_width(dt.ptype)));
            const uint64_t bases = (dl / 1024) * lanes + (dl % 1024 ? 1 : 0);
            std::vector<Kid> k = {{dt, bases}, {dt, dl}};
            if (o.validity == VXG_VALIDITY_ARRAY) k.push_back({validity_dt, len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_FL_FOR: {  // encodings/fastlanes/src/for/mod.rs:20-24, 56-66
            need_prim("FoR");
            const Flex m = meta(a, true);
            uint8_t ref[16];
            if (scalar_bytes(m.req("reference"), dt, ref)) bad("FoR reference must not be null");
            std::memcpy(&o.meta.for_.reference, ref, 8);
            o.meta.for_.shift = uint8_t(m.req("shift").as_u64());
            const DType enc_dt = is_signed_int(dt.ptype) ? DType::prim(unsigned_of(dt.ptype), dt.nullable) : dt;
            children(a, {{enc_dt, len}}, o, depth);
            break;
        }
        case VXG_ENC_FSST: {  // encodings/fsst/src/array.rs:21-26, 107-148
            const Flex m = meta(a, true);
            const uint64_t sl = m.req("symbols_len").as_u64();
            const bool cn = m.req("codes_nullability").as_bool();
            const int up = parse_ptype_name(m.req("uncompressed_lengths_ptype").as_string());
            o.meta.fsst.symbols_len = sl;
            o.meta.fsst.codes_nullable = cn;
            o.meta.fsst.uncompressed_lengths_ptype = uint8_t(up);
            DType codes;
            codes.kind = DType::Binary;
            codes.nullable = cn;
            children(a, {{DType::prim(VXG_U64, false), sl}, {kBytes, sl}, {codes, len}, {DType::prim(up, false), len}},
                     o, depth);
            break;
        }
        case VXG_ENC_RUN_END: {  // encodings/runend/src/array.rs:24-29, 127-170
            const Flex m = meta(a, true);
            o.validity = parse_validity(m);
            const int ep = parse_ptype_name(m.req("ends_ptype").as_string());
            const uint64_t nr = m.req("num_runs").as_u64();
            o.meta.runend.ends_ptype = uint8_t(ep);
            o.meta.runend.num_runs = nr;
            o.meta.runend.offset = m.req("offset").as_u64();
            std::vector<Kid> k = {{DType::prim(ep, false), nr}, {dt, nr}};
            if (o.validity == VXG_VALIDITY_ARRAY) k.push_back({validity_dt, len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_RUN_END_BOOL: {  // encodings/runend-bool/src/array.rs:21-28, 96-112
            const Flex m = meta(a, true);
            o.validity = parse_validity(m);
            const int ep = parse_ptype_name(m.req("ends_ptype").as_string());
            const uint64_t nr = m.req("num_runs").as_u64();
            o.meta.runendbool.start = m.req("start").as_bool();
            o.meta.runendbool.ends_ptype = uint8_t(ep);
            o.meta.runendbool.num_runs = nr;
            o.meta.runendbool.offset = m.req("offset").as_u64();
            std::vector<Kid> k = {{DType::prim(ep, false), nr}};
            if (o.validity == VXG_VALIDITY_ARRAY) k.push_back({validity_dt, len});
            children(a, k, o, depth);
            break;
        }
        case VXG_ENC_ZIGZAG: {  // encodings/zigzag/src/array.rs:25, 56-64 (unit metadata)
            need_prim("ZigZag");
            children(a, {{DType::prim(unsigned_of(dt.ptype), dt.nullable), len}}, o, depth);
            break;
        }
        case VXG_ENC_ROARING_BOOL: {  // encodings/roaring/src/boolean/mod.rs:25-67 (unit metadata,
                                      // one buffer: croaring Native bytes, no children)
            if (dt.kind != DType::Bool) bad("RoaringBool must have a Bool dtype");
            children(a, {}, o, depth);
            break;
        }
        default:
            unsupported("no reader for encoding id " + std::to_string(enc));
        }
    }
};

// =========================================================================== file
constexpr uint16_t kVersion = 1;            // layouts/mod.rs:8
constexpr size_t kPostscript = 32;          // layouts/mod.rs:11
constexpr size_t kEof = 8;                  // layouts/mod.rs:12
enum : uint16_t { kFlat = 1, kChunkedLayout = 2, kColumnLayout = 3, kInlineSchema = 4 };

struct Chunk {
    uint64_t row_offset = 0, rows = 0, begin = 0, end = 0, fb_begin = 0, fb_len = 0, buffers_begin = 0;
};
struct Column {
    std::string name;
    DType dtype;
    std::vector<Chunk> chunks;
    uint64_t rows = 0;
};

}  // namespace

struct vxg_file {
    const uint8_t* bytes = nullptr;
    uint64_t len = 0;
    uint64_t row_count = 0;
    DType schema;
    std::vector<Column> cols;
    std::mutex mu;
    Pool pool;
};

namespace {

// length-prefixed flatbuffer message at [begin, end): returns (fb position, fb length)
void message_at(const vxg_file& f, uint64_t begin, uint64_t end, uint64_t* fb, uint64_t* fb_len) {
    if (begin > end || end > f.len || end - begin < 4) bad("message range out of the file");
    const uint32_t n = rd<uint32_t>(f.bytes, f.len, begin);
    if (n == 0) bad("Invalid IPC stream");
    if (uint64_t(n) > end - begin - 4) bad("message longer than its range");
    *fb = begin + 4;
    *fb_len = n;
}

FbTable message_header(const vxg_file& f, uint64_t fb, uint64_t fb_len, uint8_t want, const char* what) {
    const FbTable msg = FbTable::root(f.bytes + fb, fb_len);
    if (msg.get<uint8_t>(0, 0) != 0) bad("unsupported message version");
    if (msg.get<uint8_t>(1, 0) != want) bad(std::string("message is not a ") + what);
    FbTable h;
    if (!msg.table(2, &h)) bad(std::string(what) + " message without header");
    return h;
}

DType read_schema(const vxg_file& f, uint64_t begin, uint64_t end) {
    uint64_t fb, n;
    message_at(f, begin, end, &fb, &n);
    const FbTable schema = message_header(f, fb, n, 1, "schema");
    FbTable dt;
    if (!schema.table(0, &dt)) bad("Schema missing DType");
    return parse_fb_dtype(dt);
}

// Batch message: chunk geometry + the buffer split of ArrayBufferReader::read
Chunk read_batch_geometry(const vxg_file& f, uint64_t begin, uint64_t end, FbTable* batch_out,
                          BatchBuffers* bb) {
    Chunk c;
    c.begin = begin;
    c.end = end;
    message_at(f, begin, end, &c.fb_begin, &c.fb_len);
    const FbTable batch = message_header(f, c.fb_begin, c.fb_len, 2, "batch");
    c.rows = batch.get<uint64_t>(1, 0);
    c.buffers_begin = c.fb_begin + c.fb_len;
    const uint64_t total = batch.get<uint64_t>(3, 0);
    if (total > end - c.buffers_begin) bad("batch buffers run past the message");
    if (bb) {
        uint32_t nb = 0;
        size_t d = 0;
        batch.vector(2, 16, &nb, &d);
        uint64_t cursor = 0;
        for (uint32_t i = 0; i < nb; i++) {
            const uint64_t off = rd<uint64_t>(batch.buf, batch.len, d + 16 * i);
            const uint16_t pad = rd<uint16_t>(batch.buf, batch.len, d + 16 * i + 8);
            const uint8_t comp = rd<uint8_t>(batch.buf, batch.len, d + 16 * i + 10);
            if (comp != 0) unsupported("compressed IPC buffers");
            const uint64_t next = i + 1 < nb ? rd<uint64_t>(batch.buf, batch.len, d + 16 * (i + 1)) : total;
            if (next < off + pad) bad("IPC buffer offsets not ascending");
            const uint64_t bl = next - off - pad;
            if (cursor + bl + pad > total) bad("IPC buffer out of range");
            bb->off.push_back(c.buffers_begin + cursor);
            bb->len.push_back(bl);
            cursor += bl + pad;
        }
    }
    if (batch_out) *batch_out = batch;
    return c;
}

// the metadata table of a column's chunked layout: Struct{row_offset: u64} (writer.rs:120-157)
std::vector<uint64_t> read_row_offsets(const vxg_file& f, const FbTable& layout) {
    if (layout.get<uint16_t>(0, 0) != kInlineSchema) unsupported("chunked layout metadata is not an inline-schema layout");
    uint32_t nb = 0, nc = 0;
    size_t db = 0, dc = 0;
    if (!layout.vector(1, 16, &nb, &db) || nb < 1) bad("inline-schema layout without its dtype buffer");
    if (!layout.vector(2, 4, &nc, &dc) || nc < 1) bad("inline-schema layout without children");
    const DType dt = read_schema(f, rd<uint64_t>(layout.buf, layout.len, db), rd<uint64_t>(layout.buf, layout.len, db + 8));
    if (dt.kind != DType::Struct || dt.fields.size() != 1 || dt.names[0] != "row_offset" ||
        dt.fields[0].kind != DType::Prim || dt.fields[0].ptype != VXG_U64)
        unsupported("column metadata table is not Struct{row_offset: u64}");
    const FbTable flat = layout.vec_table(dc, 0);
    uint32_t fbn = 0;
    size_t fbd = 0;
    if (flat.get<uint16_t>(0, 0) != kFlat || !flat.vector(1, 16, &fbn, &fbd) || fbn < 1) bad("metadata table is not a flat layout");
    FbTable batch;
    BatchBuffers bb;
    const Chunk c = read_batch_geometry(f, rd<uint64_t>(flat.buf, flat.len, fbd), rd<uint64_t>(flat.buf, flat.len, fbd + 8),
                                        &batch, &bb);
    FbTable arr;
    if (!batch.table(0, &arr)) bad("Chunk missing Array");
    if (arr.get<uint16_t>(2, 0) != VXG_ENC_STRUCT) unsupported("metadata table array is not a StructArray");
    uint32_t nk = 0;
    size_t dk = 0;
    if (!arr.vector(5, 4, &nk, &dk) || nk < 1) bad("metadata StructArray without its field");
    const FbTable field = arr.vec_table(dk, 0);
    if (field.get<uint16_t>(2, 0) != VXG_ENC_PRIMITIVE || !field.has(1)) unsupported("row_offset is not a canonical PrimitiveArray");
    const uint64_t bi = field.get<uint64_t>(1, 0);
    if (bi >= bb.off.size() || bb.len[bi] < c.rows * 8) bad("row_offset buffer out of range");
    std::vector<uint64_t> out(c.rows);
    if (c.rows) std::memcpy(out.data(), f.bytes + bb.off[bi], c.rows * 8);
    return out;
}

void read_column(vxg_file& f, const FbTable& layout, Column& col) {
    const uint16_t id = layout.get<uint16_t>(0, 0);
    std::vector<FbTable> flats;
    std::vector<uint64_t> row_offsets;
    bool have_offsets = false;
    if (id == kFlat) {
        flats.push_back(layout);
    } else if (id == kChunkedLayout) {
        uint32_t mn = 0, nc = 0;
        size_t md = 0, dc = 0;
        const bool has_meta = layout.vector(3, 1, &mn, &md) && mn >= 1 && layout.buf[md] != 0;  // chunked.rs:78-83
        if (!layout.vector(2, 4, &nc, &dc)) bad("Missing children");
        for (uint32_t i = 0; i < nc; i++) {
            const FbTable c = layout.vec_table(dc, i);
            if (i == 0 && has_meta) {
                row_offsets = read_row_offsets(f, c);
                have_offsets = true;
                continue;
            }
            if (c.get<uint16_t>(0, 0) != kFlat) unsupported("nested layouts other than flat chunks");
            flats.push_back(c);
        }
    } else {
        unsupported("column layout id " + std::to_string(id));
    }
    if (have_offsets && row_offsets.size() != flats.size()) bad("row_offset table length != chunk count");
    uint64_t row = 0;
    for (size_t i = 0; i < flats.size(); i++) {
        uint32_t nb = 0;
        size_t db = 0;
        if (!flats[i].vector(1, 16, &nb, &db) || nb < 1) bad("No buffers");  // flat.rs:38-42
        Chunk c = read_batch_geometry(f, rd<uint64_t>(flats[i].buf, flats[i].len, db),
                                      rd<uint64_t>(flats[i].buf, flats[i].len, db + 8), nullptr, nullptr);
        if (have_offsets && row_offsets[i] != row) bad("row_offset table disagrees with the chunk lengths");
        c.row_offset = row;
        row += c.rows;
        col.chunks.push_back(c);
    }
    col.rows = row;
}

void open_file(vxg_file& f) {
    // read/footer.rs:140-187
    if (f.len < kEof + kPostscript) bad("Malformed vortex file, size " + std::to_string(f.len) + " too small");
    const uint64_t eof = f.len - kEof;
    if (std::memcmp(f.bytes + f.len - 4, "VRTX", 4) != 0) bad("Malformed file, invalid magic bytes");
    const uint16_t version = rd<uint16_t>(f.bytes, f.len, eof);
    if (version != kVersion) bad("Malformed file, unsupported version " + std::to_string(version));
    const FbTable ps = FbTable::root(f.bytes + eof - kPostscript, kPostscript);
    const uint64_t schema_off = ps.get<uint64_t>(0, 0), footer_off = ps.get<uint64_t>(1, 0);
    if (schema_off >= footer_off || footer_off >= eof - kPostscript) bad("postscript offsets out of range");
    f.schema = read_schema(f, schema_off, footer_off);
    // the footer: a length-prefixed flatbuffer whose root is Footer (writer.rs:159-172)
    uint64_t fb, n;
    message_at(f, footer_off, eof - kPostscript, &fb, &n);
    const FbTable footer = FbTable::root(f.bytes + fb, eof - kPostscript - fb);
    FbTable top;
    if (!footer.table(0, &top)) bad("Footer must contain a layout");
    f.row_count = footer.get<uint64_t>(1, 0);
    if (f.schema.kind != DType::Struct) unsupported("file schema is not a struct");
    if (top.get<uint16_t>(0, 0) != kColumnLayout) unsupported("top-level layout is not a column layout");
    uint32_t nc = 0;
    size_t dc = 0;
    if (!top.vector(2, 4, &nc, &dc)) bad("Missing children");
    if (nc != f.schema.fields.size()) bad("column layout children != schema fields");
    f.cols.resize(nc);
    for (uint32_t i = 0; i < nc; i++) {
        f.cols[i].name = f.schema.names[i];
        f.cols[i].dtype = f.schema.fields[i];
        read_column(f, top.vec_table(dc, i), f.cols[i]);
        if (f.cols[i].rows != f.row_count) bad("column '" + f.cols[i].name + "' row count != footer row_count");
    }
}

vxg_status guard(const char* what, auto&& fn) {
    try {
        fn();
        return VXG_OK;
    } catch (const SerdeError& e) {
        return vxg::set_error(e.st, std::string(what) + ": " + e.what());
    } catch (const std::bad_alloc&) {
        return vxg::set_error(VXG_ERR_OUT_OF_MEMORY, std::string(what) + ": out of host memory");
    } catch (const std::exception& e) {
        return vxg::set_error(VXG_ERR_INVALID_SERDE, std::string(what) + ": " + e.what());
    }
}

}  // namespace

extern "C" {

vxg_status vxg_file_open(const void* bytes, uint64_t len, vxg_file** out) {
    if (!bytes || !out) return vxg::set_error(VXG_ERR_INVALID_ARGUMENT, "vxg_file_open: null argument");
    *out = nullptr;
    auto f = std::make_unique<vxg_file>();
    f->bytes = static_cast<const uint8_t*>(bytes);
    f->len = len;
    const vxg_status st = guard("vxg_file_open", [&] { open_file(*f); });
    if (st == VXG_OK) *out = f.release();
    return st;
}

vxg_status vxg_file_close(vxg_file* file) {
    delete file;
    return VXG_OK;
}

vxg_status vxg_file_info(const vxg_file* file, uint64_t* row_count, uint32_t* n_columns) {
    if (!file) return vxg::set_error(VXG_ERR_INVALID_ARGUMENT, "null vxg_file");
    if (row_count) *row_count = file->row_count;
    if (n_columns) *n_columns = uint32_t(file->cols.size());
    return VXG_OK;
}

vxg_status vxg_file_column_info(const vxg_file* file, uint32_t column, vxg_file_column* out) {
    if (!file || !out) return vxg::set_error(VXG_ERR_INVALID_ARGUMENT, "null argument");
    if (column >= file->cols.size()) return vxg::set_error(VXG_ERR_OUT_OF_BOUNDS, "column index out of range");
    const Column& c = file->cols[column];
    std::memset(out, 0, sizeof(*out));
    out->name = c.name.c_str();
    out->n_chunks = uint32_t(c.chunks.size());
    out->rows = c.rows;
    out->nullable = c.dtype.nullable;
    const DType* st = &c.dtype;
    DType storage;
    if (c.dtype.kind == DType::Ext) {
        out->is_extension = 1;
        out->extension_id = c.dtype.ext_id.c_str();
        out->extension_metadata = c.dtype.ext_meta.data();
        out->extension_metadata_len = c.dtype.ext_meta.size();
        // the storage dtype is in each chunk's ExtensionMetadata; report the first chunk's
        if (!c.chunks.empty()) {
            const vxg_status s = guard("vxg_file_column_info", [&] {
                FbTable batch;
                read_batch_geometry(*file, c.chunks[0].begin, c.chunks[0].end, &batch, nullptr);
                FbTable arr;
                if (!batch.table(0, &arr)) bad("Chunk missing Array");
                uint32_t n;
                size_t p;
                if (!arr.vector(3, 1, &n, &p)) bad("Array requires metadata bytes");
                storage = parse_serde_dtype(Flex::root(arr.buf + p, n).req("storage_dtype"));
            });
            if (s != VXG_OK) return s;
            st = &storage;
        }
    }
    if (st->kind == DType::Struct || st->kind == DType::List || st->kind == DType::Ext)
        out->dtype = 0xff;
    else
        out->dtype = st->vxg_dtype();
    out->ptype = uint8_t(st->kind == DType::Prim ? st->ptype : VXG_U8);
    return VXG_OK;
}

vxg_status vxg_file_chunk_info(const vxg_file* file, uint32_t column, uint32_t chunk, vxg_file_chunk* out) {
    if (!file || !out) return vxg::set_error(VXG_ERR_INVALID_ARGUMENT, "null argument");
    if (column >= file->cols.size() || chunk >= file->cols[column].chunks.size())
        return vxg::set_error(VXG_ERR_OUT_OF_BOUNDS, "column/chunk index out of range");
    const Chunk& c = file->cols[column].chunks[chunk];
    out->row_offset = c.row_offset;
    out->rows = c.rows;
    out->message_begin = c.begin;
    out->message_end = c.end;
    out->buffers_begin = c.buffers_begin;
    return VXG_OK;
}

vxg_status vxg_file_chunk_offsets(const vxg_file* file, uint32_t column, uint32_t chunk_begin, uint32_t chunk_end,
                                  uint64_t* host_out) {
    if (!file || !host_out) return vxg::set_error(VXG_ERR_INVALID_ARGUMENT, "null argument");
    if (column >= file->cols.size() || chunk_begin > chunk_end || chunk_end > file->cols[column].chunks.size())
        return vxg::set_error(VXG_ERR_OUT_OF_BOUNDS, "column/chunk range out of range");
    const auto& ch = file->cols[column].chunks;
    uint64_t acc = 0;
    host_out[0] = 0;
    for (uint32_t i = chunk_begin; i < chunk_end; i++) {
        acc += ch[i].rows;
        host_out[i - chunk_begin + 1] = acc;
    }
    return VXG_OK;
}

vxg_status vxg_file_column_array(vxg_file* file, uint32_t column, uint32_t chunk_begin, uint32_t chunk_end,
                                 const void* region, uint64_t region_file_offset, uint64_t region_len,
                                 const void* chunk_offsets_dev, const vxg_array** out) {
    if (!file || !out) return vxg::set_error(VXG_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (column >= file->cols.size() || chunk_begin >= chunk_end || chunk_end > file->cols[column].chunks.size())
        return vxg::set_error(VXG_ERR_OUT_OF_BOUNDS, "column/chunk range out of range");
    const Column& col = file->cols[column];
    if (col.chunks[chunk_begin].begin < region_file_offset ||
        col.chunks[chunk_end - 1].end > region_file_offset + region_len)
        return vxg::set_error(VXG_ERR_INVALID_ARGUMENT, "region does not cover the chunks' messages");
    std::lock_guard<std::mutex> lock(file->mu);
    return guard("vxg_file_column_array", [&] {
        const uint32_t n = chunk_end - chunk_begin;
        vxg_array* root = file->pool.alloc_nodes(1);
        vxg_array* kids = file->pool.alloc_nodes(n + 1);
        // child 0: chunk_offsets (u64, n + 1), a device copy supplied by the caller (or none)
        const DType& dt = col.dtype;
        vxg_array& co = kids[0];
        co.encoding = VXG_ENC_PRIMITIVE;
        co.dtype = VXG_DTYPE_PRIMITIVE;
        co.ptype = VXG_U64;
        co.len = n + 1;
        co.validity = VXG_VALIDITY_NON_NULLABLE;
        if (chunk_offsets_dev) {
            vxg_buffer* b = file->pool.alloc_buf();
            b->ptr = chunk_offsets_dev;
            b->len = uint64_t(n + 1) * 8;
            co.buffers = b;
            co.n_buffers = 1;
        }
        for (uint32_t i = 0; i < n; i++) {
            const Chunk& c = col.chunks[chunk_begin + i];
            FbTable batch;
            BatchBuffers bb;
            read_batch_geometry(*file, c.begin, c.end, &batch, &bb);
            FbTable arr;
            if (!batch.table(0, &arr)) bad("Chunk missing Array");
            if (c.begin < region_file_offset || c.end > region_file_offset + region_len)
                bad("region does not cover chunk " + std::to_string(chunk_begin + i) + "'s message");
            Builder b{file->bytes, file->len, &bb, static_cast<const uint8_t*>(region), region_file_offset, region_len,
                      &file->pool};
            b.build(arr, dt, c.rows, kids[i + 1], 0);
        }
        vxg_array& r = root[0];
        r.encoding = VXG_ENC_CHUNKED;
        r.dtype = kids[1].dtype;
        r.ptype = kids[1].ptype;
        r.nullable = kids[1].nullable;
        r.validity = VXG_VALIDITY_NON_NULLABLE;
        r.len = 0;
        for (uint32_t i = 0; i < n; i++) r.len += kids[i + 1].len;
        r.meta.chunked.nchunks = n;
        r.children = kids;
        r.n_children = n + 1;
        *out = root;
    });
}

}  // extern "C"
