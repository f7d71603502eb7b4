"""Vortex file WRITER (input generation for tests and bench.py; not the product path).

The reference writes files with vortex-serde's LayoutWriter (layouts/write/writer.rs:40-201):
every column's chunks as IPC Batch messages (MessageWriter::write_batch, message_writer.rs:51-73;
IPCBatch/IPCArray, messages.rs:63-163), then per column a Schema message + a Batch holding the
Struct{row_offset: u64} metadata table, then the file Schema message, the Footer (a
length-prefixed flatbuffer, footer.rs:18-34), the raw 32-byte Postscript and the 8-byte EOF
(version u16 = 1, 2 zero bytes, "VRTX"; layouts/mod.rs:8-16).  Every message and buffer is padded
to 64 bytes (lib.rs:15).  This module restates that layout byte for byte in Python, with a small
flatbuffers builder (back-to-front, vtables, u32 forward offsets: the flatbuffers wire format of
vortex-flatbuffers/flatbuffers/*.fbs) and a flexbuffers builder following the reference
implementation's layout rules (FlexbufferSerializer: serde structs -> maps with sorted keys, unit
enum variants -> strings; metadata.rs:35-47).  Neither library exists in this image.

The engine's reader (vortex_amd/csrc/serde.cpp, include/vortex_file.h) is what parses these
files; the tests check it against the trees written here and the decode against the oracle.
No reference-generated file exists to pin the bytes (the reference cannot be built here), so
byte-level parity of this writer with the Rust LayoutWriter is unpinned; the reader is a generic
flatbuffers/flexbuffers decoder, so it does not depend on this writer's particular choices.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from vortex_amd._lib import DTYPE, ENC, PTYPES, VALIDITY
from vortex_amd.arrays import Array

ALIGNMENT = 64                 # vortex-serde/src/lib.rs:15
VERSION = 1                    # layouts/mod.rs:8
MAGIC = b"VRTX"                # layouts/mod.rs:9
FLAT, CHUNKED_LAYOUT, COLUMN, INLINE_SCHEMA = 1, 2, 3, 4   # layouts/mod.rs:13-16
ENC_STRUCT, ENC_EXTENSION = 4, 7                           # encoding/mod.rs:115-118


def _align(n: int, a: int = ALIGNMENT) -> int:
    return (n + a - 1) & ~(a - 1)


# ============================================================================ flexbuffers
FX_NULL, FX_INT, FX_UINT, FX_FLOAT, FX_KEY, FX_STRING = 0, 1, 2, 3, 4, 5
FX_MAP, FX_VECTOR, FX_VEC_KEY, FX_BOOL = 9, 10, 14, 26
_INLINE = {FX_NULL, FX_INT, FX_UINT, FX_FLOAT, FX_BOOL}
TYPED_VECTORS = True  # homogeneous scalar vectors as typed vectors (reference builder behaviour)
_WCODE = {1: 0, 2: 1, 4: 2, 8: 3}


def _uwidth(u: int) -> int:
    return 1 if u < 1 << 8 else 2 if u < 1 << 16 else 4 if u < 1 << 32 else 8


def _iwidth(i: int) -> int:
    for w in (1, 2, 4):
        if -(1 << (8 * w - 1)) <= i < (1 << (8 * w - 1)):
            return w
    return 8


class _FV:
    """A pending value: inline scalar (val = number, width = its minimal byte width) or an
    object already written at buffer position val (width = its element byte width)."""
    __slots__ = ("type", "width", "val")

    def __init__(self, type_: int, width: int, val):
        self.type, self.width, self.val = type_, width, val

    def elem_width(self, buf_size: int, index: int) -> int:
        if self.type in _INLINE:
            return self.width
        for w in (1, 2, 4, 8):  # where the slot would land at this width
            loc = buf_size + (-buf_size) % w + index * w
            if _uwidth(loc - self.val) <= w:
                return w
        raise ValueError("flexbuffer offset too large")


class Flex:
    """Minimal flexbuffers builder (layout rules of the reference flexbuffers implementation).
    Build with the typed push methods / start_map/end_map / start_vector/end_vector, then
    finish()."""

    def __init__(self):
        self.buf = bytearray()
        self.stack: list[_FV] = []

    # ---- scalars
    def null(self):
        self.stack.append(_FV(FX_NULL, 1, 0))

    def boolean(self, b: bool):
        self.stack.append(_FV(FX_BOOL, 1, int(bool(b))))

    def int(self, i: int):
        self.stack.append(_FV(FX_INT, _iwidth(int(i)), int(i)))

    def uint(self, u: int):
        self.stack.append(_FV(FX_UINT, _uwidth(int(u)), int(u)))

    def float(self, x: float, width: int = 8):
        self.stack.append(_FV(FX_FLOAT, width, float(x)))

    def _pad(self, w: int):
        self.buf += b"\0" * ((-len(self.buf)) % w)

    def string(self, s: str):
        b = s.encode()
        w = _uwidth(len(b))
        self._pad(w)
        self.buf += len(b).to_bytes(w, "little")
        loc = len(self.buf)
        self.buf += b + b"\0"
        self.stack.append(_FV(FX_STRING, w, loc))

    def key(self, s: str):
        loc = len(self.buf)
        self.buf += s.encode() + b"\0"
        self.stack.append(_FV(FX_KEY, 1, loc))

    # ---- containers
    def start_vector(self) -> int:
        return len(self.stack)

    def start_map(self) -> int:
        return len(self.stack)

    def _write_any(self, v: _FV, w: int):
        if v.type == FX_NULL:
            self.buf += bytes(w)
        elif v.type == FX_FLOAT:
            self.buf += struct.pack("<f" if w == 4 else "<d", v.val)
        elif v.type == FX_INT:
            self.buf += int(v.val).to_bytes(w, "little", signed=True)
        elif v.type in (FX_UINT, FX_BOOL):
            self.buf += int(v.val).to_bytes(w, "little")
        else:  # offset back to the object
            self.buf += (len(self.buf) - v.val).to_bytes(w, "little")

    def _stored_type(self, v: _FV, w: int) -> int:
        return (v.type << 2) | _WCODE[max(v.width, w) if v.type in _INLINE else v.width]

    def _create_vector(self, elems: list, typed: bool, keys: Optional[_FV] = None) -> _FV:
        n = len(elems)
        w = _uwidth(n)
        prefix = 1
        if keys is not None:
            w = max(w, keys.elem_width(len(self.buf), 0))
            prefix += 2
        for i, e in enumerate(elems):
            w = max(w, e.elem_width(len(self.buf), i + prefix))
        if any(e.type == FX_FLOAT for e in elems):
            w = max(w, max(e.width for e in elems if e.type == FX_FLOAT))
        self._pad(w)
        if keys is not None:
            self.buf += (len(self.buf) - keys.val).to_bytes(w, "little")
            self.buf += keys.width.to_bytes(w, "little")
        self.buf += n.to_bytes(w, "little")
        loc = len(self.buf)
        for e in elems:
            self._write_any(e, w)
        if not typed:
            for e in elems:
                self.buf.append(self._stored_type(e, w))
        if keys is not None:
            t = FX_MAP
        elif typed:
            t = {FX_KEY: FX_VEC_KEY, FX_INT: 11, FX_UINT: 12, FX_FLOAT: 13, FX_BOOL: 36}[elems[0].type] if elems else FX_VEC_KEY
        else:
            t = FX_VECTOR
        return _FV(t, w, loc)

    def end_vector(self, start: int, typed: Optional[bool] = None):
        """typed=None: a typed vector (VectorInt/UInt/Float/Bool) when every element is a
        scalar of one type, as the reference builder emits for [u16; 8] / Vec<u32>."""
        elems = self.stack[start:]
        del self.stack[start:]
        if typed is None:
            typed = TYPED_VECTORS and len(elems) > 0 and len({e.type for e in elems}) == 1 and \
                elems[0].type in (FX_INT, FX_UINT, FX_FLOAT, FX_BOOL)
        self.stack.append(self._create_vector(elems, typed=typed))

    def end_map(self, start: int):
        items = self.stack[start:]
        del self.stack[start:]
        pairs = [(items[i], items[i + 1]) for i in range(0, len(items), 2)]

        def kbytes(k: _FV) -> bytes:
            e = self.buf.index(0, k.val)
            return bytes(self.buf[k.val: e])
        pairs.sort(key=lambda kv: kbytes(kv[0]))  # maps are sorted by key
        keys = self._create_vector([k for k, _ in pairs], typed=True)
        self.stack.append(self._create_vector([v for _, v in pairs], typed=False, keys=keys))

    def finish(self) -> bytes:
        assert len(self.stack) == 1, "flexbuffer root must be one value"
        v = self.stack[0]
        w = v.elem_width(len(self.buf), 0)
        self._pad(w)
        self._write_any(v, w)
        self.buf.append((v.type << 2) | _WCODE[v.width])
        self.buf.append(w)
        return bytes(self.buf)


def flex_encode(obj) -> bytes:
    """serde value -> flexbuffer: dict -> map (keys sorted), list/tuple -> vector, None -> null,
    bool, int (Int if negative else UInt, minimal width), float (f64) / ('f32', x), str.  Use
    ('i', v) / ('u', v) to force the signedness of an integer."""
    fb = Flex()

    def put(o):
        if o is None:
            fb.null()
        elif isinstance(o, bool):
            fb.boolean(o)
        elif isinstance(o, tuple) and len(o) == 2 and o[0] in ("i", "u", "f32", "f64"):
            tag, v = o
            if tag == "i":
                fb.int(int(v))
            elif tag == "u":
                fb.uint(int(v))
            else:
                fb.float(float(v), 4 if tag == "f32" else 8)
        elif isinstance(o, (int, np.integer)):
            fb.int(int(o)) if int(o) < 0 else fb.uint(int(o))
        elif isinstance(o, (float, np.floating)):
            fb.float(float(o))
        elif isinstance(o, str):
            fb.string(o)
        elif isinstance(o, dict):
            s = fb.start_map()
            for k, v in o.items():
                fb.key(k)
                put(v)
            fb.end_map(s)
        elif isinstance(o, (list, tuple)):
            s = fb.start_vector()
            for v in o:
                put(v)
            fb.end_vector(s)
        else:
            raise TypeError(f"cannot flex-encode {type(o)}")

    put(obj)
    return fb.finish()


# ============================================================================ flatbuffers
class FBB:
    """Back-to-front flatbuffers builder: objects are referenced by their distance from the
    buffer end; uoffsets point forward; vtables precede their tables."""

    def __init__(self):
        self.b = bytearray()
        self.minalign = 1
        self.vtable: list = []
        self.obj_start = 0

    def _prepend(self, data: bytes):
        self.b[0:0] = data

    def prep(self, size: int, additional: int):
        self.minalign = max(self.minalign, size)
        self._prepend(bytes((-(len(self.b) + additional)) % size))

    def scalar(self, fmt: str, v):
        self.prep(struct.calcsize(fmt), 0)
        self._prepend(struct.pack("<" + fmt, v))

    def uoffset(self, off: int):
        self.prep(4, 0)
        self._prepend(struct.pack("<I", len(self.b) - off + 4))

    def create_bytes(self, data: bytes, string: bool = False) -> int:
        self.prep(4, len(data) + (1 if string else 0))
        if string:
            self._prepend(b"\0")
        self._prepend(bytes(data))
        self._prepend(struct.pack("<I", len(data)))
        return len(self.b)

    def create_offsets(self, offs: Sequence[int]) -> int:
        self.prep(4, 4 * len(offs))
        for o in reversed(offs):
            self.uoffset(o)
        self._prepend(struct.pack("<I", len(offs)))
        return len(self.b)

    def create_structs(self, items: Sequence[bytes], size: int, align: int) -> int:
        self.prep(4, size * len(items))
        self.prep(align, size * len(items))
        for it in reversed(items):
            self._prepend(it)
        self._prepend(struct.pack("<I", len(items)))
        return len(self.b)

    def start(self, nfields: int):
        self.vtable = [0] * nfields
        self.obj_start = len(self.b)

    def field(self, i: int, fmt: str, v):
        self.scalar(fmt, v)
        self.vtable[i] = len(self.b)

    def field_offset(self, i: int, off: int):
        self.uoffset(off)
        self.vtable[i] = len(self.b)

    def end(self) -> int:
        self.prep(4, 0)
        self._prepend(b"\0\0\0\0")
        obj = len(self.b)
        vt = [obj - f if f else 0 for f in self.vtable]
        while vt and vt[-1] == 0:
            vt.pop()
        for f in reversed(vt):
            self._prepend(struct.pack("<H", f))
        self._prepend(struct.pack("<H", obj - self.obj_start))
        self._prepend(struct.pack("<H", 4 + 2 * len(vt)))
        vt_off = len(self.b)
        struct.pack_into("<i", self.b, len(self.b) - obj, vt_off - obj)
        return obj

    def finish(self, root: int) -> bytes:
        self.prep(self.minalign, 4)
        self.uoffset(root)
        return bytes(self.b)


# ---- dtype.fbs -----------------------------------------------------------------------------
@dataclass
class DType:
    kind: str                  # "null" | "bool" | "primitive" | "utf8" | "binary" | "struct" | "extension"
    ptype: str = "u8"
    nullable: bool = False
    names: tuple = ()
    fields: tuple = ()
    ext_id: str = ""
    ext_meta: bytes = b""

    def serde(self):
        """serde-derive form (DType enum; Nullability as bool)."""
        if self.kind == "null":
            return "Null"
        if self.kind == "bool":
            return {"Bool": self.nullable}
        if self.kind == "primitive":
            return {"Primitive": [self.ptype, self.nullable]}
        if self.kind in ("utf8", "binary"):
            return {self.kind.capitalize(): self.nullable}
        raise NotImplementedError(self.kind)


def dtype_of(a: Array) -> DType:
    if a.encoding == ENC_EXTENSION:
        return a.meta["ext_dtype"]
    k = {DTYPE["NULL"]: "null", DTYPE["BOOL"]: "bool", DTYPE["PRIMITIVE"]: "primitive", DTYPE["UTF8"]: "utf8",
         DTYPE["BINARY"]: "binary"}[a.dtype]
    return DType(k, a.ptype if k == "primitive" else "u8", bool(a.nullable))


_FB_TYPE = {"null": 1, "bool": 2, "primitive": 3, "utf8": 5, "binary": 6, "struct": 7, "extension": 9}


def write_dtype(fbb: FBB, d: DType) -> int:
    """dtype.fbs DType {type_type, type} (vortex-dtype/src/serde/flatbuffers/mod.rs:103-170)."""
    if d.kind == "null":
        fbb.start(0)
        inner = fbb.end()
    elif d.kind in ("bool", "utf8", "binary"):
        fbb.start(1)
        fbb.field(0, "B", int(d.nullable))
        inner = fbb.end()
    elif d.kind == "primitive":
        fbb.start(2)
        fbb.field(0, "B", PTYPES.index(d.ptype))
        fbb.field(1, "B", int(d.nullable))
        inner = fbb.end()
    elif d.kind == "struct":
        names = [fbb.create_bytes(n.encode(), string=True) for n in d.names]
        nv = fbb.create_offsets(names)
        dts = [write_dtype(fbb, f) for f in d.fields]
        dv = fbb.create_offsets(dts)
        fbb.start(3)
        fbb.field_offset(0, nv)
        fbb.field_offset(1, dv)
        fbb.field(2, "B", int(d.nullable))
        inner = fbb.end()
    elif d.kind == "extension":
        idv = fbb.create_bytes(d.ext_id.encode(), string=True)
        mv = fbb.create_bytes(d.ext_meta) if d.ext_meta is not None else 0
        fbb.start(3)
        fbb.field_offset(0, idv)
        if mv:
            fbb.field_offset(1, mv)
        fbb.field(2, "B", int(d.nullable))
        inner = fbb.end()
    else:
        raise NotImplementedError(d.kind)
    fbb.start(2)
    fbb.field(0, "B", _FB_TYPE[d.kind])
    fbb.field_offset(1, inner)
    return fbb.end()


# ---- array metadata (the reference serde structs) --------------------------------------------
_VALIDITY_NAME = {v: k for k, v in {"NonNullable": VALIDITY["NON_NULLABLE"], "AllValid": VALIDITY["ALL_VALID"],
                                    "AllInvalid": VALIDITY["ALL_INVALID"], "Array": VALIDITY["ARRAY"]}.items()}


def _scalar(raw: bytes, is_null: bool, d: DType):
    """ScalarValue::serialize (vortex-scalar/src/serde/serde.rs:10-45) of a value stored as LE
    bytes in the dtype's ptype."""
    if is_null:
        return None
    if d.kind == "bool":
        return bool(raw[0])
    p = d.ptype
    if p in ("f32", "f64"):
        return (p, float(np.frombuffer(raw[: 4 if p == "f32" else 8], dtype=np.float32 if p == "f32" else np.float64)[0]))
    if p == "f16":
        return ("u", int.from_bytes(raw[:2], "little"))  # PValue::F16 serializes its u16 bits
    w = int(p[1:]) // 8
    return ("i", int.from_bytes(raw[:w], "little", signed=True)) if p[0] == "i" else ("u", int.from_bytes(raw[:w], "little"))


def ref_metadata(a: Array):
    """The reference's metadata struct of `a` as a serde value (None = no metadata bytes)."""
    e, m = a.encoding, a.meta
    d = dtype_of(a)
    val = _VALIDITY_NAME.get(a.validity, "NonNullable")
    if e == ENC["PRIMITIVE"] or e == ENC["BYTE_BOOL"]:
        return {"validity": val}
    if e == ENC["BOOL"]:
        return {"validity": val, "first_byte_bit_offset": m.get("first_byte_bit_offset", 0)}
    if e == ENC["VARBIN"]:
        return {"validity": val, "offsets_ptype": PTYPES[m["offsets_ptype"]], "bytes_len": m["bytes_len"]}
    if e == ENC["VARBINVIEW"]:
        return {"validity": val, "buffer_lens": [c.len for c in a.children[1: 1 + m["n_buffers"]]]}
    if e == ENC["SPARSE"]:
        return {"indices_offset": m["indices_offset"], "indices_len": m["indices_len"],
                "fill_value": _scalar(bytes(m["fill"]), m["fill_is_null"], d)}
    if e == ENC["CONSTANT"]:
        return {"scalar_value": _scalar(bytes(m["scalar"]), m["is_null"], d)}
    if e == ENC["CHUNKED"]:
        return {"nchunks": m["nchunks"]}
    if e == ENC["ALP"]:
        return {"exponents": {"e": m["e"], "f": m["f"]}}
    if e == ENC["ALP_RD"]:
        return {"right_bit_width": m["right_bit_width"], "dict_len": m["dict_len"],
                "dict": [("u", int(x)) for x in list(m["dict"])[:8]] + [("u", 0)] * (8 - len(list(m["dict"])[:8])),
                "left_parts_ptype": PTYPES[m["left_parts_ptype"]], "has_exceptions": bool(m["has_exceptions"])}
    if e == ENC["DICT"]:
        return {"codes_ptype": PTYPES[m["codes_ptype"]], "values_len": m["values_len"]}
    if e == ENC["FL_BITPACKED"]:
        return {"validity": val, "bit_width": m["bit_width"], "offset": m["offset"],
                "has_patches": bool(m["has_patches"])}
    if e == ENC["FL_DELTA"]:
        return {"validity": val, "deltas_len": m["deltas_len"], "offset": m["offset"]}
    if e == ENC["FL_FOR"]:
        w = int(a.ptype[1:]) // 8
        raw = int(m["reference"]).to_bytes(8, "little")[:w].ljust(16, b"\0")
        return {"reference": _scalar(raw, False, d), "shift": m["shift"]}
    if e == ENC["FSST"]:
        return {"symbols_len": m["symbols_len"], "codes_nullability": bool(m["codes_nullable"]),
                "uncompressed_lengths_ptype": PTYPES[m["uncompressed_lengths_ptype"]]}
    if e == ENC["RUN_END"]:
        return {"validity": val, "ends_ptype": PTYPES[m["ends_ptype"]], "num_runs": m["num_runs"], "offset": m["offset"]}
    if e == ENC["RUN_END_BOOL"]:
        return {"start": bool(m["start"]), "validity": val, "ends_ptype": PTYPES[m["ends_ptype"]],
                "num_runs": m["num_runs"], "offset": m["offset"]}
    if e == ENC["ZIGZAG"] or e == ENC["ROARING_BOOL"]:
        return None  # unit structs ZigZagMetadata / RoaringBoolMetadata -> flexbuffer null
    if e == ENC_STRUCT:
        return {"validity": val}
    if e == ENC_EXTENSION:
        return {"storage_dtype": dtype_of(a.children[0]).serde()}
    raise NotImplementedError(f"no reference metadata for encoding {e}")


def extension(storage: Array, ext_id: str, ext_meta: bytes) -> Array:
    """ExtensionArray::new (array/extension/mod.rs:28-40) over `storage`."""
    d = DType("extension", nullable=bool(storage.nullable), ext_id=ext_id, ext_meta=ext_meta)
    return Array(ENC_EXTENSION, storage.len, storage.dtype, storage.ptype, storage.nullable, VALIDITY["NON_NULLABLE"],
                 {"ext_dtype": d}, [], [storage])


def date_column(storage: Array) -> Array:
    """TemporalArray::new_date (array/datetime/mod.rs:70-90): vortex.date, TimeUnit::D (tag 4,
    vortex-datetime-dtype/src/unit.rs:22-29) over i32 days."""
    return extension(storage, "vortex.date", bytes([4]))


# ---- IPC messages (messages.rs) ---------------------------------------------------------------
def _preorder(a: Array):
    yield a
    for c in a.children:
        yield from _preorder(c)


def _buffer_of(a: Array) -> Optional[bytes]:
    if not a.buffers:
        return None
    if len(a.buffers) != 1:
        raise ValueError("a Vortex array node holds at most one buffer")
    b = a.buffers[0]
    if hasattr(b, "cpu"):
        b = b.cpu().numpy()
    return np.ascontiguousarray(b).view(np.uint8).reshape(-1).tobytes()


def _write_array(fbb: FBB, a: Array, counter: list) -> int:
    """IPCArray::write_flatbuffer (messages.rs:104-163): buffer indices in pre-order."""
    bi = None
    if _buffer_of(a) is not None:
        bi = counter[0]
        counter[0] += 1
    kids = [_write_array(fbb, c, counter) for c in a.children]
    md = ref_metadata(a)
    mv = fbb.create_bytes(flex_encode(md))
    fbb.start(10)  # ArrayStats: no statistics recorded
    stats = fbb.end()
    cv = fbb.create_offsets(kids)
    fbb.start(6)
    if bi is not None:
        fbb.field(1, "Q", bi)
    fbb.field(2, "H", a.encoding)
    fbb.field_offset(3, mv)
    fbb.field_offset(4, stats)
    fbb.field_offset(5, cv)
    return fbb.end()


def _message(header_type: int, build_header) -> bytes:
    """MessageWriter::write_message (message_writer.rs:88-126): u32 length (of the padded
    flatbuffer) + Message flatbuffer + zero padding to 64 bytes."""
    fbb = FBB()
    h = build_header(fbb)
    fbb.start(3)
    fbb.field(1, "B", header_type)
    fbb.field_offset(2, h)
    fb = fbb.finish(fbb.end())
    size = _align(4 + len(fb))
    return struct.pack("<I", size - 4) + fb + bytes(size - 4 - len(fb))


def schema_message(d: DType) -> bytes:
    def hdr(fbb):
        dt = write_dtype(fbb, d)
        fbb.start(1)
        fbb.field_offset(0, dt)
        return fbb.end()
    return _message(1, hdr)


def batch_message(a: Array) -> bytes:
    """MessageWriter::write_batch (message_writer.rs:51-73) + IPCBatch (messages.rs:63-102)."""
    bufs = [b for b in (_buffer_of(n) for n in _preorder(a)) if b is not None]
    descs, off = [], 0
    for b in bufs:
        al = _align(len(b))
        descs.append(struct.pack("<QHB5x", off, al - len(b), 0))
        off += al

    def hdr(fbb):
        arr = _write_array(fbb, a, [0])
        bv = fbb.create_structs(descs, 16, 8)
        fbb.start(4)
        fbb.field(1, "Q", a.len)
        fbb.field(3, "Q", off)
        fbb.field_offset(0, arr)
        fbb.field_offset(2, bv)
        return fbb.end()
    body = bytearray()
    for b in bufs:
        body += b + bytes(_align(len(b)) - len(b))
    return _message(2, hdr) + bytes(body)


# ---- layouts + footer (layouts/write/{layouts,footer,writer}.rs) ------------------------------
@dataclass
class Layout:
    id: int
    buffers: Optional[list] = None   # [(begin, end)]
    children: Optional[list] = None
    metadata: Optional[bytes] = None


def _write_layout(fbb: FBB, l: Layout) -> int:
    bv = fbb.create_structs([struct.pack("<QQ", b, e) for b, e in l.buffers], 16, 8) if l.buffers is not None else 0
    md = fbb.create_bytes(l.metadata) if l.metadata is not None else 0
    kids = [_write_layout(fbb, c) for c in l.children] if l.children is not None else None
    cv = fbb.create_offsets(kids) if kids is not None else 0
    fbb.start(4)
    fbb.field(0, "H", l.id)
    if bv:
        fbb.field_offset(1, bv)
    if cv:
        fbb.field_offset(2, cv)
    if md:
        fbb.field_offset(3, md)
    return fbb.end()


def write_file(columns: Sequence[tuple], row_count: Optional[int] = None,
               message_order: Optional[Sequence[tuple]] = None) -> bytes:
    """LayoutWriter::write_array_columns + finalize for a StructArray whose fields are
    ChunkedArrays (bench-vortex tpch/mod.rs:249-307): `columns` = [(name, [chunk Array, ...])].
    Each chunk is one Batch message; every column's chunks are written consecutively, unless
    `message_order` (a permutation of (column, chunk) pairs) says otherwise (test input for
    readers that must not assume ascending, contiguous chunk messages)."""
    out = bytearray()
    order = list(message_order) if message_order is not None else \
        [(ci, k) for ci, (_, chunks) in enumerate(columns) for k in range(len(chunks))]
    if sorted(order) != [(ci, k) for ci, (_, chunks) in enumerate(columns) for k in range(len(chunks))]:
        raise ValueError("message_order must be a permutation of the (column, chunk) pairs")
    spans = {}
    for ci, k in order:
        b = len(out)
        out += batch_message(columns[ci][1][k])
        spans[(ci, k)] = (b, len(out))
    col_ranges = []
    nrows = None
    for ci, (name, chunks) in enumerate(columns):
        rows = [0]
        for c in chunks:
            rows.append(rows[-1] + c.len)
        col_ranges.append(([spans[(ci, k)] for k in range(len(chunks))], rows))
        nrows = rows[-1] if nrows is None else nrows
        if rows[-1] != nrows:
            raise ValueError("columns of different lengths")
    # per-column metadata tables (writer.rs:120-157)
    layouts = []
    meta_dtype = DType("struct", names=("row_offset",), fields=(DType("primitive", "u64"),))
    for spans_c, rows in col_ranges:
        flats = [Layout(FLAT, buffers=[(b, e)]) for b, e in spans_c]
        row_offsets = np.array(rows[:-1], dtype=np.uint64)
        table = Array(ENC_STRUCT, len(row_offsets), DTYPE["NULL"], "u8", False, VALIDITY["NON_NULLABLE"], {}, [],
                      [Array(ENC["PRIMITIVE"], len(row_offsets), DTYPE["PRIMITIVE"], "u64", False,
                             VALIDITY["NON_NULLABLE"], {}, [row_offsets])])
        d0 = len(out)
        out += schema_message(meta_dtype)
        d1 = len(out)
        out += batch_message(table)
        flats.insert(0, Layout(INLINE_SCHEMA, buffers=[(d0, d1)], children=[Layout(FLAT, buffers=[(d1, len(out))])]))
        layouts.append(Layout(CHUNKED_LAYOUT, children=flats, metadata=bytes([1])))
    schema = DType("struct", names=tuple(n for n, _ in columns),
                   fields=tuple(dtype_of(ch[0]) for _, ch in columns))
    schema_offset = len(out)
    out += schema_message(schema)
    footer_offset = len(out)
    fbb = FBB()
    lay = _write_layout(fbb, Layout(COLUMN, children=layouts))
    fbb.start(2)
    fbb.field(1, "Q", nrows if row_count is None else row_count)
    fbb.field_offset(0, lay)
    fb = fbb.finish(fbb.end())
    size = _align(4 + len(fb))
    out += struct.pack("<I", size - 4) + fb + bytes(size - 4 - len(fb))
    fbb = FBB()  # Postscript: the raw 32-byte flatbuffer (writer.rs:191-201, FOOTER_POSTSCRIPT_SIZE)
    fbb.start(2)
    fbb.field(1, "Q", footer_offset)
    fbb.field(0, "Q", schema_offset)
    ps = fbb.finish(fbb.end())
    assert len(ps) == 32, len(ps)
    out += ps
    out += struct.pack("<H", VERSION) + b"\0\0" + MAGIC
    return bytes(out)
