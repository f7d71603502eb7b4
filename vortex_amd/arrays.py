"""Host-side mirror of the Vortex array model for the canonicalize hot path.

`Array` mirrors vortex-array's `Array`/`ArrayData` (vortex-array/src/data.rs:14-22): an encoding
id (encoding/mod.rs:106-147), a dtype, a length, the encoding's metadata struct, its buffers
and its children in the reference's child order.  The factory functions restate the
reference constructors *including their validation* (e.g. `BitPackedArray::try_new`,
bitpacking/mod.rs:54-130) so malformed trees fail the same way, with the same VortexError
kind, before anything reaches the GPU.

`canonicalize(array, ctx)` is `Array::into_canonical` (canonical.rs:353-357): the tree is
flattened into `vxg_array` descriptors and handed to the C ABI (`vxg_canonicalize`); the result
is a `Canonical` whose buffers are torch tensors in HBM.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Any, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import DTYPE, ENC, PTYPE, PTYPES, VALIDITY, VortexGpuError

NP_OF_PTYPE = {"u8": np.uint8, "u16": np.uint16, "u32": np.uint32, "u64": np.uint64,
               "i8": np.int8, "i16": np.int16, "i32": np.int32, "i64": np.int64,
               "f16": np.float16, "f32": np.float32, "f64": np.float64}
PTYPE_OF_NP = {np.dtype(v): k for k, v in NP_OF_PTYPE.items()}


def ptype_width(p: str) -> int:
    return np.dtype(NP_OF_PTYPE[p]).itemsize


def unsigned_of(p: str) -> str:
    return "u" + p[1:] if p[0] == "i" else p


class VortexError(VortexGpuError):
    pass


def _bail(kind: str, msg: str):
    code = {v: k for k, v in _lib.STATUS.items()}[kind]
    raise VortexError(code, msg)


@dataclass
class Array:
    encoding: int
    len: int
    dtype: int = DTYPE["PRIMITIVE"]
    ptype: str = "u8"
    nullable: bool = False
    validity: int = VALIDITY["NON_NULLABLE"]
    meta: dict = field(default_factory=dict)
    buffers: list = field(default_factory=list)  # numpy arrays (host) or torch tensors (device)
    children: list = field(default_factory=list)

    # ---- movement -----------------------------------------------------------------
    def to(self, device) -> "Array":
        """Copy every buffer into device memory (torch tensors; 16-byte aligned)."""
        import torch

        def mv(b):
            if isinstance(b, torch.Tensor):
                return b.to(device)
            a = np.ascontiguousarray(b).view(np.uint8).reshape(-1)
            if not a.flags.writeable:
                a = a.copy()  # torch.from_numpy needs a writable buffer
            t = torch.empty(max(a.size, 16), dtype=torch.uint8, device=device)
            if a.size:
                t[: a.size].copy_(torch.from_numpy(a))
            return t[: a.size] if a.size else t[:0]

        return Array(self.encoding, self.len, self.dtype, self.ptype, self.nullable, self.validity,
                     dict(self.meta), [mv(b) for b in self.buffers],
                     [c.to(device) for c in self.children])

    def nbytes(self) -> int:
        """Bytes of all buffers in the tree (the compressed size the decoder reads)."""
        tot = 0
        for b in self.buffers:
            tot += b.numel() * b.element_size() if hasattr(b, "element_size") else np.asarray(b).nbytes
        return tot + sum(c.nbytes() for c in self.children)


# ---- constructors (reference validation restated) -------------------------------------
def _np(x, p=None):
    a = np.ascontiguousarray(x)
    if p is not None:
        a = a.astype(NP_OF_PTYPE[p], copy=False)
    return a


def bool_validity(mask) -> "Array":
    """Canonical BoolArray validity (LSB bitmap), array/bool/mod.rs:25-28."""
    m = np.asarray(mask, dtype=bool)
    bits = np.packbits(m, bitorder="little")
    return Array(ENC["BOOL"], len(m), DTYPE["BOOL"], "u8", False, VALIDITY["NON_NULLABLE"],
                 {"first_byte_bit_offset": 0}, [bits])


def _validity_kind(nullable: bool, validity) -> tuple[int, Optional[Array]]:
    if validity is None:
        return (VALIDITY["ALL_VALID"] if nullable else VALIDITY["NON_NULLABLE"]), None
    if isinstance(validity, str):
        return VALIDITY[validity], None
    if isinstance(validity, Array):  # any Bool-dtype array (RunEndBool, ByteBool, ...)
        if validity.dtype != DTYPE["BOOL"]:
            _bail("InvalidArgument", "validity must be a Bool array")
        return VALIDITY["ARRAY"], validity
    return VALIDITY["ARRAY"], bool_validity(validity)


def primitive(values, ptype: Optional[str] = None, validity=None) -> Array:
    """PrimitiveArray (array/primitive/mod.rs:33-72)."""
    a = _np(values)
    p = ptype or PTYPE_OF_NP[a.dtype]
    a = a.astype(NP_OF_PTYPE[p], copy=False)
    nullable = validity is not None
    vk, vchild = _validity_kind(nullable, validity)
    return Array(ENC["PRIMITIVE"], len(a), DTYPE["PRIMITIVE"], p, nullable, vk, {}, [a],
                 [vchild] if vchild is not None else [])


def bitpacked(packed, ptype: str, bit_width: int, length: int, offset: int = 0,
              patches: Optional[Array] = None, validity=None) -> Array:
    """BitPackedArray::try_new_from_offset (bitpacking/mod.rs:54-130)."""
    if ptype[0] != "u":
        _bail("MismatchedTypes", f"expected type: uint but instead got {ptype}")
    if bit_width > 64:
        _bail("InvalidArgument", f"Unsupported bit width {bit_width}")
    if offset > 1023:
        _bail("InvalidArgument", f"Offset must be less than full block, i.e. 1024, got {offset}")
    packed = np.ascontiguousarray(packed).view(np.uint8).reshape(-1)
    expected = ((length + offset + 1023) // 1024) * (128 * bit_width)
    if packed.size != expected:
        _bail("InvalidArgument", f"Expected {expected} packed bytes, got {packed.size}")
    if patches is not None:
        if patches.len != length:
            _bail("InvalidArgument", "Mismatched length in BitPackedArray between encoded and patches")
        if patches.encoding == ENC["SPARSE"] and patches.children[0].len == 0:
            _bail("InvalidArgument", "cannot construct BitPackedArray using patches without indices")
    nullable = validity is not None
    vk, vchild = _validity_kind(nullable, validity)
    children = ([patches] if patches is not None else []) + ([vchild] if vchild is not None else [])
    return Array(ENC["FL_BITPACKED"], length, DTYPE["PRIMITIVE"], ptype, nullable, vk,
                 {"bit_width": bit_width, "offset": offset, "has_patches": patches is not None},
                 [packed], children)


def sparse(indices: Array, values: Array, length: int, indices_offset: int = 0,
           fill=None, ptype: Optional[str] = None) -> Array:
    """SparseArray (array/sparse/mod.rs:24-29); fill None = ScalarValue::Null."""
    p = ptype or values.ptype
    fill_bytes = bytes(16)
    if fill is not None:
        fill_bytes = np.array([fill], dtype=NP_OF_PTYPE[p]).tobytes().ljust(16, b"\0")
    return Array(ENC["SPARSE"], length, DTYPE["PRIMITIVE"], p, fill is None,
                 VALIDITY["NON_NULLABLE"],
                 {"indices_offset": indices_offset, "indices_len": indices.len,
                  "fill_is_null": fill is None, "fill": fill_bytes}, [], [indices, values])


def frame_of_reference(encoded: Array, reference: int, shift: int, ptype: str) -> Array:
    """FoRArray::try_new (for/mod.rs:26-52); encoded child dtype = unsigned(ptype) (:57-66)."""
    if encoded.ptype != unsigned_of(ptype):
        _bail("MismatchedTypes", f"FoR child must be {unsigned_of(ptype)}, got {encoded.ptype}")
    ref_bits = int(np.array([reference], dtype=NP_OF_PTYPE[ptype]).view(
        NP_OF_PTYPE[unsigned_of(ptype)])[0])
    return Array(ENC["FL_FOR"], encoded.len, DTYPE["PRIMITIVE"], ptype, encoded.nullable,
                 VALIDITY["NON_NULLABLE"], {"reference": ref_bits, "shift": shift}, [], [encoded])


def zigzag(encoded: Array) -> Array:
    """ZigZagArray (zigzag/array.rs:22-103): encoded unsigned -> signed of same width."""
    if encoded.ptype[0] != "u":
        _bail("MismatchedTypes", "ZigZag encoded child must be unsigned")
    return Array(ENC["ZIGZAG"], encoded.len, DTYPE["PRIMITIVE"], "i" + encoded.ptype[1:],
                 encoded.nullable, VALIDITY["NON_NULLABLE"], {}, [], [encoded])


def alp(encoded: Array, e: int, f: int, patches: Optional[Array] = None) -> Array:
    """ALPArray::try_new (alp/array.rs:33-77): encoded i32 -> f32, i64 -> f64."""
    fp = {"i32": "f32", "i64": "f64"}.get(encoded.ptype)
    if fp is None:
        _bail("MismatchedTypes", f"ALP encoded child must be i32/i64, got {encoded.ptype}")
    return Array(ENC["ALP"], encoded.len, DTYPE["PRIMITIVE"], fp, encoded.nullable,
                 VALIDITY["NON_NULLABLE"], {"e": e, "f": f, "has_patches": patches is not None},
                 [], [encoded] + ([patches] if patches is not None else []))


def alp_rd(ptype: str, left_parts: Array, left_dict: Sequence[int], right_parts: Array,
           right_bit_width: int, exceptions: Optional[Array] = None) -> Array:
    """ALPRDArray::try_new (alp_rd/array.rs:27-115)."""
    if left_parts.len != right_parts.len:
        _bail("InvalidArgument", "left_parts and right_parts must be of same length")
    if left_parts.ptype[0] != "u":
        _bail("InvalidArgument", "left_parts dtype must be uint")
    if right_parts.nullable or right_parts.ptype[0] != "u":
        _bail("MismatchedTypes", "right_parts must be non-nullable uint")
    d = list(left_dict) + [0] * (8 - len(left_dict))
    return Array(ENC["ALP_RD"], left_parts.len, DTYPE["PRIMITIVE"], ptype, left_parts.nullable,
                 VALIDITY["NON_NULLABLE"],
                 {"right_bit_width": right_bit_width, "dict_len": len(left_dict), "dict": d,
                  "left_parts_ptype": PTYPE[left_parts.ptype], "has_exceptions": exceptions is not None},
                 [], [left_parts, right_parts] + ([exceptions] if exceptions is not None else []))


def dict_array(values: Array, codes: Array) -> Array:
    """DictArray::try_new (dict/array.rs:34-49): codes non-nullable unsigned."""
    if codes.ptype[0] != "u" or codes.nullable:
        _bail("MismatchedTypes", f"non-nullable unsigned int, got {codes.ptype}")
    return Array(ENC["DICT"], codes.len, values.dtype, values.ptype, values.nullable,
                 VALIDITY["NON_NULLABLE"], {"codes_ptype": PTYPE[codes.ptype], "values_len": values.len},
                 [], [values, codes])


def delta(bases: Array, deltas: Array, offset: int = 0, length: Optional[int] = None,
          validity=None) -> Array:
    """DeltaArray::try_new (delta/mod.rs:89-157)."""
    length = deltas.len - offset if length is None else length
    if offset >= 1024:
        _bail("InvalidArgument", f"offset must be less than 1024: {offset}")
    if offset + length > deltas.len:
        _bail("InvalidArgument", "offset + logical_len must be <= the size of deltas")
    if bases.ptype != deltas.ptype:
        _bail("InvalidArgument", "DeltaArray: bases and deltas must have the same dtype")
    lanes = 1024 // (8 * ptype_width(deltas.ptype))
    expect = (deltas.len // 1024) * lanes + (1 if deltas.len % 1024 else 0)
    if bases.len != expect:
        _bail("InvalidArgument", f"DeltaArray: bases.len() ({bases.len}) != expected_bases_len ({expect})")
    nullable = validity is not None
    vk, vchild = _validity_kind(nullable, validity)
    return Array(ENC["FL_DELTA"], length, DTYPE["PRIMITIVE"], deltas.ptype, nullable, vk,
                 {"deltas_len": deltas.len, "offset": offset}, [],
                 [bases, deltas] + ([vchild] if vchild is not None else []))


def run_end(ends: Array, values: Array, length: Optional[int] = None, offset: int = 0,
            validity=None) -> Array:
    """RunEndArray (runend/array.rs:38-93): length defaults to the last end (try_new); a
    non-zero offset must be below the first end (with_offset_and_length :63-68)."""
    if ends.ptype[0] not in "ui":
        _bail("InvalidArgument", "Run ends must be integers")
    if ends.encoding == ENC["PRIMITIVE"] and ends.len:
        ev = np.asarray(ends.buffers[0]).view(NP_OF_PTYPE[ends.ptype])
        if length is None:
            length = int(ev[ends.len - 1])
        if offset != 0 and int(ev[0]) <= offset:
            _bail("InvalidArgument", f"First run end {int(ev[0])} must be bigger than offset {offset}")
    elif length is None and ends.len == 0:
        length = 0
    if length is None:
        _bail("InvalidArgument", "length needed for compressed ends")
    nullable = validity is not None
    vk, vchild = _validity_kind(nullable, validity)
    return Array(ENC["RUN_END"], length, DTYPE["PRIMITIVE"], values.ptype, nullable, vk,
                 {"ends_ptype": PTYPE[ends.ptype], "num_runs": ends.len, "offset": offset}, [],
                 [ends, values] + ([vchild] if vchild is not None else []))


def bool_array(mask, validity=None, bit_offset: int = 0) -> Array:
    """BoolArray (array/bool/mod.rs:25-70): LSB bit buffer starting at bit `bit_offset` (< 8,
    first_byte_bit_offset of a sliced BoolArray)."""
    m = np.asarray(mask, dtype=bool)
    bits = np.packbits(np.concatenate([np.zeros(bit_offset, bool), m]), bitorder="little")
    nullable = validity is not None
    vk, vchild = _validity_kind(nullable, validity)
    return Array(ENC["BOOL"], len(m), DTYPE["BOOL"], "u8", nullable, vk, {"first_byte_bit_offset": bit_offset},
                 [bits], [vchild] if vchild is not None else [])


def byte_bool(mask, validity=None) -> Array:
    """ByteBoolArray::try_new (encodings/bytebool/src/array.rs:36-54): one byte per bool."""
    b = np.asarray(mask).astype(np.uint8)
    nullable = validity is not None
    vk, vchild = _validity_kind(nullable, validity)
    return Array(ENC["BYTE_BOOL"], len(b), DTYPE["BOOL"], "u8", nullable, vk, {}, [b],
                 [vchild] if vchild is not None else [])


def roaring_bool(bitmap, length: int) -> Array:
    """RoaringBoolArray (encodings/roaring/src/boolean/mod.rs:36-67): DType::Bool(NonNullable),
    one buffer holding croaring's Native serialization of the set positions, no metadata."""
    b = np.ascontiguousarray(bitmap).view(np.uint8).reshape(-1)
    return Array(ENC["ROARING_BOOL"], length, DTYPE["BOOL"], "u8", False, VALIDITY["NON_NULLABLE"], {}, [b])


def run_end_bool(ends: Array, start: bool, length: Optional[int] = None, offset: int = 0, validity=None) -> Array:
    """RunEndBoolArray::with_offset_and_size (encodings/runend-bool/src/array.rs:41-80): ends
    strictly increasing unsigned ints (>= 1 element); length defaults to the last end."""
    if ends.ptype[0] != "u":
        _bail("InvalidArgument", f"Ends array must be an unsigned integer type, got {ends.ptype}")
    if ends.len == 0:
        _bail("InvalidArgument", "Ends array must have at least one element")
    if length is None:
        length = int(np.asarray(ends.buffers[0])[ends.len - 1]) if ends.encoding == ENC["PRIMITIVE"] else None
        if length is None:
            _bail("InvalidArgument", "length needed for compressed ends")
    nullable = validity is not None
    vk, vchild = _validity_kind(nullable, validity)
    return Array(ENC["RUN_END_BOOL"], length, DTYPE["BOOL"], "u8", nullable, vk,
                 {"start": bool(start), "ends_ptype": PTYPE[ends.ptype], "num_runs": ends.len, "offset": offset},
                 [], [ends] + ([vchild] if vchild is not None else []))


def constant_bool(value: Optional[bool], length: int) -> Array:
    """ConstantArray of a Bool scalar (constant/canonical.rs:26-33); None = null."""
    sc = bytes(16) if value is None else bytes([1 if value else 0]).ljust(16, b"\0")
    return Array(ENC["CONSTANT"], length, DTYPE["BOOL"], "u8", value is None, VALIDITY["NON_NULLABLE"],
                 {"is_null": value is None, "scalar": sc})


def sparse_bool(indices: Array, values: Array, length: int, indices_offset: int = 0, fill=None) -> Array:
    """SparseArray of bools (sparse/flatten.rs:41-61); fill None = null.  Canonicalizes with a
    validity bitmap set exactly at the indices, whatever the fill (the reference's behaviour)."""
    if values.dtype != DTYPE["BOOL"]:
        _bail("MismatchedTypes", "sparse_bool values must be a Bool array")
    fill_bytes = bytes(16) if fill is None else bytes([1 if fill else 0]).ljust(16, b"\0")
    return Array(ENC["SPARSE"], length, DTYPE["BOOL"], "u8", True, VALIDITY["NON_NULLABLE"],
                 {"indices_offset": indices_offset, "indices_len": indices.len,
                  "fill_is_null": fill is None, "fill": fill_bytes}, [], [indices, values])


def constant(value, length: int, ptype: str) -> Array:
    """ConstantArray (array/constant/mod.rs:22-60); value None = null scalar."""
    sc = bytes(16) if value is None else np.array([value], dtype=NP_OF_PTYPE[ptype]).tobytes().ljust(16, b"\0")
    return Array(ENC["CONSTANT"], length, DTYPE["PRIMITIVE"], ptype, value is None,
                 VALIDITY["NON_NULLABLE"], {"is_null": value is None, "scalar": sc})


def chunked(chunks: Sequence[Array]) -> Array:
    """ChunkedArray::try_new (array/chunked/mod.rs:47-80): child 0 = u64 chunk offsets."""
    if not chunks:
        _bail("InvalidArgument", "chunked needs at least one chunk for a dtype")
    d0 = (chunks[0].dtype, chunks[0].ptype)
    for c in chunks:
        if (c.dtype, c.ptype) != d0:
            _bail("MismatchedTypes", "Chunks must have the same dtype")
    offs = np.zeros(len(chunks) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([c.len for c in chunks])
    return Array(ENC["CHUNKED"], int(offs[-1]), chunks[0].dtype, chunks[0].ptype,
                 any(c.nullable for c in chunks), VALIDITY["NON_NULLABLE"],
                 {"nchunks": len(chunks)}, [], [primitive(offs)] + list(chunks))


def varbin(offsets: Array, data: Array, utf8: bool = True, validity=None) -> Array:
    """VarBinArray (array/varbin/mod.rs:35-100): children offsets, bytes, validity."""
    nullable = validity is not None
    vk, vchild = _validity_kind(nullable, validity)
    return Array(ENC["VARBIN"], offsets.len - 1, DTYPE["UTF8" if utf8 else "BINARY"], "u8", nullable,
                 vk, {"offsets_ptype": PTYPE[offsets.ptype], "bytes_len": data.len}, [],
                 [offsets, data] + ([vchild] if vchild is not None else []))


def varbinview(views, buffers: Sequence, utf8: bool = True, validity=None) -> Array:
    """VarBinViewArray::try_new (array/varbinview/mod.rs:217-262): children views (u8, 16 B per
    row), the data buffers (u8), validity.  `views` is a (n, 16) / flat u8 array of arrow
    BinaryViews; buffer_lens must fit u32."""
    v = np.ascontiguousarray(views, dtype=np.uint8).reshape(-1)
    if v.size % 16:
        _bail("InvalidArgument", "views must be a multiple of 16 bytes")
    bufs = [np.ascontiguousarray(b, dtype=np.uint8).reshape(-1) for b in buffers]
    if any(b.size >= 2 ** 32 for b in bufs):
        _bail("InvalidArgument", "buffer must be within 32-bit range")
    nullable = validity is not None
    vk, vchild = _validity_kind(nullable, validity)
    return Array(ENC["VARBINVIEW"], v.size // 16, DTYPE["UTF8" if utf8 else "BINARY"], "u8", nullable, vk,
                 {"n_buffers": len(bufs)}, [],
                 [primitive(v)] + [primitive(b) for b in bufs] + ([vchild] if vchild is not None else []))


def fsst(symbols: Array, symbol_lengths: Array, codes: Array, uncompressed_lengths: Array,
         utf8: bool = True) -> Array:
    """FSSTArray::try_new (fsst/array.rs:43-105)."""
    if symbols.len > 255:
        _bail("InvalidArgument", "symbols array must have length <= 255")
    if symbols.len != symbol_lengths.len:
        _bail("InvalidArgument", "symbols and symbol_lengths arrays must have same length")
    if uncompressed_lengths.len != codes.len:
        _bail("InvalidArgument", "uncompressed_lengths must be same len as codes")
    if codes.encoding != ENC["VARBIN"]:
        _bail("InvalidArgument", "codes array must be VarBin")
    return Array(ENC["FSST"], codes.len, DTYPE["UTF8" if utf8 else "BINARY"], "u8", codes.nullable,
                 VALIDITY["NON_NULLABLE"],
                 {"symbols_len": symbols.len, "codes_nullable": codes.nullable,
                  "uncompressed_lengths_ptype": PTYPE[uncompressed_lengths.ptype]}, [],
                 [symbols, symbol_lengths, codes, uncompressed_lengths])


# ---- flattening to the C ABI -------------------------------------------------------------
def _fill_meta(m: _lib.VxgMeta, a: Array) -> None:
    md = a.meta
    e = a.encoding
    if e == ENC["FL_BITPACKED"]:
        m.bitpacked.bit_width, m.bitpacked.has_patches, m.bitpacked.offset = (
            md["bit_width"], int(md["has_patches"]), md["offset"])
    elif e == ENC["FL_FOR"]:
        m.for_.reference, m.for_.shift = md["reference"], md["shift"]
    elif e == ENC["FL_DELTA"]:
        m.delta.deltas_len, m.delta.offset = md["deltas_len"], md["offset"]
    elif e == ENC["ALP"]:
        m.alp.e, m.alp.f, m.alp.has_patches = md["e"], md["f"], int(md["has_patches"])
    elif e == ENC["ALP_RD"]:
        m.alprd.right_bit_width = md["right_bit_width"]
        m.alprd.dict_len = md["dict_len"]
        m.alprd.left_parts_ptype = md["left_parts_ptype"]
        m.alprd.has_exceptions = int(md["has_exceptions"])
        for i, v in enumerate(md["dict"]):
            m.alprd.dict[i] = v
    elif e == ENC["DICT"]:
        m.dict.codes_ptype, m.dict.values_len = md["codes_ptype"], md["values_len"]
    elif e == ENC["FSST"]:
        m.fsst.symbols_len = md["symbols_len"]
        m.fsst.codes_nullable = int(md["codes_nullable"])
        m.fsst.uncompressed_lengths_ptype = md["uncompressed_lengths_ptype"]
    elif e == ENC["RUN_END"]:
        m.runend.ends_ptype, m.runend.num_runs, m.runend.offset = (
            md["ends_ptype"], md["num_runs"], md["offset"])
    elif e == ENC["SPARSE"]:
        m.sparse.indices_offset = md["indices_offset"]
        m.sparse.indices_len = md["indices_len"]
        m.sparse.fill_is_null = int(md["fill_is_null"])
        for i, b in enumerate(md["fill"][:16]):
            m.sparse.fill[i] = b
    elif e == ENC["CONSTANT"]:
        m.constant.is_null = int(md["is_null"])
        for i, b in enumerate(md["scalar"][:16]):
            m.constant.scalar[i] = b
    elif e == ENC["CHUNKED"]:
        m.chunked.nchunks = md["nchunks"]
    elif e == ENC["VARBIN"]:
        m.varbin.offsets_ptype, m.varbin.bytes_len = md["offsets_ptype"], md["bytes_len"]
    elif e == ENC["BOOL"]:
        m.boolean.first_byte_bit_offset = md.get("first_byte_bit_offset", 0)
    elif e == ENC["RUN_END_BOOL"]:
        m.runendbool.start, m.runendbool.ends_ptype = int(md["start"]), md["ends_ptype"]
        m.runendbool.num_runs, m.runendbool.offset = md["num_runs"], md["offset"]
    elif e == ENC["VARBINVIEW"]:
        m.varbinview.n_buffers = md["n_buffers"]


def _buf_ptr(b) -> tuple[int, int]:
    import torch
    if not isinstance(b, torch.Tensor) or not b.is_cuda:
        raise VortexError(3, "array buffers must be device tensors: call Array.to(device) first")
    return b.data_ptr(), b.numel() * b.element_size()


def flatten(a: Array, keep: list) -> _lib.VxgArray:
    node = _lib.VxgArray()
    node.encoding = a.encoding
    node.dtype = a.dtype
    node.ptype = PTYPE[a.ptype]
    node.nullable = int(a.nullable)
    node.validity = a.validity
    node.len = a.len
    _fill_meta(node.meta, a)
    if a.buffers:
        bufs = (_lib.VxgBuffer * len(a.buffers))()
        for i, b in enumerate(a.buffers):
            bufs[i].ptr, bufs[i].len = _buf_ptr(b)
            keep.append(b)  # the device tensor must outlive the node (a Plan replays it)
        keep.append(bufs)
        node.buffers = C.cast(bufs, C.POINTER(_lib.VxgBuffer))
        node.n_buffers = len(a.buffers)
    if a.children:
        kids = (_lib.VxgArray * len(a.children))()
        for i, c in enumerate(a.children):
            kids[i] = flatten(c, keep)
        keep.append(kids)
        node.children = C.cast(kids, C.POINTER(_lib.VxgArray))
        node.n_children = len(a.children)
    return node


# ---- context + canonical output ----------------------------------------------------------
class Context:
    """One vxg_ctx per device (one context per device, thread-safe calls)."""

    def __init__(self, device: int = 0):
        self.lib = _lib.gpu_lib()
        self.device = device
        h = C.c_void_p()
        _lib.check(self.lib.vxg_open(device, C.byref(h)))
        self.handle = h

    def close(self):
        if self.handle:
            self.lib.vxg_close(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream_ptr(self):
        import torch
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def sync(self):
        _lib.check(self.lib.vxg_stream_sync(self.handle, self.stream_ptr()))

    _OPTIONS = {"k1w_min_groups": _lib.OPT_K1W_MIN_GROUPS, "k1w_bpw": _lib.OPT_K1W_BPW,
                "k1_wave": _lib.OPT_K1_WAVE}

    def set_option(self, name: str, value: int):
        """vxg_set_option: a launch-shape option of this context (never changes outputs)."""
        _lib.check(self.lib.vxg_set_option(self.handle, self._OPTIONS[name], int(value)))

    def get_option(self, name: str) -> int:
        v = C.c_int64()
        _lib.check(self.lib.vxg_get_option(self.handle, self._OPTIONS[name], C.byref(v)))
        return v.value

    def launch_stats(self, reset: bool = False) -> dict:
        """vxg_get_launch_stats: the K1w launches issued (or recorded) since the last reset."""
        st = _lib.VxgLaunchStats()
        _lib.check(self.lib.vxg_get_launch_stats(self.handle, C.byref(st), int(reset)))
        return {f: getattr(st, f) for f, _ in st._fields_}


@dataclass
class Canonical:
    """Canonical::Primitive, ::Bool or ::VarBinView (canonical.rs:56-63), device tensors."""
    kind: str
    len: int
    ptype: str
    values: Any = None       # torch.uint8 tensor: len * width bytes (Primitive) / LSB bits (Bool)
    views: Any = None        # torch.uint8 tensor (16 * len) for VarBinView
    data: Any = None         # torch.uint8 tensor holding every data buffer of the view array
    validity: Any = None     # torch.uint8 LSB bitmap or None (no nulls)
    data_buffers: Any = None  # [(offset, len)] of each data buffer inside `data`
    binary: bool = False      # VarBinView of DType::Binary (else Utf8)

    def to_arrow(self):
        """Canonical::into_arrow (canonical.rs:71-85; varbinview/mod.rs:518 varbinview_as_arrow):
        the canonical buffers copied to host memory and handed to pyarrow without conversion --
        Primitive [validity, values], Bool [validity, LSB bits], VarBinView [validity, views, data
        buffer 0..n-1] (Utf8View / BinaryView).  pyarrow is optional: only this method imports it."""
        import pyarrow as pa
        validity = None if self.validity is None else pa.py_buffer(self.validity.cpu().numpy()[: (self.len + 7) // 8].copy())
        nulls = -1 if validity is not None else 0
        if self.kind == "primitive":
            t = {"u8": pa.uint8(), "u16": pa.uint16(), "u32": pa.uint32(), "u64": pa.uint64(), "i8": pa.int8(),
                 "i16": pa.int16(), "i32": pa.int32(), "i64": pa.int64(), "f16": pa.float16(), "f32": pa.float32(),
                 "f64": pa.float64()}[self.ptype]
            return pa.Array.from_buffers(t, self.len, [validity, pa.py_buffer(self.values.cpu().numpy().copy())],
                                         null_count=nulls)
        if self.kind == "bool":
            bits = self.values.cpu().numpy()[: (self.len + 7) // 8].copy()
            return pa.Array.from_buffers(pa.bool_(), self.len, [validity, pa.py_buffer(bits)], null_count=nulls)
        data = self.data.cpu().numpy()
        bufs = [pa.py_buffer(data[o: o + n].copy()) for o, n in self.data_buffers]
        views = pa.py_buffer(self.views.cpu().numpy()[: 16 * self.len].copy())
        return pa.Array.from_buffers(pa.binary_view() if self.binary else pa.string_view(), self.len,
                                     [validity, views] + bufs, null_count=nulls)

    def numpy(self):
        """Host copy: values as the ptype's numpy dtype, a bool mask, or (views u8[n,16], data u8[])."""
        if self.kind == "primitive":
            return self.values.cpu().numpy().view(NP_OF_PTYPE[self.ptype])
        if self.kind == "bool":
            return np.unpackbits(self.values.cpu().numpy(), bitorder="little")[: self.len].astype(bool)
        return self.views.cpu().numpy().reshape(-1, 16), self.data.cpu().numpy()

    def buffers(self):
        """The VarBinView's data buffers (buffer_index order) as host u8 arrays."""
        d = self.data.cpu().numpy()
        return [d[o: o + n] for o, n in self.data_buffers]

    def validity_mask(self):
        if self.validity is None:
            return None
        bits = self.validity.cpu().numpy()
        return np.unpackbits(bits, bitorder="little")[: self.len].astype(bool)


def _kind(a: Array) -> str:
    return {DTYPE["PRIMITIVE"]: "primitive", DTYPE["BOOL"]: "bool"}.get(a.dtype, "varbinview")


def canonicalize(a: Array, ctx: Context, out_values=None, sync: bool = True) -> Canonical:
    """Array::into_canonical on the GPU (vxg_canonicalize).  `out_values` (a device uint8
    tensor of len*width bytes) decodes in place, e.g. into a slice of a chunked output."""
    import torch
    keep: list = []
    node = flatten(a, keep)
    dev = torch.device("cuda", ctx.device)
    vb, db, nb = C.c_uint64(), C.c_uint64(), C.c_uint32()
    cap = 256
    while True:  # the layout (FSST heap sizes are device sums) in one call unless > cap buffers
        table = (_lib.VxgDataBuffer * cap)()
        st = ctx.lib.vxg_canonical_layout(ctx.handle, C.byref(node), C.byref(vb), C.byref(db), table, cap,
                                          C.byref(nb))
        if st == 3 and cap < (1 << 24):
            cap *= 16
            continue
        _lib.check(st)
        break
    out = _lib.VxgCanonical()
    res = Canonical(_kind(a), a.len, a.ptype, binary=a.dtype == DTYPE["BINARY"])
    nbits = ((a.len + 31) // 32) * 4
    valid_t = torch.empty(max(nbits, 4), dtype=torch.uint8, device=dev) if a.nullable else None
    if a.dtype in (DTYPE["PRIMITIVE"], DTYPE["BOOL"]):
        vals = out_values if out_values is not None else torch.empty(max(vb.value, 16), dtype=torch.uint8, device=dev)
        out.values = vals.data_ptr()
        res.values = vals[: vb.value]
    else:
        views = torch.empty(max(vb.value, 16), dtype=torch.uint8, device=dev)
        data = torch.empty(db.value + 16, dtype=torch.uint8, device=dev)
        out.views, out.data = views.data_ptr(), data.data_ptr()
        out.data_bytes = db.value
        out.data_buffers, out.n_data_buffers, out.data_buffers_cap = table, nb.value, nb.value
        res.views, res.data = views[: vb.value], data[: db.value]
        res.data_buffers = [(int(table[i].offset), int(table[i].len)) for i in range(nb.value)]
    if valid_t is not None:
        out.validity = valid_t.data_ptr()
    _lib.check(ctx.lib.vxg_canonicalize(ctx.handle, C.byref(node), C.byref(out), ctx.stream_ptr()))
    if out.validity:
        if valid_t is None or out.validity != valid_t.data_ptr():
            raise VortexError(7, "engine allocated validity for a non-nullable dtype")
        res.validity = valid_t[: (a.len + 7) // 8]
    if sync:
        ctx.sync()
    return res


def take(a: Array, indices, ctx: Context, sync: bool = True) -> Canonical:
    """compute::take (vortex-array/src/compute/take.rs:10-34) on the compressed tree
    (vxg_take_array): BitPacked / FoR / ZigZag / ALP cascades decode only the taken values, Dict
    takes its codes; `indices` is a device tensor or host array of integers."""
    import torch
    keep: list = []
    node = flatten(a, keep)
    dev = torch.device("cuda", ctx.device)
    if isinstance(indices, torch.Tensor):
        it = indices.to(dev)
        tmap = {torch.uint8: "u8", torch.int8: "i8", torch.int16: "i16", torch.int32: "i32", torch.int64: "i64"}
        for name, p in (("uint16", "u16"), ("uint32", "u32"), ("uint64", "u64")):
            if hasattr(torch, name):
                tmap[getattr(torch, name)] = p
        if it.dtype not in tmap:
            raise VortexError(3, f"take: indices must be integers, got {it.dtype}")
        ip = tmap[it.dtype]
    else:
        ia = np.ascontiguousarray(indices)
        if ia.dtype not in PTYPE_OF_NP or ia.dtype.kind not in "iu":
            raise VortexError(3, f"take: indices must be integers, got {ia.dtype}")
        ip = PTYPE_OF_NP[ia.dtype]
        it = torch.from_numpy(ia.view(np.uint8).copy()).to(dev)
    n = int(it.numel() if isinstance(indices, torch.Tensor) else np.asarray(indices).size)
    out = _lib.VxgCanonical()
    w = ptype_width(a.ptype)
    vals = torch.empty(max(n * w, 16), dtype=torch.uint8, device=dev)
    out.values = vals.data_ptr()
    vt = torch.empty(((n + 31) // 32) * 4 + 4, dtype=torch.uint8, device=dev) if a.nullable else None
    if vt is not None:
        out.validity = vt.data_ptr()
    _lib.check(ctx.lib.vxg_take_array(ctx.handle, C.byref(node), PTYPE[ip], C.c_void_p(it.data_ptr()), n,
                                      C.byref(out), ctx.stream_ptr()))
    res = Canonical("primitive", n, a.ptype, values=vals[: n * w])
    if out.validity:
        if vt is None or out.validity != vt.data_ptr():
            raise VortexError(7, "engine allocated validity for a non-nullable dtype")
        res.validity = vt[: (n + 7) // 8]
    if sync:
        ctx.sync()
    return res


def filter(a: Array, predicate: Array, ctx: Context) -> Canonical:
    """compute::filter (vortex-array/src/compute/filter.rs:23-52) on the GPU (vxg_filter_array):
    the rows of `a` whose bit in `predicate` (a non-nullable Bool array of any Bool encoding) is
    set, with the filtered validity; strings come back over one new heap of the selected rows.
    Synchronous, like the reference (the filtered length is read back)."""
    import torch
    keep: list = []
    node = flatten(a, keep)
    pnode = flatten(predicate, keep)
    dev = torch.device("cuda", ctx.device)
    n = a.len
    out = _lib.VxgCanonical()
    kind = _kind(a)
    if kind == "primitive":
        buf = torch.empty(max(n * ptype_width(a.ptype), 16), dtype=torch.uint8, device=dev)
        out.values = buf.data_ptr()
    elif kind == "bool":
        buf = torch.empty(((n + 31) // 32) * 4 + 4, dtype=torch.uint8, device=dev)
        out.values = buf.data_ptr()
    else:
        buf = torch.empty(max(16 * n, 16), dtype=torch.uint8, device=dev)
        out.views = buf.data_ptr()
    vt = torch.empty(((n + 31) // 32) * 4 + 4, dtype=torch.uint8, device=dev) if a.nullable else None
    if vt is not None:
        out.validity = vt.data_ptr()
    table = (_lib.VxgDataBuffer * 1)()
    out.data_buffers, out.data_buffers_cap = table, 1
    _lib.check(ctx.lib.vxg_filter_array(ctx.handle, C.byref(node), C.byref(pnode), C.byref(out), ctx.stream_ptr()))
    k = int(out.len)
    res = Canonical(kind, k, a.ptype, binary=a.dtype == DTYPE["BINARY"])
    if kind == "primitive":
        res.values = buf[: k * ptype_width(a.ptype)]
    elif kind == "bool":
        res.values = buf[: ((k + 31) // 32) * 4]
    else:
        res.views = buf[: 16 * k]
        hb = int(out.data_bytes)
        heap = torch.empty(hb + 16, dtype=torch.uint8, device=dev)
        if out.data:  # the engine sized and allocated the new heap: move it into a torch buffer (D2D)
            _lib.check(ctx.lib.vxg_memcpy_d2d(ctx.handle, C.c_void_p(heap.data_ptr()), C.c_void_p(out.data), hb,
                                              ctx.stream_ptr()))
            ctx.sync()
            _lib.check(ctx.lib.vxg_free(ctx.handle, C.c_void_p(out.data)))
        res.data = heap[:hb]
        res.data_buffers = [(0, hb)]
    if out.validity:
        if vt is None or out.validity != vt.data_ptr():
            raise VortexError(7, "engine allocated validity for a non-nullable dtype")
        res.validity = vt[: (k + 7) // 8]
    ctx.sync()
    return res


def _kind_of_node(node: _lib.VxgArray) -> str:
    return {DTYPE["PRIMITIVE"]: "primitive", DTYPE["BOOL"]: "bool"}.get(node.dtype, "varbinview")


def alloc_canonical(ctx: Context, node: _lib.VxgArray, keep: list, table_cap: int = 4096):
    """Caller-allocated canonical output for the flattened array `node` (vxg_canonical_layout:
    values, or views + data + the per-chunk data-buffer table, and a validity bitmap when the
    dtype is nullable) -> (VxgCanonical, Canonical of device tensors).  Everything the output
    references is appended to `keep`."""
    import torch
    dev = torch.device("cuda", ctx.device)
    vb, db, nb = C.c_uint64(), C.c_uint64(), C.c_uint32()
    table = (_lib.VxgDataBuffer * table_cap)()
    _lib.check(ctx.lib.vxg_canonical_layout(ctx.handle, C.byref(node), C.byref(vb), C.byref(db), table,
                                            table_cap, C.byref(nb)))
    n = int(node.len)
    res = Canonical(_kind_of_node(node), n, PTYPES[node.ptype], binary=node.dtype == DTYPE["BINARY"])
    o = _lib.VxgCanonical()
    if node.dtype in (DTYPE["PRIMITIVE"], DTYPE["BOOL"]):
        vals = torch.empty(max(vb.value, 16), dtype=torch.uint8, device=dev)
        o.values = vals.data_ptr()
        res.values = vals[: vb.value]
    else:
        views = torch.empty(max(vb.value, 16), dtype=torch.uint8, device=dev)
        data = torch.empty(db.value + 16, dtype=torch.uint8, device=dev)
        o.views, o.data, o.data_bytes = views.data_ptr(), data.data_ptr(), db.value
        o.data_buffers, o.n_data_buffers, o.data_buffers_cap = table, nb.value, table_cap
        res.views, res.data = views[: vb.value], data[: db.value]
        res.data_buffers = [(int(table[k].offset), int(table[k].len)) for k in range(nb.value)]
        keep.append(table)
    if node.nullable:
        vt = torch.empty(((n + 31) // 32) * 4 + 4, dtype=torch.uint8, device=dev)
        o.validity = vt.data_ptr()
        res.validity = vt[: (n + 7) // 8]
    keep.append(res)
    return o, res


class Plan:
    """vxg_plan: the launches of canonicalizing `arrays` into preallocated outputs, recorded
    once as a HIP graph and replayed by launch() (one hipGraphLaunch; every kernel runs on
    every replay).  Outputs are allocated here with vxg_canonical_layout and exposed as
    Canonical objects; the device arrays must stay alive (and in place) with the plan.
    `arrays` are Array trees (device buffers) or already-flattened VxgArray nodes (e.g. the
    trees a vxg_file reader built over a file's bytes in HBM)."""

    def __init__(self, arrays: Sequence, ctx: Context, measure: bool = False):
        """measure=True: VXG_PLAN_MEASURE -- record both candidates and keep the faster (runs the
        decode several times at create; inputs must be resident and valid)."""
        self.ctx = ctx
        self.keep: list = []
        n = len(arrays)
        self.nodes = (_lib.VxgArray * max(n, 1))()
        self.outs = (_lib.VxgCanonical * max(n, 1))()
        self.results = []
        for i, a in enumerate(arrays):
            self.nodes[i] = a if isinstance(a, _lib.VxgArray) else flatten(a, self.keep)
            o, res = alloc_canonical(ctx, self.nodes[i], self.keep)
            self.outs[i] = o
            self.results.append(res)
        h = C.c_void_p()
        flags = _lib.PLAN_MEASURE if measure else 0
        _lib.check(ctx.lib.vxg_plan_create_ex(ctx.handle, self.nodes, self.outs, n, flags, C.byref(h)))
        self.handle = h
        # a nullable array whose validity turned out all-valid leaves out.validity NULL
        for i, res in enumerate(self.results):
            if res.validity is not None and not self.outs[i].validity:
                res.validity = None

    def info(self) -> dict:
        """vxg_plan_get_info: the kept graph's shape, the candidates' measured replay times and
        the create call's wall time."""
        i = _lib.VxgPlanInfo()
        _lib.check(self.ctx.lib.vxg_plan_get_info(self.handle, C.byref(i)))
        cands = [{"batched": bool(i.candidate_batched[c]), "ms": round(float(i.candidate_ms[c]), 4)}
                 for c in range(i.n_candidates)]
        for c in range(i.n_candidates):
            cands[c]["cost"] = int(i.candidate_cost[c])
        return {"batched": bool(i.batched), "branches": int(i.branches), "direct_nodes": int(i.direct_nodes),
                "candidates": cands, "selection": _lib.PLAN_SELECTION.get(int(i.selection), str(i.selection)),
                "create_ms": round(float(i.create_ms), 3)}

    def launch(self, sync: bool = False):
        _lib.check(self.ctx.lib.vxg_plan_launch(self.handle, self.ctx.stream_ptr()))
        if sync:
            self.ctx.sync()
        return self.results

    def close(self):
        if getattr(self, "handle", None):
            self.ctx.lib.vxg_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
