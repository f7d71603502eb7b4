"""Encoders: numpy data -> Vortex array trees (host buffers), via libvortex_enc.so.

These restate the reference encoders (bitpack_encode, for_compress, alp_encode, dict_encode,
delta_compress, runend_encode, zigzag_encode, RDEncoder, FSST compress) so the decode engine is
fed exactly the layouts the reference writes, and compose them into the cascades the
reference's sampling compressor produces (vortex-sampling-compressor/src/compressors/*):
  Dict -> codes BitPacked;  ALP -> FoR -> BitPacked (+Sparse patches);
  BitPacked patches -> Sparse(indices BitPacked u64, values Primitive);
  FSST -> codes VarBin(offsets FoR/BitPacked), lengths FoR/BitPacked.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import _lib
from . import arrays as A
from .arrays import NP_OF_PTYPE, PTYPE, PTYPE_OF_NP, Array, ptype_width


def _p(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


def _lib_enc():
    return _lib.enc_lib()


def bit_width_of(v: int) -> int:
    return int(v).bit_length()


def bitpack_buffer(values: np.ndarray, bit_width: int) -> np.ndarray:
    """bitpack_primitive (bitpacking/compress.rs:82-137) -> packed bytes."""
    v = np.ascontiguousarray(values)
    if v.dtype.kind != "u":
        v = v.view(np.dtype(f"u{v.dtype.itemsize}"))
    n = v.size
    out = np.zeros(((n + 1023) // 1024) * 128 * bit_width + 16, dtype=np.uint8)
    nbytes = _lib_enc().vxe_bitpack(PTYPE[PTYPE_OF_NP[v.dtype]], bit_width, _p(v), n, _p(out))
    return out[:nbytes]


def encode_bitpacked(values, bit_width: Optional[int] = None, allow_patches: bool = True,
                     compress_patch_indices: bool = True, offset: int = 0,
                     validity=None) -> Array:
    """BitPackedArray::encode (bitpacking/mod.rs:190-196, compress.rs:16-41) with the
    compressor's bit-width choice (compressors/bitpacked.rs:30-34).  `offset` > 0 builds the
    sliced form (a BitPacked array whose first `offset` packed values are skipped)."""
    v = np.ascontiguousarray(values)
    p = PTYPE_OF_NP[v.dtype]
    if p[0] != "u":
        raise A.VortexError(6, f"expected type: uint but instead got {p}")
    lib = _lib_enc()
    full = np.concatenate([np.zeros(offset, dtype=v.dtype), v]) if offset else v
    if bit_width is None:
        fn = lib.vxe_best_bit_width if allow_patches else lib.vxe_min_patchless_bit_width
        bit_width = int(fn(PTYPE[p], _p(full), full.size))
    if bit_width >= 8 * v.dtype.itemsize:
        raise A.VortexError(3, "Cannot pack -- specified bit width is greater than or equal to raw bit width")
    packed = bitpack_buffer(full, bit_width)
    patches = None
    cap = v.size
    idx = np.zeros(max(cap, 1), dtype=np.uint64)
    pv = np.zeros(max(cap, 1), dtype=v.dtype)
    n_exc = int(lib.vxe_gather_patches(PTYPE[p], bit_width, _p(v), v.size, _p(idx), _p(pv), cap))
    if n_exc:
        idx, pv = idx[:n_exc], pv[:n_exc]
        if compress_patch_indices:
            iw = max(1, bit_width_of(int(idx.max())))
            ind = encode_bitpacked(idx, bit_width=iw, allow_patches=False) if iw < 64 else A.primitive(idx)
        else:
            ind = A.primitive(idx)
        # gather_patches (bitpacking/compress.rs:138-163): values PrimitiveArray with Validity::AllValid
        patches = A.sparse(ind, A.primitive(pv, validity="ALL_VALID"), v.size)
    return A.bitpacked(packed, p, bit_width, v.size, offset=offset, patches=patches, validity=validity)


def for_compress(values) -> tuple[np.ndarray, int, int]:
    """for_compress (for/compress.rs:13-85) -> (encoded unsigned, reference, shift)."""
    v = np.ascontiguousarray(values)
    p = PTYPE_OF_NP[v.dtype]
    enc = np.zeros(v.size, dtype=NP_OF_PTYPE[A.unsigned_of(p)])
    ref, sh = C.c_uint64(), C.c_uint()
    const = _lib_enc().vxe_for_compress(PTYPE[p], _p(v), v.size, _p(enc), C.byref(ref), C.byref(sh))
    ref_val = np.array([ref.value], dtype=np.uint64).astype(NP_OF_PTYPE[A.unsigned_of(p)]).view(v.dtype)[0]
    return enc, int(ref_val), int(sh.value) if not const else int(sh.value)


def encode_for_bitpacked(values, allow_patches: bool = True) -> Array:
    """FoR -> BitPacked cascade (compressors/for.rs:53-88 + bitpacked.rs)."""
    v = np.ascontiguousarray(values)
    p = PTYPE_OF_NP[v.dtype]
    enc, ref, shift = for_compress(v)
    if shift >= 8 * v.dtype.itemsize:
        return A.constant(0, v.size, p)
    child = encode_bitpacked(enc, allow_patches=allow_patches) if bit_width_of(int(enc.max(initial=0))) < 8 * v.dtype.itemsize else A.primitive(enc)
    return A.frame_of_reference(child, ref, shift, p)


def zigzag_encode(values) -> np.ndarray:
    """zigzag_encode_primitive (zigzag/compress.rs:24-33): the unsigned encoded words."""
    v = np.ascontiguousarray(values)
    p = PTYPE_OF_NP[v.dtype]
    out = np.zeros(v.size, dtype=NP_OF_PTYPE[A.unsigned_of(p)])
    _lib_enc().vxe_zigzag_encode(PTYPE[p], _p(v), v.size, _p(out))
    return out


def encode_zigzag(values) -> Array:
    """ZigZag -> BitPacked (zigzag/compress.rs:10-33, compressors/zigzag.rs)."""
    return A.zigzag(encode_bitpacked(zigzag_encode(values)))


def alp_encode(values) -> tuple[int, int, np.ndarray, np.ndarray, np.ndarray]:
    """ALPFloat::encode with find_best_exponents (alp/mod.rs:51-140) -> (e, f, encoded,
    patch positions, patch values)."""
    v = np.ascontiguousarray(values)
    n = v.size
    e, f = C.c_uint8(), C.c_uint8()
    if v.dtype == np.float64:
        enc = np.zeros(n, dtype=np.int64)
        idx = np.zeros(max(n, 1), dtype=np.uint64)
        pv = np.zeros(max(n, 1), dtype=np.float64)
        m = _lib_enc().vxe_alp_encode_f64(_p(v), n, C.byref(e), C.byref(f), _p(enc), _p(idx), _p(pv), n)
    elif v.dtype == np.float32:
        enc = np.zeros(n, dtype=np.int32)
        idx = np.zeros(max(n, 1), dtype=np.uint64)
        pv = np.zeros(max(n, 1), dtype=np.float32)
        m = _lib_enc().vxe_alp_encode_f32(_p(v), n, C.byref(e), C.byref(f), _p(enc), _p(idx), _p(pv), n)
    else:
        raise A.VortexError(3, "ALP can only encode f32 and f64")
    return e.value, f.value, enc, idx[:m], pv[:m]


def encode_alp(values, cascade: bool = True) -> Array:
    """alp_encode (alp/compress.rs:48-59) + the compressor cascade ALP -> FoR -> BitPacked."""
    v = np.ascontiguousarray(values)
    e, f, enc, idx, pv = alp_encode(v)
    patches = None
    if idx.size:
        iw = max(1, bit_width_of(int(idx.max())))
        ind = encode_bitpacked(idx, bit_width=iw, allow_patches=False) if cascade and iw < 64 else A.primitive(idx)
        # alp/compress.rs:38-45: exception values PrimitiveArray with Validity::AllValid
        patches = A.sparse(ind, A.primitive(pv, validity="ALL_VALID"), v.size)
    child = encode_for_bitpacked(enc, allow_patches=True) if cascade else A.primitive(enc)
    return A.alp(child, e, f, patches)


def encode_alprd(values) -> Array:
    """RDEncoder::new + encode (alp_rd/mod.rs:140-250)."""
    v = np.ascontiguousarray(values)
    n = v.size
    rbw, dl = C.c_uint8(), C.c_uint8()
    d = np.zeros(8, dtype=np.uint16)
    left = np.zeros(n, dtype=np.uint16)
    ep = np.zeros(max(n, 1), dtype=np.uint64)
    ex = np.zeros(max(n, 1), dtype=np.uint16)
    if v.dtype == np.float64:
        right = np.zeros(n, dtype=np.uint64)
        m = _lib_enc().vxe_alprd_encode_f64(_p(v), n, C.byref(rbw), _p(d), C.byref(dl), _p(left), _p(right), _p(ep), _p(ex), n)
        p = "f64"
    else:
        right = np.zeros(n, dtype=np.uint32)
        m = _lib_enc().vxe_alprd_encode_f32(_p(v), n, C.byref(rbw), _p(d), C.byref(dl), _p(left), _p(right), _p(ep), _p(ex), n)
        p = "f32"
    lbw = max(1, bit_width_of(int(dl.value) - 1))
    left_a = encode_bitpacked(left, bit_width=lbw, allow_patches=False)
    right_a = encode_bitpacked(right, bit_width=rbw.value, allow_patches=False)
    exc = None
    if m:
        ep, ex = ep[:m], ex[:m]
        bw = max(1, bit_width_of(int(ep.max())))
        # alp_rd/mod.rs:235-236: exceptions with Validity::AllValid
        exc = A.sparse(encode_bitpacked(ep, bit_width=bw, allow_patches=False), A.primitive(ex, validity="ALL_VALID"), n)
    return A.alp_rd(p, left_a, list(d[: dl.value]), right_a, rbw.value, exc)


def dict_encode(values) -> tuple[np.ndarray, np.ndarray]:
    """dict_encode_typed_primitive (dict/compress.rs:33-86) -> (codes u64, values)."""
    v = np.ascontiguousarray(values)
    codes = np.zeros(v.size, dtype=np.uint64)
    dv = np.zeros(v.size, dtype=v.dtype)
    nd = _lib_enc().vxe_dict_encode(v.dtype.itemsize, _p(v), v.size, _p(codes), _p(dv), v.size)
    return codes, dv[:nd]


def encode_dict(values, bitpack_codes: bool = True) -> Array:
    codes, dv = dict_encode(values)
    c = encode_bitpacked(codes, allow_patches=False) if bitpack_codes else A.primitive(codes)
    return A.dict_array(A.primitive(dv), c)


def dict_encode_nullable(values, validity) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """dict_encode_typed_primitive over a NULLABLE array (dict/compress.rs:39-86): the dictionary
    starts with a null slot (zero value, invalid) and every null row gets code 0 -> (codes u64,
    values, values validity)."""
    v = np.ascontiguousarray(values)
    valid = np.asarray(validity, dtype=bool)
    pos: dict = {}
    dv = [v.dtype.type(0)]
    codes = np.zeros(v.size, dtype=np.uint64)
    for i in range(v.size):
        if valid[i]:
            key = v[i].tobytes()
            if key not in pos:
                pos[key] = len(dv)
                dv.append(v[i])
            codes[i] = pos[key]
    vvalid = np.ones(len(dv), dtype=bool)
    vvalid[0] = False
    return codes, np.array(dv, dtype=v.dtype), vvalid


def encode_dict_nullable(values, validity, bitpack_codes: bool = True) -> Array:
    codes, dv, vvalid = dict_encode_nullable(values, validity)
    c = encode_bitpacked(codes, allow_patches=False) if bitpack_codes else A.primitive(codes)
    return A.dict_array(A.primitive(dv, validity=vvalid), c)


def encode_dict_strings_nullable(strings: Sequence[Optional[bytes]], utf8: bool = True) -> Array:
    """dict_encode_typed_varbin over a nullable VarBin (dict/compress.rs:118-143): slot 0 is the
    null entry (empty bytes, invalid), null rows get code 0, u32 offsets."""
    pos: dict = {}
    codes = np.zeros(len(strings), dtype=np.uint64)
    uniq: list = []
    for i, s in enumerate(strings):
        if s is not None:
            if s not in pos:
                pos[s] = len(uniq) + 1
                uniq.append(s)
            codes[i] = pos[s]
    heap, offs, _ = strings_to_heap([b""] + uniq)
    vvalid = np.ones(len(uniq) + 1, dtype=bool)
    vvalid[0] = False
    values = A.varbin(A.primitive(offs.astype(np.uint32)), A.primitive(heap), utf8=utf8, validity=vvalid)
    return A.dict_array(values, encode_bitpacked(codes, allow_patches=False))


def encode_delta(values, bitpack_deltas: bool = True) -> Array:
    """DeltaArray::try_from_primitive_array (delta/mod.rs:72-78, compress.rs:14-98)."""
    v = np.ascontiguousarray(values)
    p = PTYPE_OF_NP[v.dtype]
    if p[0] != "u":
        raise A.VortexError(6, "Delta encodes unsigned integers")
    lanes = 1024 // (8 * v.dtype.itemsize)
    nb = (v.size // 1024) * lanes + (1 if v.size % 1024 else 0)
    bases = np.zeros(max(nb, 1), dtype=v.dtype)
    deltas = np.zeros(max(v.size, 1), dtype=v.dtype)
    _lib_enc().vxe_delta_compress(PTYPE[p], _p(v), v.size, _p(bases), _p(deltas))
    bases, deltas = bases[:nb], deltas[: v.size]
    d = encode_bitpacked(deltas, allow_patches=False) if bitpack_deltas and v.size and \
        bit_width_of(int(deltas.max())) < 8 * v.dtype.itemsize else A.primitive(deltas)
    return A.delta(A.primitive(bases), d)


def runend_encode(values) -> tuple[np.ndarray, np.ndarray]:
    v = np.ascontiguousarray(values)
    ends = np.zeros(max(v.size, 1), dtype=np.uint64)
    rv = np.zeros(max(v.size, 1), dtype=v.dtype)
    r = _lib_enc().vxe_runend_encode(v.dtype.itemsize, _p(v), v.size, _p(ends), _p(rv))
    return ends[:r], rv[:r]


def encode_runend(values, bitpack_ends: bool = True, compress_values: bool = False) -> Array:
    """runend_encode (runend/compress.rs:15-93) + the compressor cascade (compressors/runend.rs:
    45-70: ends -> BitPacked, values -> FoR/BitPacked when `compress_values`)."""
    v = np.ascontiguousarray(values)
    ends, rv = runend_encode(v)
    e = encode_bitpacked(ends, allow_patches=False) if bitpack_ends and ends.size else A.primitive(ends)
    vals = encode_for_bitpacked(rv) if compress_values and rv.size and rv.dtype.kind in "iu" else A.primitive(rv)
    return A.run_end(e, vals, length=v.size)


def runend_bool_encode(mask) -> tuple[np.ndarray, bool]:
    """runend_bool_encode_slice (encodings/runend-bool/src/compress.rs:16-41): the ends of the
    alternating runs (u64) and the value of the first run.  No set bit: ([len], false)."""
    m = np.asarray(mask, dtype=bool)
    n = m.size
    if not m.any():
        return np.array([n], dtype=np.uint64), False
    flips = np.flatnonzero(m[1:] != m[:-1]) + 1  # where the value changes = run ends
    return np.concatenate([flips, [n]]).astype(np.uint64), bool(m[0])


def encode_runend_bool(mask, bitpack_ends: bool = False, validity=None) -> Array:
    """RunEndBoolArray::try_new (runend-bool/src/array.rs:36-39) over runend_bool_encode; the
    ends optionally BitPacked (a compressor cascade on the ends child)."""
    ends, start = runend_bool_encode(mask)
    e = encode_bitpacked(ends, allow_patches=False) if bitpack_ends else A.primitive(ends)
    return A.run_end_bool(e, start, length=int(np.asarray(mask).size), validity=validity)


def roaring_bool_encode(mask) -> np.ndarray:
    """roaring_bool_encode (roaring/src/boolean/compress.rs:7-14): croaring Native bytes."""
    m = np.asarray(mask, dtype=bool)
    bits = np.packbits(m, bitorder="little")
    if bits.size == 0:
        bits = np.zeros(1, np.uint8)
    lib = _lib_enc()
    need = int(lib.vxe_roaring_bool_encode(_p(bits), m.size, None, 0))
    out = np.zeros(max(need, 1), np.uint8)
    lib.vxe_roaring_bool_encode(_p(bits), m.size, _p(out), out.size)
    return out[:need]


def encode_roaring_bool(mask) -> Array:
    """RoaringBoolArray::encode (roaring/src/boolean/mod.rs:74-80)."""
    m = np.asarray(mask, dtype=bool)
    return A.roaring_bool(roaring_bool_encode(m), m.size)


def encode_dict_strings(strings: Sequence[bytes], utf8: bool = True) -> Array:
    """dict_encode_varbin (dict/compress.rs:88-143): values = VarBin of the distinct strings in
    first-appearance order (i32 offsets), codes u64 -> BitPacked (compressors/dict.rs)."""
    pos: dict = {}
    codes = np.fromiter((pos.setdefault(s, len(pos)) for s in strings), dtype=np.uint64, count=len(strings))
    uniq = list(pos.keys())
    heap, offs, _ = strings_to_heap(uniq)
    values = A.varbin(A.primitive(offs.astype(np.int32)), A.primitive(heap), utf8=utf8)
    return A.dict_array(values, encode_bitpacked(codes, allow_patches=False))


def strings_to_heap(strings: Sequence[Optional[bytes]]) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """-> (heap u8, offsets i64[n+1], valid bool[n]); None entries are null, empty."""
    lens = np.fromiter((0 if s is None else len(s) for s in strings), dtype=np.int64, count=len(strings))
    offs = np.zeros(len(strings) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    heap = np.frombuffer(b"".join(s for s in strings if s is not None), dtype=np.uint8).copy()
    valid = np.fromiter((s is not None for s in strings), dtype=bool, count=len(strings))
    return heap, offs, valid


def encode_fsst_from_heap(heap: np.ndarray, offsets: np.ndarray, valid: Optional[np.ndarray] = None,
                          compress_children: bool = True) -> Array:
    """fsst_compress (fsst/compress.rs:83-129) + compressor cascade (compressors/fsst.rs:80-120):
    codes VarBin with i32 offsets, i32 uncompressed lengths."""
    heap = np.ascontiguousarray(heap, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    n = offsets.size - 1
    t = _lib.VxeFsstTable()
    lib = _lib_enc()
    lib.vxe_fsst_train(_p(heap), _p(offsets), n, C.byref(t))
    cap = 2 * int(heap.size) + 16
    codes = np.zeros(cap, dtype=np.uint8)
    coffs = np.zeros(n + 1, dtype=np.int32)
    nc = lib.vxe_fsst_compress(C.byref(t), _p(heap), _p(offsets), n, _p(codes), cap, _p(coffs))
    if nc == 2 ** 64 - 1:
        raise A.VortexError(2, "FSST code buffer overflow")
    codes = codes[:nc]
    lens = np.diff(offsets).astype(np.int32)
    syms = np.array(list(t.symbols)[: t.n_symbols], dtype=np.uint64)
    slen = np.array(list(t.lens)[: t.n_symbols], dtype=np.uint8)
    if compress_children:
        offs_a = encode_for_bitpacked(coffs, allow_patches=False)
        lens_a = encode_for_bitpacked(lens, allow_patches=False)
    else:
        offs_a, lens_a = A.primitive(coffs), A.primitive(lens)
    code_vb = A.varbin(offs_a, A.primitive(codes), utf8=False,
                       validity=None if valid is None or valid.all() else valid)
    return A.fsst(A.primitive(syms), A.primitive(slen), code_vb, lens_a)


def encode_fsst(strings: Sequence[Optional[bytes]], compress_children: bool = True) -> Array:
    heap, offs, valid = strings_to_heap(strings)
    return encode_fsst_from_heap(heap, offs, valid if not valid.all() else None, compress_children)


def encode_varbinview(strings: Sequence[Optional[bytes]], utf8: bool = True) -> Array:
    """VarBinViewArray::from_iter (varbinview/mod.rs:318-337 via arrow's GenericByteViewBuilder):
    one data buffer holding the non-inlined strings; views per arrow make_view (len <= 12
    inline, else [len][prefix][buffer 0][offset]); nulls are all-zero views."""
    n = len(strings)
    views = np.zeros((n, 16), dtype=np.uint8)
    parts, off = [], 0
    for i, st in enumerate(strings):
        if st is None:
            continue
        ln = len(st)
        views[i, :4] = np.frombuffer(np.uint32(ln).tobytes(), np.uint8)
        if ln <= 12:
            views[i, 4: 4 + ln] = np.frombuffer(st, np.uint8)
        else:
            views[i, 4:8] = np.frombuffer(st[:4], np.uint8)
            views[i, 12:16] = np.frombuffer(np.uint32(off).tobytes(), np.uint8)
            parts.append(st)
            off += ln
    data = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    valid = [s is not None for s in strings]
    return A.varbinview(views, [data], utf8=utf8, validity=None if all(valid) else valid)
