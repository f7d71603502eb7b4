"""GPU encoders: values resident in HBM -> Vortex array trees whose
buffers are device tensors, through the C ABI's encoder entry points (include/vortex_gpu.h).

Each function restates the same-named host encoder in `encode.py` (which the tests hold it
equal to, byte for byte) and the reference algorithm it cites:

  * `int_stats`            -- the compressor's statistics pass (stats/mod.rs:178-189, bit-width
                              frequencies of compute_stats), one HBM read on the GPU;
  * `best_bit_width`       -- compressors/bitpacked.rs:30-34 + bitpacking/compress.rs best_bit_width,
                              a host decision over the 65-entry GPU histogram;
  * `encode_bitpacked`     -- BitPackedArray::encode (bitpacking/compress.rs:16-41, 82-163): K15
                              FastLanes pack + ordered patch compaction;
  * `encode_for_bitpacked` -- for_compress (for/compress.rs:13-85) -> BitPacked, fused into one
                              K15 pass when no patches are taken;
  * `encode_alp`           -- ALPFloat::encode with find_best_exponents (alp/mod.rs:51-140) ->
                              FoR -> BitPacked, exceptions as Sparse patches (alp/compress.rs:38-59);
  * `fsst_train`           -- fsst_train_compressor (fsst/compress.rs:46-81): training stays on the
                              host, as Compressor::train does; only the trainer's sample of the
                              device column is gathered and copied back;
  * `encode_fsst`          -- fsst_compress_iter (fsst/compress.rs:83-129): K17 compresses every
                              string against the table on the GPU (codes VarBin with i32 offsets,
                              i32 uncompressed lengths).

The only host work is the choice of parameters from the statistics the GPU returns (and FSST's
table training on a bounded sample); no value passes through host memory.  There is no CPU fallback: without the HIP library this raises.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from . import arrays as A
from .arrays import DTYPE, ENC, NP_OF_PTYPE, PTYPE, VALIDITY, Array, ptype_width, unsigned_of


def _torch():
    import torch
    return torch


def _bytes(t):
    """Flat uint8 view of a contiguous device tensor."""
    torch = _torch()
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise A.VortexError(3, "GPU encoders take device tensors")
    return t.contiguous().view(torch.uint8).reshape(-1)


def _ptr(t) -> C.c_void_p:
    return C.c_void_p(t.data_ptr() if t.numel() else 0)


def _empty(ctx, nbytes: int):
    torch = _torch()
    # 16 bytes of slack so a zero-length buffer still has a valid device address
    t = torch.empty(max(nbytes, 0) + 16, dtype=torch.uint8, device=torch.device("cuda", ctx.device))
    return t[:nbytes]


def _from_bits(bits: int, ptype: str) -> int:
    return int(np.array([bits], dtype=np.uint64).astype(NP_OF_PTYPE[unsigned_of(ptype)]).view(NP_OF_PTYPE[ptype])[0])


@dataclass
class IntStats:
    n: int
    min: int
    max: int
    trailing_zeros: int
    bit_width_freq: list  # T + 1 entries: values of bit width 0..T (unsigned view)


def int_stats(ctx, values, ptype: str, n: int | None = None) -> IntStats:
    """vxg_compute_int_stats: min, max, min trailing zeros and bit-width frequencies."""
    b = _bytes(values)
    w = ptype_width(ptype)
    n = b.numel() // w if n is None else n
    st = _lib.VxgIntStats()
    _lib.check(ctx.lib.vxg_compute_int_stats(ctx.handle, PTYPE[ptype], _ptr(b), n, C.byref(st), ctx.stream_ptr()))
    T = 8 * w
    return IntStats(int(st.n), _from_bits(st.min_bits, ptype), _from_bits(st.max_bits, ptype),
                    int(st.trailing_zeros), [int(x) for x in st.bit_width_freq[: T + 1]])


def best_bit_width(freq: list, width: int) -> int:
    """best_bit_width (bitpacking/compress.rs): minimise packed bytes + (width + 4) bytes per
    patch; restates vxe_best_bit_width over the histogram."""
    bpe = width + 4
    n = sum(freq)
    best, best_cost, num_packed = 0, n * bpe, 0
    for bw, c in enumerate(freq):
        num_packed += c
        cost = (n - num_packed) * bpe + (bw * n + 7) // 8
        if cost < best_cost:
            best, best_cost = bw, cost
    return best


def min_patchless_bit_width(freq: list) -> int:
    return max((bw for bw, c in enumerate(freq) if c), default=0)


def bitpack(ctx, values, ptype: str, bit_width: int, n: int | None = None):
    """vxg_bitpack (K15): FastLanes-packed bytes, ceil(n / 1024) * 128 * bit_width long."""
    b = _bytes(values)
    n = b.numel() // ptype_width(ptype) if n is None else n
    out = _empty(ctx, ((n + 1023) // 1024) * 128 * bit_width)
    _lib.check(ctx.lib.vxg_bitpack(ctx.handle, PTYPE[ptype], bit_width, _ptr(b), n, _ptr(out), out.numel(),
                                   ctx.stream_ptr()))
    return out


def for_encode(ctx, values, ptype: str, reference: int, shift: int, n: int | None = None):
    """vxg_for_encode: the FoR-encoded child ((v - reference) >> shift) as unsigned(ptype) bytes."""
    b = _bytes(values)
    w = ptype_width(ptype)
    n = b.numel() // w if n is None else n
    out = _empty(ctx, n * w)
    ref_bits = int(np.array([reference], dtype=NP_OF_PTYPE[ptype]).view(NP_OF_PTYPE[unsigned_of(ptype)])[0])
    _lib.check(ctx.lib.vxg_for_encode(ctx.handle, PTYPE[ptype], _ptr(b), n, ref_bits, shift, _ptr(out),
                                      ctx.stream_ptr()))
    return out


def gather_patches(ctx, values, ptype: str, bit_width: int, count: int, n: int | None = None):
    """vxg_gather_patches (bitpacking/compress.rs:138-163): (u64 indices, values) of the
    elements wider than bit_width, in index order; `count` from the histogram."""
    b = _bytes(values)
    w = ptype_width(ptype)
    n = b.numel() // w if n is None else n
    idx, vals = _empty(ctx, 8 * count), _empty(ctx, w * count)
    got = C.c_uint64()
    _lib.check(ctx.lib.vxg_gather_patches(ctx.handle, PTYPE[ptype], bit_width, _ptr(b), n, _ptr(idx), _ptr(vals),
                                          count, C.byref(got), ctx.stream_ptr()))
    if got.value != count:
        raise A.VortexError(3, f"gather_patches: {got.value} patches, histogram said {count}")
    return idx, vals


def _primitive(buf, ptype: str, n: int, validity: str = "NON_NULLABLE") -> Array:
    return Array(ENC["PRIMITIVE"], n, DTYPE["PRIMITIVE"], ptype, validity != "NON_NULLABLE", VALIDITY[validity],
                 {}, [buf])


def _bitpacked(packed, ptype: str, bit_width: int, n: int, patches: Array | None) -> Array:
    return Array(ENC["FL_BITPACKED"], n, DTYPE["PRIMITIVE"], ptype, False, VALIDITY["NON_NULLABLE"],
                 {"bit_width": bit_width, "offset": 0, "has_patches": patches is not None}, [packed],
                 [patches] if patches is not None else [])


def _patch_indices(ctx, idx, count: int, length: int) -> Array:
    """Patch positions as the host encoders store them: BitPacked u64 at the width of the
    largest index (a sorted list, so the last one), no patches of their own."""
    last = int(idx[-8:].view(_torch().int64).item()) if count else 0
    iw = max(1, last.bit_length())
    if iw >= 64:
        return _primitive(idx, "u64", count)
    return _bitpacked(bitpack(ctx, idx, "u64", iw, count), "u64", iw, count, None)


def encode_bitpacked(ctx, values, ptype: str, bit_width: int | None = None, allow_patches: bool = True,
                     stats: IntStats | None = None) -> Array:
    """BitPackedArray::encode of an unsigned device array (encode.encode_bitpacked)."""
    if ptype[0] != "u":
        raise A.VortexError(6, f"expected type: uint but instead got {ptype}")
    w = ptype_width(ptype)
    n = _bytes(values).numel() // w
    st = stats or int_stats(ctx, values, ptype, n)
    if bit_width is None:
        bit_width = best_bit_width(st.bit_width_freq, w) if allow_patches else min_patchless_bit_width(st.bit_width_freq)
    if bit_width >= 8 * w:
        raise A.VortexError(3, "Cannot pack -- specified bit width is greater than or equal to raw bit width")
    packed = bitpack(ctx, values, ptype, bit_width, n)
    count = sum(st.bit_width_freq[bit_width + 1:])
    patches = None
    if count:
        idx, pv = gather_patches(ctx, values, ptype, bit_width, count, n)
        patches = A.sparse(_patch_indices(ctx, idx, count, n), _primitive(pv, ptype, count, "ALL_VALID"), n)
    return _bitpacked(packed, ptype, bit_width, n, patches)


def encode_for_bitpacked(ctx, values, ptype: str, allow_patches: bool = True) -> Array:
    """FoR -> BitPacked cascade (encode.encode_for_bitpacked; compressors/for.rs:53-88)."""
    w, T = ptype_width(ptype), 8 * ptype_width(ptype)
    n = _bytes(values).numel() // w
    st = int_stats(ctx, values, ptype, n)
    if n == 0:
        st.trailing_zeros = T
    ref, shift = (st.min if n else 0), st.trailing_zeros
    if shift >= T:
        return A.constant(0, n, ptype)
    up = unsigned_of(ptype)
    ref_bits = int(np.array([ref], dtype=NP_OF_PTYPE[ptype]).view(NP_OF_PTYPE[up])[0])
    max_bits = int(np.array([st.max], dtype=NP_OF_PTYPE[ptype]).view(NP_OF_PTYPE[up])[0])
    raw = (max_bits - ref_bits) & ((1 << T) - 1)
    span = raw >> shift
    # (v - min) never wraps the signed type when max - min fits in T - 1 bits, so the arithmetic
    # shift of a signed ptype equals the logical one and the encoded maximum is `span`
    fits = ptype[0] == "u" or shift == 0 or raw < (1 << (T - 1))
    if not allow_patches and fits and span.bit_length() < T:
        W = span.bit_length()  # fused K15 FoR+pack: one read of the values, no encoded copy
        packed = _empty(ctx, ((n + 1023) // 1024) * 128 * W)
        _lib.check(ctx.lib.vxg_for_bitpack(ctx.handle, PTYPE[ptype], ref_bits, shift, W, _ptr(_bytes(values)), n,
                                           _ptr(packed), packed.numel(), ctx.stream_ptr()))
        return A.frame_of_reference(_bitpacked(packed, up, W, n, None), ref, shift, ptype)
    enc = for_encode(ctx, values, ptype, ref, shift, n)
    est = int_stats(ctx, enc, up, n)
    if min_patchless_bit_width(est.bit_width_freq) >= T:  # encoded values need the full width
        return A.frame_of_reference(_primitive(enc, up, n), ref, shift, ptype)
    return A.frame_of_reference(encode_bitpacked(ctx, enc, up, allow_patches=allow_patches, stats=est), ref, shift,
                                ptype)


def alp_encode(ctx, values, ptype: str):
    """vxg_alp_encode -> (e, f, encoded device bytes, patch index bytes, patch value bytes, count)."""
    if ptype not in ("f32", "f64"):
        raise A.VortexError(3, "ALP can only encode f32 and f64")
    b = _bytes(values)
    w = ptype_width(ptype)
    n = b.numel() // w
    enc = _empty(ctx, n * w)
    e, f, got = C.c_uint8(), C.c_uint8(), C.c_uint64()
    cap = max(1024, n // 16)
    while True:
        idx, pv = _empty(ctx, 8 * cap), _empty(ctx, w * cap)
        _lib.check(ctx.lib.vxg_alp_encode(ctx.handle, PTYPE[ptype], _ptr(b), n, C.byref(e), C.byref(f), _ptr(enc),
                                          _ptr(idx), _ptr(pv), cap, C.byref(got), ctx.stream_ptr()))
        if got.value <= cap:
            break
        cap = int(got.value)  # more exceptions than the first guess: encode again with room for all
    m = int(got.value)
    return int(e.value), int(f.value), enc, idx[: 8 * m], pv[: w * m], m


def encode_alp(ctx, values, ptype: str) -> Array:
    """alp_encode + the compressor cascade ALP -> FoR -> BitPacked (encode.encode_alp)."""
    e, f, enc, idx, pv, m = alp_encode(ctx, values, ptype)
    n = _bytes(values).numel() // ptype_width(ptype)
    patches = None
    if m:
        patches = A.sparse(_patch_indices(ctx, idx, m, n), _primitive(pv, ptype, m, "ALL_VALID"), n)
    ip = {"f32": "i32", "f64": "i64"}[ptype]
    return A.alp(encode_for_bitpacked(ctx, enc, ip, allow_patches=True), e, f, patches)


def _offsets_host(offsets, offs_ptype: str, n: int) -> np.ndarray:
    b = _bytes(offsets)[: (n + 1) * ptype_width(offs_ptype)]
    return b.cpu().numpy().view(NP_OF_PTYPE[offs_ptype]).astype(np.int64)


def fsst_train(ctx, offsets, offs_ptype: str, data, n: int):
    """The host trainer (encode.cpp vxe_fsst_train) over exactly the strings it samples: every
    (n // 20000)-th string until 1 MiB is read.  Only those strings are gathered on the device
    and copied back; the table equals the one trained on the whole column in host memory.
    -> (symbols u64[k], lengths u8[k]) host arrays."""
    torch = _torch()
    from .encode import _lib_enc, _p
    offs = _offsets_host(offsets, offs_ptype, n)
    step = n // 20000 if n > 20000 else 1
    picks, sampled = [], 0
    for i in range(0, n, step):
        if sampled >= (1 << 20):
            break
        picks.append(i)
        sampled += int(offs[i + 1] - offs[i])
    picks = np.array(picks, dtype=np.int64)
    lens = (offs[picks + 1] - offs[picks]) if picks.size else np.zeros(0, np.int64)
    new_offs = np.zeros(picks.size + 1, np.int64)
    np.cumsum(lens, out=new_offs[1:])
    if new_offs[-1]:
        idx = np.repeat(offs[picks] - new_offs[:-1], lens) + np.arange(new_offs[-1])
        heap = _bytes(data)[torch.from_numpy(idx).to(_bytes(data).device)].cpu().numpy()
    else:
        heap = np.zeros(1, np.uint8)
    t = _lib.VxeFsstTable()
    _lib_enc().vxe_fsst_train(_p(heap), _p(new_offs), picks.size, C.byref(t))
    k = int(t.n_symbols)
    return np.array(list(t.symbols)[:k], dtype=np.uint64), np.array(list(t.lens)[:k], dtype=np.uint8)


def fsst_compress(ctx, offsets, offs_ptype: str, data, n: int, symbols, lengths, validity=None):
    """vxg_fsst_compress (K17): -> (codes, code_offsets i32[n + 1], uncompressed_lengths i32[n]),
    device tensors (codes trimmed to the bytes written)."""
    torch = _torch()
    d = _bytes(data)
    syms = np.ascontiguousarray(symbols, dtype=np.uint64)
    slen = np.ascontiguousarray(lengths, dtype=np.uint8)
    cap = 2 * d.numel()
    codes = _empty(ctx, cap)
    coffs = _empty(ctx, 4 * (n + 1))
    ulens = _empty(ctx, 4 * n)
    got = C.c_uint64()
    vb = _ptr(_bytes(validity)) if validity is not None else C.c_void_p(0)
    _lib.check(ctx.lib.vxg_fsst_compress(ctx.handle, syms.ctypes.data_as(C.c_void_p), slen.ctypes.data_as(C.c_void_p),
                                         syms.size, PTYPE[offs_ptype], _ptr(_bytes(offsets)), _ptr(d), d.numel(), vb,
                                         n, _ptr(codes), cap, _ptr(coffs), _ptr(ulens), C.byref(got), ctx.stream_ptr()))
    return codes[: got.value], coffs, ulens


def encode_fsst(ctx, offsets, offs_ptype: str, data, n: int, validity=None, table=None, utf8: bool = True) -> Array:
    """fsst_compress (fsst/compress.rs:19-44) of a device-resident VarBin (offsets + bytes,
    optional LSB validity bits): the table is trained on the host (fsst_train) unless given,
    every string is compressed on the GPU.  -> FSSTArray(symbols, symbol_lengths,
    codes = VarBin(i32 offsets, binary), uncompressed_lengths i32) with device buffers, the
    tree encode.encode_fsst_from_heap(compress_children=False) builds on the host."""
    torch = _torch()
    dev = torch.device("cuda", ctx.device)
    symbols, lengths = table if table is not None else fsst_train(ctx, offsets, offs_ptype, data, n)
    codes, coffs, ulens = fsst_compress(ctx, offsets, offs_ptype, data, n, symbols, lengths, validity)
    k = int(np.asarray(symbols).size)
    sym_t = torch.from_numpy(np.ascontiguousarray(symbols, dtype=np.uint64).view(np.uint8).copy()).to(dev)
    len_t = torch.from_numpy(np.ascontiguousarray(lengths, dtype=np.uint8).copy()).to(dev)
    code_vb = A.varbin(_primitive(coffs, "i32", n + 1), _primitive(codes, "u8", int(codes.numel())), utf8=False)
    if validity is not None:
        vbits = _bytes(validity)
        mask = np.unpackbits(vbits.cpu().numpy(), bitorder="little")[:n].astype(bool)
        if not mask.all():
            code_vb = A.varbin(_primitive(coffs, "i32", n + 1), _primitive(codes, "u8", int(codes.numel())),
                               utf8=False, validity=mask)
    return A.fsst(_primitive(sym_t, "u64", k), _primitive(len_t, "u8", k), code_vb, _primitive(ulens, "i32", n),
                  utf8=utf8)
