"""GPU encoders (vortex_amd/gpu_encode.py, C ABI vxg_bitpack / vxg_for_bitpack / vxg_for_encode /
vxg_gather_patches / vxg_compute_int_stats / vxg_alp_encode) against the host encoders
(vortex_amd/encode.py over libvortex_enc.so), byte for byte: the same tree, the same metadata,
the same packed buffers, the same patches — and decode(encode(x)) == x through the GPU decoder.
The host encoders are themselves pinned to the reference's ALP / bit-packing known answers
(tests/test_oracle.py, tests/golden/kat.json), which are replayed here on the GPU path.
"""
import json
import struct
from pathlib import Path

import numpy as np
import pytest

import vortex_amd as V
import vortex_amd.arrays as A
import vortex_amd.encode as E
import vortex_amd.gpu_encode as G
from oracle_tree import canon

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).resolve().parent / "golden"
KATS = {k["name"]: k for k in json.loads((GOLD / "kat.json").read_text())}
UT = {8: np.uint8, 16: np.uint16, 32: np.uint32, 64: np.uint64}
ST = {8: np.int8, 16: np.int16, 32: np.int32, 64: np.int64}
SIZES = [0, 1, 1023, 1024, 1025, 5000]


def dev(a: np.ndarray):
    import torch
    a = np.ascontiguousarray(a)
    t = torch.empty(max(a.nbytes, 16), dtype=torch.uint8, device="cuda:0")
    if a.nbytes:
        t[: a.nbytes].copy_(torch.from_numpy(a.view(np.uint8).reshape(-1).copy()))
    return t[: a.nbytes]


def host_bytes(b) -> bytes:
    if hasattr(b, "cpu"):
        return b.cpu().numpy().tobytes()
    return np.ascontiguousarray(b).view(np.uint8).tobytes()


def assert_same_tree(g: A.Array, h: A.Array, path="root"):
    assert (g.encoding, g.len, g.dtype, g.ptype, g.nullable, g.validity) == \
        (h.encoding, h.len, h.dtype, h.ptype, h.nullable, h.validity), path
    assert g.meta == h.meta, path
    assert len(g.buffers) == len(h.buffers), path
    for i, (gb, hb) in enumerate(zip(g.buffers, h.buffers)):
        assert host_bytes(gb) == host_bytes(hb), f"{path}.buffer[{i}]"
    assert len(g.children) == len(h.children), path
    for i, (gc, hc) in enumerate(zip(g.children, h.children)):
        assert_same_tree(gc, hc, f"{path}.child[{i}]")


def roundtrip(arr: A.Array, ctx, vals: np.ndarray):
    import torch
    res = V.canonicalize(arr.to(torch.device("cuda", 0)), ctx)
    assert res.numpy().tobytes() == np.ascontiguousarray(vals).tobytes()


# ------------------------------------------------------------------ statistics
@pytest.mark.parametrize("T", [8, 16, 32, 64])
@pytest.mark.parametrize("signed", [False, True])
def test_int_stats(ctx, T, signed):
    rng = np.random.default_rng(T + signed)
    dt = (ST if signed else UT)[T]
    for n in [1, 1000, 70_000]:
        v = rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, n, dtype=dt, endpoint=True)
        v[::7] &= dt(0x70)
        st = G.int_stats(ctx, dev(v), A.PTYPE_OF_NP[np.dtype(dt)])
        assert (st.n, st.min, st.max) == (n, int(v.min()), int(v.max()))
        u = v.view(UT[T]).astype(np.uint64)
        tz = [T if x == 0 else (int(x) & -int(x)).bit_length() - 1 for x in u]
        assert st.trailing_zeros == min(tz)
        bw = np.array([int(x).bit_length() for x in u])
        assert st.bit_width_freq == np.bincount(bw, minlength=T + 1).tolist()


# ------------------------------------------------------------------ K15 pack
@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_bitpack_every_width(ctx, T):
    rng = np.random.default_rng(100 + T)
    dt = UT[T]
    for W in range(0, T):
        for n in SIZES:
            v = (rng.integers(0, 2**63, n, dtype=np.uint64) & np.uint64((1 << W) - 1)).astype(dt)
            g = G.bitpack(ctx, dev(v), f"u{T}", W)
            assert host_bytes(g) == E.bitpack_buffer(v, W).tobytes(), (T, W, n)


@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_encode_bitpacked_with_patches(ctx, T):
    rng = np.random.default_rng(200 + T)
    dt = UT[T]
    for n in SIZES + [33_000]:
        v = rng.integers(0, 1 << min(T - 3, 12), n, dtype=np.uint64).astype(dt)
        if n:
            hot = rng.choice(n, max(1, n // 200), replace=False)
            v[hot] = np.iinfo(dt).max - rng.integers(0, 5, hot.size).astype(dt)
        for allow in (True, False):
            try:
                h = E.encode_bitpacked(v, allow_patches=allow)
            except A.VortexError as err:  # T-bit packing is refused by both encoders
                with pytest.raises(A.VortexError) as gerr:
                    G.encode_bitpacked(ctx, dev(v), f"u{T}", allow_patches=allow)
                assert gerr.value.args[0] == err.args[0]
                continue
            g = G.encode_bitpacked(ctx, dev(v), f"u{T}", allow_patches=allow)
            assert_same_tree(g, h)
            roundtrip(g, ctx, v)


def test_bitpacked_patch_max_kat(ctx):
    k = KATS["bitpacked_u64_w1_patch_max"]
    v = np.array(k["values"], dtype=np.uint64)
    h = E.encode_bitpacked(v, bit_width=1)
    g = G.encode_bitpacked(ctx, dev(v), "u64", bit_width=1)
    assert_same_tree(g, h)
    roundtrip(g, ctx, v)


# ------------------------------------------------------------------ FoR (+ fused pack)
def _for_cases(rng, dt, n):
    lo, hi = np.iinfo(dt).min, np.iinfo(dt).max
    yield rng.integers(lo, hi, n, dtype=dt, endpoint=True)                    # full range
    yield (rng.integers(-1000, 1000, n) * 8 + 77).astype(dt) if lo < 0 else \
        (rng.integers(0, 1000, n) * 8 + 77).astype(dt)                          # offset, no shift
    yield (rng.integers(0, 100, n) * 16).astype(dt)                           # shift 4
    yield np.full(n, 48, dt)                                                  # one value
    yield np.zeros(n, dt)                                                     # ConstantArray(0)
    if lo < 0 and n >= 2:
        w = np.where(np.arange(n) % 2 == 0, lo, hi - 1).astype(dt)            # signed wrap, shift 1
        yield w


@pytest.mark.parametrize("T", [8, 16, 32, 64])
@pytest.mark.parametrize("signed", [False, True])
def test_for_bitpacked(ctx, T, signed):
    rng = np.random.default_rng(300 + T + signed)
    dt = (ST if signed else UT)[T]
    p = A.PTYPE_OF_NP[np.dtype(dt)]
    for n in [1, 1025, 20_000]:
        for v in _for_cases(rng, dt, n):
            for allow in (True, False):
                h = E.encode_for_bitpacked(v, allow_patches=allow)
                g = G.encode_for_bitpacked(ctx, dev(v), p, allow_patches=allow)
                assert_same_tree(g, h)
                if g.encoding != A.ENC["CONSTANT"]:
                    roundtrip(g, ctx, v)


def test_for_encode_matches_host(ctx):
    rng = np.random.default_rng(9)
    for dt in (np.int8, np.int32, np.uint16, np.int64):
        v = rng.integers(np.iinfo(dt).min // 2, np.iinfo(dt).max // 2, 3000, dtype=dt) * 2
        enc, ref, shift = E.for_compress(v)
        g = G.for_encode(ctx, dev(v), A.PTYPE_OF_NP[np.dtype(dt)], ref, shift)
        assert host_bytes(g) == enc.tobytes()


# ------------------------------------------------------------------ ALP
def _f(bits_hex, ptype):
    fmt = "<f" if ptype == "f32" else "<d"
    return np.array([struct.unpack(fmt, bytes.fromhex(h))[0] for h in bits_hex],
                    dtype=np.float32 if ptype == "f32" else np.float64)


def assert_alp_same(ctx, vals, ptype):
    he, hf, henc, hidx, hpv = E.alp_encode(vals)
    ge, gf, genc, gidx, gpv, m = G.alp_encode(ctx, dev(vals), ptype)
    assert (ge, gf) == (he, hf)
    assert host_bytes(genc) == henc.tobytes()
    assert m == hidx.size
    assert host_bytes(gidx) == hidx.tobytes() and host_bytes(gpv) == hpv.tobytes()
    g = G.encode_alp(ctx, dev(vals), ptype)
    h = E.encode_alp(vals)
    assert_same_tree(g, h)
    # The reference finds exceptions with float `!=` (alp/mod.rs:194, 216): -0.0 == 0.0, so a
    # negative zero encodes as 0 and decodes as +0.0.  Bit-exact against the oracle's decode of
    # the same tree; value-exact (NaN at NaN) against the input.
    import torch
    got = V.canonicalize(g.to(torch.device("cuda", 0)), ctx).numpy()
    assert got.tobytes() == canon(h)[0].tobytes()
    assert np.array_equal(got, vals, equal_nan=True)


@pytest.mark.parametrize("name,ptype", [("alp_f32_constant_1025", "f32"), ("alp_f32_nullable", "f32"),
                                        ("alp_f64_patched", "f64"), ("alp_f32_close_fractional", "f32")])
def test_alp_kats(ctx, name, ptype):
    k = KATS[name]
    vals = _f(k["values_bits"], ptype)
    ge, gf, genc, _, _, _ = G.alp_encode(ctx, dev(vals), ptype)
    if "expect_e" in k:
        assert (ge, gf) == (k["expect_e"], k["expect_f"])
    if "expect_encoded" in k:
        assert np.frombuffer(host_bytes(genc), dtype=np.int32 if ptype == "f32" else np.int64).tolist() == \
            k["expect_encoded"]
    assert_alp_same(ctx, vals, ptype)


def test_alp_reference_doc_example(ctx):
    import math
    vals = np.array([1.234, 2.718, math.pi, 4.0])
    ge, gf, *_ = G.alp_encode(ctx, dev(vals), "f64")
    assert (ge, gf) == (16, 13)
    assert_alp_same(ctx, vals, "f64")


@pytest.mark.parametrize("n", [1, 31, 33, 1024, 100_000])
def test_alp_prices_f64(ctx, n):
    rng = np.random.default_rng(n)
    vals = np.round(rng.uniform(1, 100000, n) * 100) / 100
    if n > 10:
        vals[rng.choice(n, n // 1000 + 1, replace=False)] = rng.standard_normal(n // 1000 + 1) * 1e9
    assert_alp_same(ctx, vals, "f64")


def test_alp_f32_and_specials(ctx):
    rng = np.random.default_rng(5)
    vals = (np.round(rng.uniform(-500, 500, 50_000) * 10) / 10).astype(np.float32)
    assert_alp_same(ctx, vals, "f32")
    sp = np.round(rng.uniform(0, 100, 4096) * 100) / 100
    sp[[3, 100, 2000]] = [np.nan, np.inf, -np.inf]
    sp[[5, 6]] = [1e300, -0.0]
    assert_alp_same(ctx, sp, "f64")


def test_alp_many_exceptions_regrows_capacity(ctx):
    rng = np.random.default_rng(6)
    vals = rng.standard_normal(20_000)  # nearly every value is an exception
    vals[::2] = np.round(vals[::2] * 100) / 100
    assert_alp_same(ctx, vals, "f64")


# ------------------------------------------------------------------ K17 FSST compress
FSST_SENTENCES = [  # encodings/fsst/tests/fsst_tests.rs:19-35
    b"The Greeks never said that the limit could not he overstepped",
    b"They said it existed and that whoever dared to exceed it was mercilessly struck down",
    b"Nothing in present history can contradict them",
]


def _dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).reshape(-1).copy()).cuda()


def _fsst_gpu_vs_host(ctx, strings, offs_ptype="i64"):
    """GPU FSST (host-trained table from the device column's sample + K17 compress) against the
    host encoder (encode.encode_fsst_from_heap, plain children): the same table, byte-equal
    codes, i32 code offsets and i32 uncompressed lengths; then decode(encode(x)) == x through
    the K6/K7 canonicalize."""
    import torch
    heap, offs, valid = E.strings_to_heap(strings)
    has_nulls = not valid.all()
    host = E.encode_fsst_from_heap(heap, offs, valid if has_nulls else None, compress_children=False)
    n = len(strings)
    vbits = np.packbits(valid, bitorder="little") if has_nulls else None
    d_offs = _dev(offs.astype(A.NP_OF_PTYPE[offs_ptype]))
    d_heap = _dev(heap if heap.size else np.zeros(1, np.uint8))[: heap.size]
    arr = G.encode_fsst(ctx, d_offs, offs_ptype, d_heap, n, validity=_dev(vbits) if has_nulls else None)
    syms, slen, codes_vb, ulens = arr.children
    hsyms, hslen, hcodes_vb, hulens = host.children
    assert syms.buffers[0].cpu().numpy().tobytes() == np.ascontiguousarray(hsyms.buffers[0]).tobytes()
    assert slen.buffers[0].cpu().numpy().tobytes() == np.ascontiguousarray(hslen.buffers[0]).tobytes()
    assert codes_vb.children[0].buffers[0].cpu().numpy().tobytes() == \
        np.ascontiguousarray(hcodes_vb.children[0].buffers[0]).astype(np.int32).tobytes()
    assert codes_vb.children[1].buffers[0].cpu().numpy().tobytes() == \
        np.ascontiguousarray(hcodes_vb.children[1].buffers[0]).tobytes()
    assert ulens.buffers[0].cpu().numpy().tobytes() == np.ascontiguousarray(hulens.buffers[0]).astype(np.int32).tobytes()
    assert codes_vb.nullable == hcodes_vb.nullable
    res = V.canonicalize(arr.to(torch.device("cuda", 0)), ctx)
    views, _ = res.numpy()
    bufs = res.buffers()
    from oracle_tree import view_bytes
    for i in range(0, n, max(1, n // 5000)):
        if strings[i] is not None:
            assert view_bytes(views, bufs, i) == strings[i], i
    return arr


def test_fsst_compress_reference_sentences(ctx):
    """The reference's FSST test input (fsst_tests.rs:19-35), i32 and i64 offsets."""
    for op in ("i32", "i64"):
        _fsst_gpu_vs_host(ctx, FSST_SENTENCES, op)


def test_fsst_compress_comments_1m(ctx):
    """1 Mi synthetic l_comment strings (bench C4's generator), plus escapes: bytes no symbol
    covers, empty strings and nulls."""
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import bench
    rng = np.random.default_rng(17)
    heap, offs = bench.c4_heap(rng, 1 << 20)
    strings = [heap[offs[i]:offs[i + 1]].tobytes() for i in range(offs.size - 1)]
    for i in range(0, len(strings), 997):
        strings[i] = None
    for i in range(5, len(strings), 1009):
        strings[i] = b""
    for i in range(7, len(strings), 4999):
        strings[i] = bytes(rng.integers(0, 256, int(rng.integers(1, 90)), dtype=np.uint8))
    _fsst_gpu_vs_host(ctx, strings)


def test_fsst_compress_edge_cases(ctx):
    """Empty input, one string, all-null, long strings, every byte value, strings shorter than
    the symbols that would match them."""
    _fsst_gpu_vs_host(ctx, [])
    _fsst_gpu_vs_host(ctx, [b"a"])
    _fsst_gpu_vs_host(ctx, [None, None, None])
    rng = np.random.default_rng(5)
    long = [bytes(rng.integers(97, 100, int(rng.integers(100, 5000)), dtype=np.uint8)) for _ in range(50)]
    _fsst_gpu_vs_host(ctx, long + [bytes(range(256))] + [b"ab", b"abc", b"a"] * 30)


def test_fsst_compress_bad_offsets(ctx):
    """Offsets that run backwards or past the bytes are rejected, not read."""
    heap = np.frombuffer(b"hello world", np.uint8).copy()
    offs = np.array([0, 5, 3, 11], np.int64)
    syms, lens = np.array([int.from_bytes(b"lo", "little")], np.uint64), np.array([2], np.uint8)
    with pytest.raises(V.VortexGpuError, match="offsets"):
        G.fsst_compress(ctx, _dev(offs), "i64", _dev(heap), 3, syms, lens)
    with pytest.raises(V.VortexGpuError, match="symbol length"):
        G.fsst_compress(ctx, _dev(np.array([0, 5], np.int64)), "i64", _dev(heap), 1, syms,
                        np.array([9], np.uint8))
