"""GPU parity: the HIP engine (through the C ABI) against the oracle, bit-exact.

Every case builds a Vortex array tree with the reference encoders, canonicalizes it on the
MI355X with vxg_canonicalize (or a per-encoding entry point), and compares every output byte
with the oracle's CPU canonicalize of the same tree (tests/oracle_tree.py) — and with the
original data (decode(encode(x)) == x).  Floating point is compared as raw bits.
"""
import contextlib
import ctypes as C
import dataclasses

import numpy as np
import pytest

import vortex_amd as V
import vortex_amd.arrays as A
import vortex_amd.encode as E
from oracle_tree import canon, view_bytes

pytestmark = pytest.mark.gpu

UT = {8: np.uint8, 16: np.uint16, 32: np.uint32, 64: np.uint64}


def gpu(arr, ctx):
    import torch
    dev = arr.to(torch.device("cuda", 0))
    return V.canonicalize(dev, ctx)


def assert_primitive_parity(arr, ctx, expect=None):
    res = gpu(arr, ctx)
    got = res.numpy()
    ref, rvalid = canon(arr)
    assert got.dtype == ref.dtype and got.size == ref.size
    assert got.tobytes() == ref.tobytes()
    if expect is not None:
        assert got.tobytes() == np.ascontiguousarray(expect).astype(got.dtype).tobytes()
    gvalid = res.validity_mask()
    if rvalid is None:
        assert gvalid is None or gvalid.all()
    else:
        assert np.array_equal(gvalid, rvalid)
    return got


def assert_string_parity(arr, ctx, strings=None):
    res = gpu(arr, ctx)
    views, _ = res.numpy()
    heap = res.buffers()
    (rviews, rheap), rvalid = canon(arr)
    rheap = rheap if isinstance(rheap, list) else [rheap]
    assert len(heap) == len(rheap)
    for g, r in zip(heap, rheap):
        assert g.tobytes() == r.tobytes()
    assert views.tobytes() == rviews.tobytes()
    gvalid = res.validity_mask()
    if rvalid is None:
        assert gvalid is None
    else:
        assert np.array_equal(gvalid, rvalid)
    if strings is not None:
        for i, s in enumerate(strings):
            if s is not None:
                assert view_bytes(views, heap, i) == s


# ------------------------------------------------------------------ K1 BitPacked
@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_bitunpack_every_width(ctx, T):
    rng = np.random.default_rng(T)
    dt = UT[T]
    n = 3 * 1024 + 17
    for W in range(T):
        vals = (rng.integers(0, 1 << W, n, dtype=np.uint64) if W else np.zeros(n, np.uint64)).astype(dt)
        arr = E.encode_bitpacked(vals, bit_width=W, allow_patches=False)
        assert_primitive_parity(arr, ctx, vals)


@pytest.mark.parametrize("T,W", [(8, 3), (16, 11), (32, 7), (32, 17), (64, 24), (64, 63)])
@pytest.mark.parametrize("n", [1, 1000, 1024, 1025, 65_535, 1 << 20])
def test_bitunpack_sizes(ctx, T, W, n):
    rng = np.random.default_rng(n + W)
    vals = rng.integers(0, 1 << W, n, dtype=np.uint64).astype(UT[T])
    assert_primitive_parity(E.encode_bitpacked(vals, bit_width=W, allow_patches=False), ctx, vals)


@pytest.mark.parametrize("offset", [1, 3, 511, 1023])
@pytest.mark.parametrize("T", [8, 32, 64])
def test_bitunpack_sliced_offset(ctx, offset, T):
    rng = np.random.default_rng(offset)
    W = T // 2 - 1
    vals = rng.integers(0, 1 << W, 5000, dtype=np.uint64).astype(UT[T])
    assert_primitive_parity(E.encode_bitpacked(vals, bit_width=W, offset=offset), ctx, vals)


@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_bitunpack_with_patches(ctx, T):
    rng = np.random.default_rng(11)
    dt = UT[T]
    vals = rng.integers(0, 16, 70_000, dtype=np.uint64).astype(dt)
    vals[rng.choice(vals.size, 700, replace=False)] = np.iinfo(dt).max
    arr = E.encode_bitpacked(vals)  # best width -> patches, indices BitPacked u64
    assert arr.meta["has_patches"]
    assert_primitive_parity(arr, ctx, vals)


# K1w (the large-launch K1: burst LDS staging + wave-contiguous stores) is chosen by launch size;
# the context option K1_WAVE=2 takes it for every launch so every width, epilogue, offset and tail
# is compared with the oracle at test sizes.  Its blocks per workgroup (BPW) is the width's
# maximum, or fewer (a multiple of 4) for a launch that would have < K1W_MIN_GROUPS workgroups
# (the default rule picks an intermediate BPW for any 4-30 Mi-value plan column): every case runs
# at the maximum, intermediate values, 4 and a non-multiple of 4, and asserts the BPW it ran with
# (vxg_get_launch_stats).
def kw_bpw_max(W, lds_dict=False):
    """fl_unpack_impl.hpp kw_bpw: ~32 KiB of packed words (16 KiB beside an LDS dictionary)."""
    b = ((16 if lds_dict else 32) * 1024) // (128 * max(W, 1))
    return min(32, max(4, b // 4 * 4))


def kw_rule_bpw(blocks, bpw_max, min_groups):
    """fl_unpack_impl.hpp k1w_pick_bpw without a forced value."""
    if min_groups <= 0 or blocks >= min_groups * bpw_max:
        return bpw_max
    b = blocks // min_groups
    return min(bpw_max, 4 if b < 4 else b // 4 * 4)


# 5: the shape of the r05e failure (profiles/r05e_k1w_bpw_failure.md) -- waves of 2, 2, 1, 0 blocks
BPW_MODES = ["max", 16, 8, 6, 5, 4]


@pytest.fixture
def k1w(ctx):
    """The session context with K1w forced for every launch; the options are restored after."""
    ctx.set_option("k1_wave", 2)
    ctx.launch_stats(reset=True)
    try:
        yield ctx
    finally:
        ctx.set_option("k1_wave", -1)
        ctx.set_option("k1w_bpw", 0)
        ctx.set_option("k1w_min_groups", 1024)


def set_bpw_mode(ctx, mode):
    if mode == "max":
        ctx.set_option("k1w_min_groups", 0)
        ctx.set_option("k1w_bpw", 0)
    else:
        ctx.set_option("k1w_bpw", int(mode))


def assert_bpw_ran(ctx, mode, bpw_max=None):
    """Every K1w launch since the last check ran with the mode's BPW (forced: min(mode, max))."""
    st = ctx.launch_stats(reset=True)
    assert st["k1w_launches"] >= 1, "no K1w launch"
    if bpw_max is not None:
        assert st["k1w_last_bpw_max"] == bpw_max
    want = st["k1w_last_bpw_max"] if mode == "max" else min(int(mode), st["k1w_last_bpw_max"])
    assert st["k1w_last_bpw"] == want, (mode, st)
    if mode != "max":
        assert st["k1w_max_bpw"] <= int(mode)
    return st


@pytest.mark.parametrize("mode", BPW_MODES)
@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_k1w_every_width(k1w, T, mode):
    ctx = k1w
    set_bpw_mode(ctx, mode)
    rng = np.random.default_rng(100 + T)
    dt = UT[T]
    for W in range(T + 1) if T < 64 else list(range(0, 64, 3)) + [63]:
        if W == T:
            continue
        n = int(rng.integers(1, 40_000))
        vals = (rng.integers(0, 1 << W, n, dtype=np.uint64) if W else np.zeros(n, np.uint64)).astype(dt)
        off = int(rng.integers(0, 1024)) if W % 2 else 0
        assert_primitive_parity(E.encode_bitpacked(vals, bit_width=W, allow_patches=False, offset=off), ctx, vals)
        assert_bpw_ran(ctx, mode, kw_bpw_max(W))


@pytest.mark.parametrize("min_groups", [1, 3, 7])
def test_k1w_runtime_rule(k1w, min_groups):
    """The default rule at test sizes: K1W_MIN_GROUPS small enough that blocks / min_groups lands
    between 4 and the width's maximum (the same rule a 4-30 Mi-value plan column takes at 1024)."""
    ctx = k1w
    ctx.set_option("k1w_min_groups", min_groups)
    rng = np.random.default_rng(200 + min_groups)
    seen = set()
    for T, W, n, off in [(32, 7, 40_000, 0), (32, 7, 77_777, 517), (16, 5, 90_000, 3), (64, 17, 60_000, 1000),
                         (8, 3, 150_000, 0), (64, 24, 33_000, 9)]:
        vals = rng.integers(0, 1 << W, n, dtype=np.uint64).astype(UT[T])
        assert_primitive_parity(E.encode_bitpacked(vals, bit_width=W, allow_patches=False, offset=off), ctx, vals)
        st = ctx.launch_stats(reset=True)
        blocks = (n + off + 1023) // 1024
        want = kw_rule_bpw(blocks, kw_bpw_max(W), min_groups)
        assert st["k1w_last_bpw"] == want, (T, W, n, st)
        seen.add(want)
    assert len(seen) >= 2


@pytest.mark.parametrize("mode", ["max", 8, 4])
def test_k1w_epilogues_and_chunks(k1w, mode):
    """FoR / ZigZag / ALP / Dict epilogues, patches, chunked tables (ragged, sliced, unaligned
    slices) and a plan's device table through K1w, at each blocks-per-workgroup mode."""
    import torch
    ctx = k1w
    set_bpw_mode(ctx, mode)
    rng = np.random.default_rng(7)
    cases = []
    for dt in (np.int8, np.int16, np.int32, np.int64, np.uint32):
        info = np.iinfo(dt)
        base = int(info.min) // 2 + 8 if info.min < 0 else 1000
        cases.append(E.encode_for_bitpacked((base + 4 * rng.integers(0, 25, 9000)).astype(dt)))
    cases.append(E.encode_zigzag(rng.integers(-500, 500, 20_000).astype(np.int32)))
    cases.append(E.encode_alp(c_prices(rng, 30_000)))
    cases.append(E.encode_alp(c_prices(rng, 30_000).astype(np.float32)))
    for vdt in (np.uint8, np.uint16, np.uint32, np.uint64):
        pool = rng.integers(0, 200, 300).astype(vdt)
        cases.append(E.encode_dict(pool[rng.integers(0, pool.size, 25_000)]))
    cases.append(E.encode_dict_strings([b"row-%d" % (i % 37) for i in range(20_000)]))
    big = rng.integers(0, 16, 70_000, dtype=np.uint64).astype(np.uint32)
    big[rng.choice(big.size, 700, replace=False)] = np.iinfo(np.uint32).max
    cases.append(E.encode_bitpacked(big))
    cases.append(A.chunked([E.encode_bitpacked(rng.integers(0, 1 << 9, n, dtype=np.uint64).astype(np.uint16),
                                               bit_width=9, allow_patches=False) for n in (1000, 3, 4097, 70_000)]))
    cases.append(A.chunked([E.encode_for_bitpacked(rng.integers(-99, 99, n).astype(np.int64)) for n in (5, 2048, 33_333)]))
    for a in cases:
        if a.dtype == A.DTYPE["PRIMITIVE"]:
            assert_primitive_parity(a, ctx)
        else:
            assert_string_parity(a, ctx)
        if a.encoding != A.ENC["DICT"] or a.children[0].dtype == A.DTYPE["PRIMITIVE"]:
            assert_bpw_ran(ctx, mode)  # (string dictionaries take K14, not K1w)
        ctx.launch_stats(reset=True)
    with plan_mode("0"):  # unbatched: the chunked columns' device-table K1w launches
        plan = V.Plan([a.to(torch.device("cuda", 0)) for a in cases[-2:]], ctx)
    assert_bpw_ran(ctx, mode)
    for _ in range(2):
        res = plan.launch(sync=True)
        for a, r in zip(cases[-2:], res):
            assert r.numpy().tobytes() == canon(a)[0].tobytes()
    plan.close()


@pytest.mark.parametrize("batch", ["1", "0"])
def test_k1w_mid_size_default_rule(ctx, batch):
    """plan columns of 4-30 Mi values over a device chunk table (> 32 chunks, as
    C5's 92-chunk columns) take an intermediate BPW under the DEFAULT rule (K1W_MIN_GROUPS 1024)
    -- the production path of C5's numeric columns.  u32 W=7, 48 x 256 Ki values with a sliced
    chunk (12,288 blocks -> BPW 12 of 32), and ALP f64 (W=17) + patches, 34 x 256 Ki (8,704
    blocks -> BPW 8 of 12); batched (>= 20 MiB groups keep their K1w launch) and unbatched plans,
    bit-exact against the oracle and the plain values."""
    import torch
    assert ctx.get_option("k1w_min_groups") == 1024 and ctx.get_option("k1w_bpw") == 0
    rng = np.random.default_rng(300)
    n = 1 << 18
    u_plain, u_chunks = [], []
    for c in range(48):
        v = rng.integers(0, 128, n, dtype=np.uint32)
        u_plain.append(v)
        u_chunks.append(E.encode_bitpacked(v, bit_width=7, allow_patches=False, offset=517 if c == 5 else 0))
    f_plain, f_chunks = [], []
    for c in range(34):
        v = np.round(rng.uniform(1, 1000, n) * 100) / 100
        v[rng.choice(n, 100, replace=False)] = rng.standard_normal(100) * 1e9 + 0.123456789
        f_plain.append(v)
        f_chunks.append(E.encode_alp(v))
    assert all(f.children[0].children[0].meta["bit_width"] == 17 for f in f_chunks)
    cases = [(A.chunked(u_chunks), np.concatenate(u_plain), 12, 32),
             (A.chunked(f_chunks), np.concatenate(f_plain), 8, 12)]
    for arr, plain, bpw, bpw_max in cases:
        ctx.launch_stats(reset=True)
        with plan_mode(batch):
            plan = V.Plan([arr.to(torch.device("cuda", 0))], ctx)
        st = ctx.launch_stats(reset=True)
        assert st["k1w_launches"] == 1 and st["k1w_last_bpw"] == bpw and st["k1w_last_bpw_max"] == bpw_max, st
        for _ in range(2):
            got = plan.launch(sync=True)[0].numpy()
            assert got.tobytes() == plain.tobytes()
        assert got.tobytes() == canon(arr)[0].tobytes()
        plan.close()


@pytest.mark.parametrize("dt", [np.uint8, np.uint16, np.uint32])
def test_chunked_primitive_copy_misaligned(ctx, dt):
    """a chunk whose output slice is not 16-byte aligned (after a chunk whose byte
    length is not a multiple of 16) is copied by K10's funnel-shift path at every residue
    (1-15 bytes for u8), multi-MB per chunk, byte-exact; also inside a replayed plan."""
    import torch
    rng = np.random.default_rng(400 + np.dtype(dt).itemsize)
    plains = [rng.integers(0, np.iinfo(dt).max, (1 << 20) + 3 * i + (i % 2), dtype=dt, endpoint=True)
              for i in range(17)]
    arr = A.chunked([A.primitive(p) for p in plains])
    want = np.concatenate(plains)
    assert gpu(arr, ctx).numpy().tobytes() == want.tobytes()
    plan = V.Plan([arr.to(torch.device("cuda", 0))], ctx)
    for _ in range(2):
        assert plan.launch(sync=True)[0].numpy().tobytes() == want.tobytes()
    plan.close()


def c_prices(rng, n):
    v = np.round(rng.uniform(1, 100000, n) * 100) / 100
    v[rng.choice(n, n // 500, replace=False)] = rng.uniform(1, 100000, n // 500) + 1e-7
    return v


def test_bitpacked_reference_kat_patch_max(ctx):
    vals = np.array([1, 0, 1, 0, 1, 0, 2 ** 64 - 1], np.uint64)
    arr = E.encode_bitpacked(vals, bit_width=1, validity=[True, False, True, False, True, False, True])
    got = assert_primitive_parity(arr, ctx)
    assert got.tolist() == [1, 0, 1, 0, 1, 0, 2 ** 64 - 1]


def test_signed_bitpacked_reinterpret(ctx):
    # unpack of a signed ptype reinterpret-casts (bitpacking/compress.rs:179-182)
    vals = np.arange(0, 3000, dtype=np.int32) % 100
    arr = E.encode_bitpacked(vals.view(np.uint32), bit_width=7)
    arr.ptype = "i32"
    assert_primitive_parity(arr, ctx, vals)


# ------------------------------------------------------------------ FoR / ZigZag / ALP
@pytest.mark.parametrize("dt", [np.int8, np.uint16, np.int32, np.uint32, np.int64, np.uint64])
def test_for_bitpacked_fused(ctx, dt):
    rng = np.random.default_rng(5)
    info = np.iinfo(dt)
    base = int(info.min) // 2 + 8 if info.min < 0 else 1000
    vals = (base + 4 * rng.integers(0, 25, 9000)).astype(dt)
    arr = E.encode_for_bitpacked(vals)
    assert arr.encoding == A.ENC["FL_FOR"] and arr.meta["shift"] == 2
    assert_primitive_parity(arr, ctx, vals)


def test_for_i8_overflow_kat(ctx):
    vals = np.arange(-128, 128, dtype=np.int8)
    assert_primitive_parity(E.encode_for_bitpacked(vals), ctx, vals)


def test_for_over_primitive_child(ctx):
    enc = np.arange(5000, dtype=np.uint32) * 3
    arr = A.frame_of_reference(A.primitive(enc), 1_000_000, 1, "u32")
    assert_primitive_parity(arr, ctx)


@pytest.mark.parametrize("dt", [np.int8, np.int16, np.int32, np.int64])
def test_zigzag(ctx, dt):
    vals = (np.arange(-5000, 5000) % 120 - 60).astype(dt)
    assert_primitive_parity(E.encode_zigzag(vals), ctx, vals)


@pytest.mark.parametrize("n", [3, 1025, 100_000])
def test_alp_f64_cascade(ctx, n):
    rng = np.random.default_rng(n)
    vals = np.round(rng.uniform(1, 100000, n) * 100) / 100
    if n > 10:
        vals[rng.choice(n, n // 1000 + 1, replace=False)] = rng.standard_normal(n // 1000 + 1) * 1e9
    arr = E.encode_alp(vals)
    got = assert_primitive_parity(arr, ctx)
    assert got.tobytes() == vals.tobytes()


def test_alp_reference_kats_on_gpu(ctx):
    import math
    vals = np.array([1.234, 2.718, math.pi, 4.0])
    arr = E.encode_alp(vals, cascade=False)
    assert (arr.meta["e"], arr.meta["f"]) == (16, 13)
    assert assert_primitive_parity(arr, ctx).tobytes() == vals.tobytes()
    vals32 = np.full(1025, 1.234, np.float32)
    arr = E.encode_alp(vals32)
    assert (arr.meta["e"], arr.meta["f"]) == (9, 6)
    assert assert_primitive_parity(arr, ctx).tobytes() == vals32.tobytes()


def _alp_patched(rng, n, pos, f32=False, offset=0, indices_offset=0, packed_indices=True):
    """ALP -> FoR -> BitPacked (sliced by `offset`) with outer patches at the ascending positions
    `pos` (values the ALP exponents cannot produce); returns (array, expected values)."""
    ft = np.float32 if f32 else np.float64
    vals = (np.round(rng.uniform(1, 1000 if f32 else 100000, n) * 100) / 100).astype(ft)
    e, f, enc, idx, _ = E.alp_encode(vals)
    u, ref, sh = E.for_compress(enc)
    bp = E.encode_bitpacked(u, bit_width=max(1, int(u.max()).bit_length()), allow_patches=False, offset=offset)
    child = A.frame_of_reference(bp, ref, sh, "i32" if f32 else "i64")
    allp = np.union1d(pos, idx).astype(np.int64)  # the encoder's own exceptions are patches too
    pv = vals[allp].copy()
    mine = np.isin(allp, pos)
    pv[mine] = (rng.standard_normal(int(mine.sum())) * 1e9 + 0.123456789).astype(ft)
    pos = allp
    ind = pos.astype(np.uint64) + np.uint64(indices_offset)
    ia = (E.encode_bitpacked(ind, bit_width=max(1, int(ind.max()).bit_length()), allow_patches=False)
          if packed_indices else A.primitive(ind))
    arr = A.alp(child, e, f, A.sparse(ia, A.primitive(pv, validity="ALL_VALID"), n, indices_offset=indices_offset))
    expect = vals.copy()
    expect[pos] = pv
    return arr, expect


# ALP's outer patches are written by the K1w launch itself (fl_unpack_impl.hpp unpack_chunk_w):
# a 256-patch window guessed from an even spread, or a 256-ary search when the window does not
# bracket the workgroup's output range.  Both against the separate scatter (VXG_FUSED_PATCHES=0).
@pytest.mark.parametrize("mode", ["max", 8, 6, 4])
@pytest.mark.parametrize("fused", ["1", "0"])
def test_k1w_fused_patches(k1w, fused, mode, monkeypatch):
    ctx = k1w
    set_bpw_mode(ctx, mode)
    monkeypatch.setenv("VXG_FUSED_PATCHES", fused)
    rng = np.random.default_rng(77)
    n = 300_000
    cases = [
        dict(pos=np.sort(rng.choice(n, n // 1000, replace=False))),                      # spread: windows
        dict(pos=np.concatenate([[0], np.arange(100_000, 105_000), [n - 1]])),          # clustered: search
        dict(pos=np.sort(rng.choice(n, 20_000, replace=False))),                         # dense: both
        dict(pos=np.array([n - 1])),                                                     # one, at the end
        dict(pos=np.sort(rng.choice(n, 300, replace=False)), offset=517, indices_offset=1000,
             packed_indices=False),                                                      # sliced
        dict(pos=np.sort(rng.choice(n, 3000, replace=False)), f32=True),
        dict(pos=np.concatenate([np.arange(0, 40_000, 7), np.arange(250_000, n)]), f32=True, offset=3),
    ]
    for kw in cases:
        pos = kw.pop("pos")
        arr, expect = _alp_patched(rng, n, pos, **kw)
        assert_primitive_parity(arr, ctx, expect)
        assert_bpw_ran(ctx, mode)


@pytest.mark.parametrize("mode", ["max", 4])
def test_k1w_fused_patches_errors(k1w, mode):
    """Out-of-range and descending patch indices are reported, as by the separate scatter."""
    ctx = k1w
    set_bpw_mode(ctx, mode)
    rng = np.random.default_rng(78)
    n = 50_000
    arr, _ = _alp_patched(rng, n, np.array([5, 70, n - 1]))
    arr.children[1].children[0] = A.primitive(np.array([5, 70, n], np.uint64))
    with pytest.raises(V.VortexGpuError, match="out of bounds"):
        gpu(arr, ctx)
    arr, _ = _alp_patched(rng, n, np.array([5, 70, 900]))
    arr.children[1].children[0] = A.primitive(np.array([5, 900, 70], np.uint64))
    with pytest.raises(V.VortexGpuError, match="not sorted"):
        gpu(arr, ctx)


def _alp_bad_cluster(rng, n=300_000):
    """> 256 patches clustered (so workgroups take the 256-ary search, not a window) with first and
    last index in range and one middle index past the end: a malformed file's patches."""
    pos = np.concatenate([[0], np.arange(100_000, 105_000), [n - 1]])
    arr, _ = _alp_patched(rng, n, pos, packed_indices=False)
    idx = np.asarray(arr.children[1].children[0].buffers[0]).view(np.uint64).copy()
    assert idx.size > 256 and idx[0] == 0 and idx[-1] == n - 1
    idx[idx.size // 2] = n + 5
    arr.children[1].children[0] = A.primitive(idx)
    return arr


@pytest.mark.parametrize("mode", ["max", 4])
def test_k1w_fused_patches_unsorted_cluster_never_writes_out_of_range(k1w, mode):
    """the search fallback stores only keys inside the workgroup's range; an index
    past the end inside an unsorted cluster is reported, not written (the device would fault or
    corrupt the neighbour allocation otherwise)."""
    ctx = k1w
    set_bpw_mode(ctx, mode)
    rng = np.random.default_rng(79)
    with pytest.raises(V.VortexGpuError, match="not sorted|out of bounds"):
        gpu(_alp_bad_cluster(rng), ctx)
    ctx.sync()  # the error word was cleared by the failing sync


def test_plan_measure_flag_and_info(ctx):
    """vxg_plan_create executes nothing and records one candidate; VXG_PLAN_MEASURE records both,
    times them and reports a device error found by its runs from create itself."""
    import torch
    rng = np.random.default_rng(80)
    arrs = [E.encode_for_bitpacked(rng.integers(-99, 99, 50_000).astype(np.int64)),
            E.encode_dict_strings([b"row-%d" % (i % 37) for i in range(20_000)])]
    dev = [a.to(torch.device("cuda", 0)) for a in arrs]
    p0 = V.Plan(dev, ctx)
    i0 = p0.info()
    assert len(i0["candidates"]) == 1 and i0["candidates"][0]["ms"] == 0.0 and i0["batched"]
    p1 = V.Plan(dev, ctx, measure=True)
    i1 = p1.info()
    assert len(i1["candidates"]) == 2 and all(c["ms"] > 0 for c in i1["candidates"])
    assert {c["batched"] for c in i1["candidates"]} == {False, True} and i1["create_ms"] > 0
    for p in (p0, p1):
        res = p.launch(sync=True)
        for a, r in zip(arrs, res):
            ref = canon(a)[0]
            if isinstance(ref, tuple):
                assert r.numpy()[0].tobytes() == ref[0].tobytes()
            else:
                assert r.numpy().tobytes() == ref.tobytes()
        p.close()
    bad = _alp_patched(rng, 50_000, np.array([5, 70, 900]))[0]
    bad.children[1].children[0] = A.primitive(np.array([5, 70, 50_000], np.uint64))
    bdev = [bad.to(torch.device("cuda", 0))]
    with pytest.raises(V.VortexGpuError, match="out of bounds"):
        V.Plan(bdev, ctx, measure=True)
    ctx.sync()  # nothing left behind for the caller's next sync
    p2 = V.Plan(bdev, ctx)  # no measurement: nothing ran, the error comes from the replay
    ctx.sync()
    with pytest.raises(V.VortexGpuError, match="out of bounds"):
        p2.launch(sync=True)
    p2.close()


def test_plan_measure_leaves_pending_caller_error(ctx):
    """a measuring create must not take over an error of the caller's earlier,
    unsynced work.  A bad decode is left pending (no sync), then a good plan is created with
    VXG_PLAN_MEASURE: create succeeds without measuring (selection "unmeasured", the smaller
    graph kept), and the caller's next sync still reports the pending error."""
    import torch
    rng = np.random.default_rng(81)
    bad = _alp_patched(rng, 50_000, np.array([5, 70, 900]))[0]
    bad.children[1].children[0] = A.primitive(np.array([5, 70, 50_000], np.uint64))
    A.canonicalize(bad.to(torch_dev()), ctx, sync=False)  # pending, not synced
    good = [E.encode_for_bitpacked(rng.integers(-99, 99, 50_000).astype(np.int64)),
            E.encode_dict_strings([b"row-%d" % (i % 37) for i in range(20_000)])]
    dev = [a.to(torch_dev()) for a in good]
    p = V.Plan(dev, ctx, measure=True)
    info = p.info()
    assert info["selection"] == "unmeasured" and all(c["ms"] == 0.0 for c in info["candidates"])
    costs = [c["cost"] for c in info["candidates"]]
    kept = [c for c in info["candidates"] if c["batched"] == info["batched"]][0]
    assert kept["cost"] == min(costs)
    with pytest.raises(V.VortexGpuError, match="out of bounds"):
        ctx.sync()
    ctx.sync()  # reported once
    res = p.launch(sync=True)
    assert res[0].numpy().tobytes() == canon(good[0])[0].tobytes()
    p.close()
    # with nothing pending, the same create measures both candidates
    p = V.Plan(dev, ctx, measure=True)
    assert p.info()["selection"] in ("faster", "tie_fewer_nodes")
    assert all(c["ms"] > 0 for c in p.info()["candidates"])
    p.close()


def test_alp_f32_cascade(ctx):
    rng = np.random.default_rng(4)
    vals = (np.round(rng.uniform(-500, 500, 50_000) * 10) / 10).astype(np.float32)
    assert assert_primitive_parity(E.encode_alp(vals), ctx).tobytes() == vals.tobytes()


@pytest.mark.parametrize("ptype", ["f32", "f64"])
def test_alprd(ctx, ptype):
    rng = np.random.default_rng(8)
    vals = (rng.standard_normal(40_000) * 1000).astype(A.NP_OF_PTYPE[ptype])
    vals[::997] = rng.standard_normal(vals[::997].size).astype(vals.dtype) * 1e30
    assert assert_primitive_parity(E.encode_alprd(vals), ctx).tobytes() == vals.tobytes()


# ------------------------------------------------------------------ Dict / take
@pytest.mark.parametrize("vdt", [np.uint8, np.int16, np.float32, np.uint64])
@pytest.mark.parametrize("card", [1, 2, 200, 4000])
def test_dict_fused(ctx, vdt, card):
    rng = np.random.default_rng(card)
    pool = rng.integers(0, 120, card * 2).astype(vdt)
    pool = np.unique(pool)[:card]
    vals = pool[rng.integers(0, pool.size, 30_000)]
    arr = E.encode_dict(vals)
    assert_primitive_parity(arr, ctx, vals)


def test_dict_unpacked_codes_take(ctx):
    arr = A.dict_array(A.primitive(np.array([1, 2, 3, 4, 5], np.int32)), A.primitive(np.array([0, 0, 4, 2], np.uint64)))
    assert assert_primitive_parity(arr, ctx).tolist() == [1, 1, 5, 3]


def test_take_out_of_bounds_is_an_error(ctx):
    arr = A.dict_array(A.primitive(np.array([1, 2], np.int32)), A.primitive(np.array([0, 5], np.uint64)))
    with pytest.raises(V.VortexGpuError) as ei:
        gpu(arr, ctx)
    assert ei.value.kind == "OutOfBounds"


def test_dict_strings(ctx):
    strings = [b"hello", b"world", b"hello", b"again", b"world", b"a much longer string value"] * 500
    codes, _ = E.dict_encode(np.array([hash(s) for s in strings], np.int64))
    uniq = []
    for s in strings:
        if s not in uniq:
            uniq.append(s)
    heap, offs, _ = E.strings_to_heap(uniq)
    values = A.varbin(A.primitive(offs.astype(np.int32)), A.primitive(heap))
    arr = A.dict_array(values, E.encode_bitpacked(codes, allow_patches=False))
    assert_string_parity(arr, ctx, strings)


# ------------------------------------------------------------------ Delta / RunEnd
@pytest.mark.parametrize("dt", [np.uint8, np.uint16, np.uint32, np.uint64])
@pytest.mark.parametrize("n", [1, 1024, 4097, 200_000])
def test_delta(ctx, dt, n):
    rng = np.random.default_rng(n)
    vals = np.cumsum(rng.integers(0, 5, n)).astype(dt)
    assert_primitive_parity(E.encode_delta(vals), ctx, vals)


def test_delta_sliced(ctx):
    vals = np.cumsum(np.random.default_rng(5).integers(0, 9, 9000)).astype(np.uint32)
    arr = E.encode_delta(vals)
    sl = A.delta(arr.children[0], arr.children[1], offset=300, length=7000)
    assert_primitive_parity(sl, ctx, vals[300:7300])


@pytest.mark.parametrize("vdt", [np.int8, np.int32, np.float64])
def test_runend(ctx, vdt):
    rng = np.random.default_rng(2)
    vals = np.repeat(rng.integers(-100, 100, 3000).astype(vdt), rng.integers(1, 40, 3000))
    arr = E.encode_runend(vals)
    assert_primitive_parity(arr, ctx, vals)
    arr.meta["offset"] = 33
    arr.len = vals.size - 100
    assert_primitive_parity(arr, ctx, vals[33:33 + arr.len])


# ------------------------------------------------------------------ Sparse / Constant / Chunked
def test_sparse_null_fill_validity(ctx):
    idx = E.encode_bitpacked(np.array([3, 5, 9, 4000], np.uint64), bit_width=12, allow_patches=False)
    arr = A.sparse(idx, A.primitive(np.array([7, 8, 9, 10], np.int64)), 5000, fill=None)
    assert_primitive_parity(arr, ctx)


def test_constant(ctx):
    assert_primitive_parity(A.constant(-3, 10_000, "i16"), ctx, np.full(10_000, -3, np.int16))
    assert_primitive_parity(A.constant(None, 100, "u32"), ctx)


def test_chunked_grouped_dict(ctx):
    rng = np.random.default_rng(3)
    chunks, expect = [], []
    for c in range(12):
        dv = rng.integers(0, 2 ** 63, 1024, dtype=np.uint64)
        vals = dv[rng.zipf(1.1, 50_000 + 1024 * (c % 3)) % 1024]
        codes = E.dict_encode(vals)[0]
        chunks.append(A.dict_array(A.primitive(E.dict_encode(vals)[1]), E.encode_bitpacked(codes, bit_width=10, allow_patches=False)))
        expect.append(vals)
    arr = A.chunked(chunks)
    assert_primitive_parity(arr, ctx, np.concatenate(expect))


@pytest.mark.parametrize("kind", ["bitpacked", "for", "zigzag", "alp64", "alp32", "dict8"])
def test_chunked_grouped_every_epilogue(ctx, kind):
    """Chunked arrays whose chunks are one K1 decode each share launches (chunk tables of up
    to 32 per kernel, grouped by (T, W, epilogue)): 70 chunks -> several batches, per-chunk
    widths / FoR references / ALP exponents differ, ragged chunk lengths, and patches (inner
    BitPacked patches and outer ALP patches) applied after the grouped launches."""
    rng = np.random.default_rng(len(kind))
    chunks, expect = [], []
    for c in range(70):
        n = 4096 * (1 + c % 3) + (c * 37) % 1000
        if kind == "bitpacked":
            v = rng.integers(0, 1 << (3 + c % 5), n, dtype=np.uint64).astype(np.uint32)
            v[rng.choice(n, 3, replace=False)] = 2 ** 31 + c   # patches
            arr = E.encode_bitpacked(v)
        elif kind == "for":
            v = (rng.integers(-500, 500, n) + 10_000 * c).astype(np.int64)
            arr = E.encode_for_bitpacked(v)
        elif kind == "zigzag":
            v = rng.integers(-(1 << (4 + c % 4)), 1 << (4 + c % 4), n).astype(np.int32)
            arr = E.encode_zigzag(v)
        elif kind == "alp64":
            v = np.round(rng.uniform(0, 10 ** (1 + c % 5), n), 2 + c % 2)
            v[rng.choice(n, 2, replace=False)] = rng.standard_normal(2) * 1e300
            arr = E.encode_alp(v)
        elif kind == "alp32":
            v = (np.round(rng.uniform(0, 100, n), 1)).astype(np.float32)
            arr = E.encode_alp(v)
        else:
            dv = rng.integers(0, 2 ** 63, 17 + c, dtype=np.uint64)
            v = dv[rng.integers(0, dv.size, n)]
            arr = E.encode_dict(v)
        chunks.append(arr)
        expect.append(v)
    assert_primitive_parity(A.chunked(chunks), ctx, np.concatenate(expect))


def test_chunked_mixed_with_validity(ctx):
    a = E.encode_bitpacked(np.arange(3000, dtype=np.uint32) % 77, validity=(np.arange(3000) % 5 != 0))
    b = A.primitive(np.arange(1001, dtype=np.uint32), validity=None)
    c = E.encode_delta(np.arange(2048, dtype=np.uint32))
    assert_primitive_parity(A.chunked([a, b, c]), ctx)


# ------------------------------------------------------------------ strings: VarBin, FSST
def test_varbin_views_boundary(ctx):
    strings = [None, None, b"123456789012", b"1234567890123", b"", b"x" * 100]
    heap, offs, valid = E.strings_to_heap(strings)
    arr = A.varbin(A.primitive(offs.astype(np.int32)), A.primitive(heap), validity=valid)
    assert_string_parity(arr, ctx, strings)


@pytest.mark.parametrize("n", [3, 1000, 40_000])
def test_fsst(ctx, n):
    rng = np.random.default_rng(n)
    words = [b"carefully", b"final", b"deposits", b"sleep", b"quickly", b"ironic", b"packages",
             b"blithely", b"regular", b"accounts", b"\x00\xff", b"furiously"]
    strings = []
    for i in range(n):
        if i % 23 == 7:
            strings.append(None)
        else:
            k = int(rng.integers(1, 7))
            strings.append(b" ".join(words[j] for j in rng.integers(0, len(words), k)))
    assert_string_parity(E.encode_fsst(strings), ctx, strings)


def _fsst_handmade(strings, symbols):
    """FSST array from a fixed symbol table and a greedy longest-match coder that escapes every
    other byte (code 255 + literal) — the trainer would learn 0xFF runs as symbols instead."""
    syms = [s for s in symbols]
    codes, coffs, lens = bytearray(), [0], []
    for s in strings:
        s = s or b""
        k = 0
        while k < len(s):
            best = max((j for j, y in enumerate(syms) if s.startswith(y, k)), key=lambda j: len(syms[j]),
                       default=None)
            if best is None:
                codes += bytes([255, s[k]])
                k += 1
            else:
                codes.append(best)
                k += len(syms[best])
        coffs.append(len(codes))
        lens.append(len(s))
    valid = np.array([s is not None for s in strings])
    sym_u64 = np.array([int.from_bytes(y.ljust(8, b"\0"), "little") for y in syms], np.uint64)
    code_vb = A.varbin(A.primitive(np.array(coffs, np.int32)), A.primitive(np.frombuffer(bytes(codes), np.uint8)),
                       utf8=False, validity=None if valid.all() else valid)
    return A.fsst(A.primitive(sym_u64), A.primitive(np.array([len(y) for y in syms], np.uint8)), code_vb,
                  A.primitive(np.array(lens, np.int32)))


def _fsst_onebyte(strings, alphabet):
    """_fsst_handmade for a table of one-byte symbols (byte alphabet[i] = code i, any other byte
    escaped), vectorised."""
    lens = np.array([0 if s is None else len(s) for s in strings], np.int64)
    heap = np.frombuffer(b"".join(s or b"" for s in strings), np.uint8)
    lut = np.full(256, 255, np.int32)
    lut[np.frombuffer(alphabet, np.uint8)] = np.arange(len(alphabet))
    code = lut[heap]
    esc = code == 255
    width = 1 + esc.astype(np.int64)
    pos = np.zeros(heap.size + 1, np.int64)
    np.cumsum(width, out=pos[1:])
    codes = np.zeros(int(pos[-1]), np.uint8)
    codes[pos[:-1]] = code.astype(np.uint8)
    codes[pos[:-1][esc] + 1] = heap[esc]
    sb = np.zeros(len(strings) + 1, np.int64)
    np.cumsum(lens, out=sb[1:])
    coffs = pos[sb]
    valid = np.array([s is not None for s in strings])
    syms = [bytes([c]) for c in alphabet]
    sym_u64 = np.array([int.from_bytes(y.ljust(8, b"\0"), "little") for y in syms], np.uint64)
    code_vb = A.varbin(A.primitive(coffs.astype(np.int32)), A.primitive(codes), utf8=False,
                       validity=None if valid.all() else valid)
    return A.fsst(A.primitive(sym_u64), A.primitive(np.ones(len(syms), np.uint8)), code_vb,
                  A.primitive(lens.astype(np.int32)))


def _comment_strings(rng, n, vocab=40):
    words = [bytes(rng.integers(97, 123, rng.integers(2, 10)).astype(np.uint8)) for _ in range(vocab)]
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 8))
        out.append(b" ".join(words[j] for j in rng.integers(0, vocab, k))[: int(rng.integers(1, 44))])
    return out


@pytest.mark.parametrize("kind", ["fsst", "varbin", "dict", "varbinview", "mixed"])
def test_chunked_strings_pack_views(ctx, kind):
    """ChunkedArray of strings -> one VarBinView whose data buffers are the chunks' buffers in
    order and whose non-inlined views carry the rebased buffer_index (pack_views,
    chunked/canonical.rs:194-236); nulls in some chunks; FSST chunks have their own tables."""
    rng = np.random.default_rng(len(kind))
    chunks, strings = [], []
    for c in range(9):
        n = 3000 + 517 * c
        ss = _comment_strings(rng, n, vocab=20 + c)
        if c % 3 == 1:
            for i in rng.choice(n, n // 10, replace=False):
                ss[i] = None
        k = kind if kind != "mixed" else ["fsst", "varbin", "dict", "varbinview"][c % 4]
        if k == "fsst":
            arr = E.encode_fsst(ss)
        elif k == "varbin":
            heap, offs, valid = E.strings_to_heap(ss)
            arr = A.varbin(A.primitive(offs.astype(np.int64)), A.primitive(heap),
                           validity=None if valid.all() else valid)
        elif k == "dict":
            ss = [s if s is not None else b"" for s in ss]  # dictionary values are non-null
            uniq = sorted(set(ss))
            pos = {s: i for i, s in enumerate(uniq)}
            heap, offs, _ = E.strings_to_heap(uniq)
            values = A.varbin(A.primitive(offs.astype(np.int32)), A.primitive(heap))
            codes = np.array([pos[s] for s in ss], dtype=np.uint32)
            arr = A.dict_array(values, E.encode_bitpacked(codes, allow_patches=False))
        else:
            arr = E.encode_varbinview(ss)
        chunks.append(arr)
        strings.extend(ss)
    arr = A.chunked(chunks)
    assert_string_parity(arr, ctx, strings)


def test_fsst_escape_runs(ctx):
    # runs of 0xFF bytes escape as 255 255 pairs: code segments start inside such runs, and an
    # escape can be the last byte of a 16-byte segment (its literal in the next segment)
    rng = np.random.default_rng(7)
    strings = []
    for i in range(3000):  # ~2.6 KB of codes per 256-string tile: the staged (LDS) path
        k = int(rng.integers(0, 14))
        s = bytes(rng.choice([0xFF, 0xFE, 0x41, 0x20], size=k, p=[0.7, 0.1, 0.1, 0.1]).astype(np.uint8))
        strings.append(None if i % 97 == 3 else s)
    strings[10] = b"\xff" * 200
    arr = _fsst_handmade(strings, [b"A ", b"\xfe\xfe\xfe", b"AAAAAAAA", b" "])
    codes = arr.children[2].children[1].buffers[0]
    assert (codes == 255).mean() > 0.5
    assert_string_parity(arr, ctx, strings)


@pytest.mark.parametrize("compress_children", [False, True])
def test_fsst_many_scan_blocks(ctx, compress_children):
    # > 1024 tiles of 256 strings: the decode adds the totals of preceding scan blocks
    rng = np.random.default_rng(11)
    n = 300_000
    lens = rng.integers(0, 30, n)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    heap = rng.choice(np.frombuffer(b"abcdefgh ijkl", np.uint8), size=int(offs[-1]))
    arr = E.encode_fsst_from_heap(heap, offs, compress_children=compress_children)
    assert_string_parity(arr, ctx)


def test_fsst_chunk_and_scan_block_boundaries(ctx):
    """FSST tiles next to a chunk boundary (each chunk its own symbol table), a scan-block boundary
    inside a chunk (chunk-relative tiles 127 | 128: a different block prefix), a chunk's direct-path
    tile next to a staged one, and one-tile chunks -- in a chunked array and in a plan."""
    import torch
    rng = np.random.default_rng(31)
    sizes = [100, 40_000, 256 * 3, 513, 70]  # tiles 1, 157, 3, 3, 1
    chunks, strings = [], []
    for c, n in enumerate(sizes):
        ss = _comment_strings(rng, n, vocab=15 + 3 * c)
        if c == 3:  # long strings: one tile of this chunk overflows the LDS images (direct path)
            for i in range(256, 400):
                ss[i] = bytes(rng.integers(97, 123, 90).astype(np.uint8))
        if c in (1, 4):
            for i in rng.choice(n, n // 9, replace=False):
                ss[i] = None
        chunks.append(E.encode_fsst(ss))
        strings.extend(ss)
    arr = A.chunked(chunks)
    assert_string_parity(arr, ctx, strings)
    plan = V.Plan([arr.to(torch.device("cuda", 0))], ctx)
    res = plan.launch(sync=True)[0]
    (rv, rh), _ = canon(arr)
    assert res.numpy()[0].tobytes() == rv.tobytes()
    assert [b.tobytes() for b in res.buffers()] == [h.tobytes() for h in rh]
    plan.close()


def test_fsst_inconsistent_lengths_is_an_error(ctx):
    strings = [b"carefully final deposits"] * 600
    arr = E.encode_fsst(strings, compress_children=False)
    lens = arr.children[3].buffers[0].copy()
    lens[5] += 3  # codes no longer decode to uncompressed_lengths
    bad = A.fsst(arr.children[0], arr.children[1], arr.children[2], A.primitive(lens))
    with pytest.raises(V.VortexGpuError) as ei:
        gpu(bad, ctx)
    assert ei.value.kind == "InvalidArgument"


@pytest.mark.parametrize("escapes", [False, True])
def test_fsst_segment_sizes(ctx, escapes):
    # one-byte symbols: tile t's code span is 256 x its string length, so the staged tiles cover
    # every segment size of the decode (1..6 dwords per thread, spans 0.5..5.6 KB); with escapes
    # some tiles take the general path, and tails that end inside a segment are padded
    rng = np.random.default_rng(5 + escapes)
    alphabet = b"abcdefghij "
    strings = []
    for t, L in enumerate([2, 6, 10, 14, 18, 22, 3, 21, 0, 7]):
        for i in range(256):
            s = bytes(rng.choice(np.frombuffer(alphabet, np.uint8), L))
            if escapes and t % 2 == 1 and i % 37 == 5 and L:
                s = s[:-1] + b"\xf7"  # not a symbol: escaped
            strings.append(None if (i % 53 == 11) else s)
    strings += [b"jade"] * 77  # a partial last tile
    arr = _fsst_handmade(strings, [bytes([c]) for c in alphabet])
    codes = arr.children[2].children[1].buffers[0]
    assert ((codes == 255).any()) == escapes
    assert_string_parity(arr, ctx, strings)


def test_fsst_long_strings_direct_path(ctx):
    # strings large enough that a 256-string tile overflows the LDS images
    rng = np.random.default_rng(1)
    strings = [bytes(rng.integers(97, 123, int(rng.integers(100, 600))).astype(np.uint8)) for _ in range(700)]
    assert_string_parity(E.encode_fsst(strings), ctx, strings)


@pytest.mark.parametrize("escapes", [False, True])
def test_fsst_tile_geometry(ctx, escapes):
    """One-byte symbols make a tile's code span equal its decoded bytes: lengths that change
    every 64 strings give 256-string tiles of every code-segment size (1-6 dwords per thread),
    heap offsets of every alignment, escapes in some tiles and a partial last tile -- over 600
    tiles, i.e. several pre-pass scan blocks (a tile's heap offset is its block's prefix plus the
    tile records before it)."""
    rng = np.random.default_rng(41 + escapes)
    alphabet = b"abcdefghij "
    pattern = [3, 5, 9, 13, 15, 17, 2, 40, 1, 7, 0, 11, 60, 4, 6, 8]  # one length per tile of a range
    strings = []
    for r in range(150):  # ranges: 150 x 1024 strings (3 superblocks, the last partial)
        for t, L in enumerate(pattern[r % 3:] + pattern[:r % 3]):
            for i in range(64):
                Li = max(L + int(rng.integers(-1, 2)) * (i % 5 == 0), 0)
                s = bytes(rng.choice(np.frombuffer(alphabet, np.uint8), Li))
                if escapes and t % 3 == 1 and i % 29 == 3 and Li:
                    s = s[:-1] + b"\xf7"  # not a symbol: escaped
                strings.append(None if (i % 61 == 17) else s)
    strings += [b"tail-strings"] * 45  # partial last tile and range
    arr = _fsst_onebyte(strings, alphabet)
    if escapes:
        assert (arr.children[2].children[1].buffers[0] == 255).any()
    assert_string_parity(arr, ctx, strings)


def test_fsst_plan_replays_and_one_shots(ctx):
    """The decode's scratch (pre-pass tile records, block totals) is rewritten by every launch: a
    plan replayed many times, two plans over the same array alternated, one-shot canonicalize
    calls in between and a second plan recorded after the first one's replays -- every output
    equal to the oracle's."""
    import torch
    rng = np.random.default_rng(77)
    strings = _comment_strings(rng, 200_000, vocab=60)
    arr = E.encode_fsst(strings)
    dev = arr.to(torch_dev())
    (rv, rh), _ = canon(arr)
    p1 = V.Plan([dev], ctx)
    p2 = V.Plan([A.chunked([arr, arr]).to(torch_dev())], ctx)
    for k in range(6):
        res = p1.launch(sync=True)[0]
        assert res.numpy()[0].tobytes() == rv.tobytes(), k
        assert res.buffers()[0].tobytes() == rh.tobytes(), k
        if k % 2:
            r2 = p2.launch(sync=True)[0]
            v2 = r2.numpy()[0]
            assert [b.tobytes() for b in r2.buffers()] == [rh.tobytes()] * 2
            assert v2[: len(strings)].tobytes() == rv.tobytes()
        if k % 3 == 2:
            one = A.canonicalize(dev, ctx)
            assert one.numpy()[0].tobytes() == rv.tobytes()
    p1.close()
    p3 = V.Plan([dev], ctx)
    for _ in range(3):
        assert p3.launch(sync=True)[0].numpy()[0].tobytes() == rv.tobytes()
    p3.close()
    p2.close()


# ------------------------------------------------------------------ direct C-ABI entry points
def test_direct_bitunpack_entry(ctx):
    import torch
    lib = V.gpu_lib()
    vals = (np.arange(1 << 16, dtype=np.uint32) * 2654435761 % 128).astype(np.uint32)
    packed = E.bitpack_buffer(vals, 7)
    dp = torch.from_numpy(packed).cuda()
    out = torch.empty(vals.size * 4, dtype=torch.uint8, device="cuda")
    st = lib.vxg_bitunpack(ctx.handle, V.PTYPE["u32"], 7, 0, vals.size, C.c_void_p(dp.data_ptr()),
                           packed.size, C.c_void_p(out.data_ptr()), ctx.stream_ptr())
    assert st == 0
    ctx.sync()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), vals)
    # wrong packed length is rejected like BitPackedArray::try_new (bitpacking/mod.rs:80-88)
    st = lib.vxg_bitunpack(ctx.handle, V.PTYPE["u32"], 7, 0, vals.size + 5000, C.c_void_p(dp.data_ptr()),
                           packed.size, C.c_void_p(out.data_ptr()), ctx.stream_ptr())
    assert st == 3 and b"packed bytes" in lib.vxg_last_error()


def _bench():
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import bench
    return bench


def test_full_size_c1_roundtrip(ctx):
    """BASELINE config 1 at full size (64 Mi u32, W=7, the bench's generator): bit-exact against
    the oracle's decode of the same packed bytes, plus the size-independent properties
    (exact roundtrip to the plain values, checksum)."""
    rng = np.random.default_rng(42)
    vals = rng.integers(0, 128, 64 << 20, dtype=np.uint32)
    arr = E.encode_bitpacked(vals, bit_width=7, allow_patches=False)
    got = gpu(arr, ctx).numpy()
    ref, _ = canon(arr)
    assert got.tobytes() == ref.tobytes()
    assert got.tobytes() == vals.tobytes()
    assert int(got.astype(np.uint64).sum()) == int(vals.astype(np.uint64).sum())


def test_full_size_c2_alp(ctx):
    """BASELINE config 2 at full size: 64 Mi f64 prices + 0.1 % exceptions (bench generator),
    ALP -> FoR -> BitPacked(u64) + patches: bit-exact against the oracle and the plain values."""
    b = _bench()
    vals = b.c2_values(np.random.default_rng(42), 64 << 20)
    arr = E.encode_alp(vals)
    got = gpu(arr, ctx).numpy()
    assert got.tobytes() == vals.tobytes()
    assert got.tobytes() == canon(arr)[0].tobytes()


def test_full_size_c3_dict_chunks(ctx):
    """BASELINE config 3 at full size: the 256-chunk Dict(BitPacked u64 W=10) table (128 Mi
    values), decoded as one plan over a device chunk table and directly; each chunk equals
    take(values, codes) of its plain data."""
    import torch
    b = _bench()
    plains = [b.c3_chunk_plain(c) for c in range(b.C3_CHUNKS)]
    arr = A.chunked([b.c3_chunk(c, p) for c, p in enumerate(plains)])
    dev = arr.to(torch.device("cuda", 0))
    plan = V.Plan([dev], ctx)
    got = plan.launch(sync=True)[0].numpy()
    plan.close()
    n = b.C3_CHUNK_VALUES
    for c, (dv, codes) in enumerate(plains):
        assert got[c * n:(c + 1) * n].tobytes() == dv[codes].tobytes(), c
    assert V.canonicalize(dev, ctx).numpy().tobytes() == got.tobytes()


def test_full_size_c4_fsst(ctx):
    """BASELINE config 4 at full size: 6 001 215 l_comment-like strings, FSST: the data buffer
    equals the plain heap, views equal make_view over it (bench.expected_views), and the oracle."""
    b = _bench()
    heap, offs = b.c4_heap(np.random.default_rng(42), 6_001_215)
    arr = E.encode_fsst_from_heap(heap, offs)
    res = gpu(arr, ctx)
    views, _ = res.numpy()
    bufs = res.buffers()
    assert len(bufs) == 1 and bufs[0].tobytes() == heap.tobytes()
    assert views.tobytes() == b.expected_views(heap, offs).tobytes()
    (rviews, rheap), _ = canon(arr)
    assert views.tobytes() == rviews.tobytes()


# ------------------------------------------------------------------ C5: TPC-H lineitem scan
def test_lineitem_scan_every_column(ctx):
    """BASELINE C5 at reduced size: all 16 lineitem columns (tools/lineitem.py cascades:
    RunEnd, FoR/BitPacked, ALP, Dict(VarBin), FSST), 3 chunks of 8 Ki rows (one ragged), each
    column canonicalized through the C ABI and compared with the oracle and the plain values."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from tools import lineitem as L
    rows, cr = 2 * 8192 + 777, 8192
    cols, plain = L.lineitem_columns(range(L.n_chunks(rows, cr)), rows=rows, chunk_rows=cr)
    for name, kind in L.COLUMNS:
        arr = cols[name]
        if kind == "utf8":
            strings = [s for part in plain[name] for s in part]
            assert_string_parity(arr, ctx, strings)
        else:
            assert_primitive_parity(arr, ctx, np.concatenate(plain[name]))


@pytest.mark.parametrize("mean_run", [1, 4, 16, 17, 300])
def test_runend_run_length_regimes(ctx, mean_run):
    """Short runs (mean <= 16 rows) expand thread-per-run, long runs by output span: both forms,
    single arrays and chunks, sliced, and ends that stop short of the length (error)."""
    rng = np.random.default_rng(mean_run)
    n_runs = 5000
    lens = rng.integers(1, 2 * mean_run, n_runs) if mean_run > 1 else np.ones(n_runs, np.int64)
    vals = np.repeat(rng.integers(-10**12, 10**12, n_runs).astype(np.int64), lens)
    arr = E.encode_runend(vals)
    assert_primitive_parity(arr, ctx, vals)
    ends, rv = E.runend_encode(vals)
    # RunEndArray::slice (runend/compute.rs:98-110): runs from the one holding `start`, ends absolute
    start, length = 5, vals.size - 9
    sb = int(np.searchsorted(ends, start, side="right"))
    sl = A.run_end(A.primitive(ends[sb:]), A.primitive(rv[sb:]), length=length, offset=start)
    assert_primitive_parity(sl, ctx, vals[start:start + length])
    ch = A.chunked([E.encode_runend(vals[:7000]), sl])
    assert_primitive_parity(ch, ctx, np.concatenate([vals[:7000], vals[start:start + length]]))
    short = A.run_end(A.primitive(ends), A.primitive(rv), length=int(ends[-1]) + 3)
    with pytest.raises(V.VortexGpuError) as ei:
        gpu(short, ctx)
    assert ei.value.kind == "InvalidArgument"


@pytest.mark.parametrize("case", ["max_direct", "one_long", "windows"])
def test_runend_short_runs_window_shapes(ctx, case):
    """K8r (runend_runs.hpp) at run-length shapes its 4,096-row windows meet: runs of exactly 32
    rows among short ones, single 33-40-row runs among 1-7-row runs, and 1-15-row runs whose
    1,024-run workgroups span two or three windows (a run carried across a window edge); plain,
    FoR-packed values, sliced and chunked.  (Written for round 6's rejected direct head fill,
    profiles/r06_k8r_direct_fill.md; kept as coverage of the max-scan form.)"""
    rng = np.random.default_rng({"max_direct": 1, "one_long": 2, "windows": 3}[case])
    n_runs = 6000
    if case == "max_direct":
        lens = np.where(rng.random(n_runs) < 0.3, 32, rng.integers(1, 8, n_runs))
    elif case == "one_long":
        lens = rng.integers(1, 8, n_runs)
        lens[[100, 2500, 5000]] = [33, 40, 33]
    else:
        lens = rng.integers(1, 16, n_runs)
    vals = np.repeat(rng.integers(-10**12, 10**12, n_runs).astype(np.int64), lens)
    for compress in (False, True):
        arr = E.encode_runend(vals, compress_values=compress)
        assert_primitive_parity(arr, ctx, vals)
    ends, rv = E.runend_encode(vals)
    start, length = 37, vals.size - 50
    sb = int(np.searchsorted(ends, start, side="right"))
    sl = A.run_end(A.primitive(ends[sb:]), A.primitive(rv[sb:]), length=length, offset=start)
    assert_primitive_parity(sl, ctx, vals[start:start + length])
    ch = A.chunked([E.encode_runend(vals[:9000], compress_values=True), sl])
    assert_primitive_parity(ch, ctx, np.concatenate([vals[:9000], vals[start:start + length]]))


def _slice_bitpacked(bp, start, length):
    """BitPackedArray::slice (bitpacking/compute/slice.rs): whole blocks from the one holding
    `start`, offset = start % 1024."""
    w = bp.meta["bit_width"]
    b0, b1 = start // 1024, (start + length + 1023) // 1024
    packed = bp.buffers[0][b0 * 128 * w: b1 * 128 * w]
    return A.bitpacked(packed, bp.ptype, w, length, offset=start % 1024)


@pytest.mark.parametrize("vdt", [np.int32, np.uint32, np.int64, np.uint64, np.float64])
def test_runend_short_runs_packed_children_in_place(ctx, vdt):
    """Short-run RunEnd whose ends are BitPacked and values FoR(BitPacked) (C5's l_orderkey):
    the runs kernel unpacks both children in place.  Single arrays and chunks, children sliced
    inside a FastLanes block (BitPacked offset), FoR with negative references, float values
    (plain bits), and a chunk mix with long-run chunks (plain temporaries)."""
    rng = np.random.default_rng(np.dtype(vdt).itemsize * 7 + (vdt == np.float64))
    n_runs = 9000
    lens = rng.integers(1, 8, n_runs)
    if vdt == np.float64:
        rv = rng.standard_normal(n_runs)
    else:
        lo = -(1 << 20) if np.dtype(vdt).kind == "i" else 0
        rv = rng.integers(lo, 1 << 21, n_runs).astype(vdt)
    vals = np.repeat(rv, lens)
    arr = E.encode_runend(vals, compress_values=True)
    assert_primitive_parity(arr, ctx, vals)
    ends, rvv = E.runend_encode(vals)
    # children sliced at a non-block boundary: runs [sb, sb + m) of the full encoding
    sb, m = 1500, 6000
    e_full = E.encode_bitpacked(ends, allow_patches=False)
    e_sl = _slice_bitpacked(e_full, sb, m)
    if rvv.dtype.kind in "iu":
        v_full = E.encode_for_bitpacked(rvv)
        inner = _slice_bitpacked(v_full.children[0], sb, m)
        v_sl = dataclasses.replace(v_full, len=m, children=[inner])  # FoRArray::slice
    else:
        v_sl = A.primitive(rvv[sb:sb + m])
    start = int(ends[sb - 1]) + 2  # a slice starting inside run sb
    length = int(ends[sb + m - 1]) - start - 3
    sl = A.run_end(e_sl, v_sl, length=length, offset=start)
    assert_primitive_parity(sl, ctx, vals[start:start + length])
    long_vals = np.repeat(rv[:200], 50)
    ch = A.chunked([arr, sl, E.encode_runend(long_vals, compress_values=True), arr])
    assert_primitive_parity(ch, ctx, np.concatenate([vals, vals[start:start + length], long_vals, vals]))


def test_chunked_runend_batched(ctx):
    """Chunked[RunEnd]: ends/values decoded with the other chunks' K1 launches into one
    temporary, expansions in shared launches; sliced chunks (offset) and primitive children."""
    rng = np.random.default_rng(21)
    chunks, expect = [], []
    for c in range(60):
        n = 5000 + 333 * c
        v = np.repeat(rng.integers(-10 ** 6, 10 ** 6, n), rng.integers(1, 6, n))[:n].astype(np.int64)
        arr = E.encode_runend(v, compress_values=c % 2 == 0, bitpack_ends=c % 3 != 0)
        if c % 5 == 4:  # RunEndArray::slice (runend/compute.rs:98-110): runs from the one holding
            ends, rv = E.runend_encode(v)  # `start`, offset = start, ends stay absolute
            sb = int(np.searchsorted(ends, 7, side="right"))
            arr = A.run_end(E.encode_bitpacked(ends[sb:], allow_patches=False), A.primitive(rv[sb:]),
                            length=n - 20, offset=7)
            v = v[7: 7 + n - 20]
        chunks.append(arr)
        expect.append(v)
    assert_primitive_parity(A.chunked(chunks), ctx, np.concatenate(expect))


def sys_path_bench():
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parent.parent)
    if root not in sys.path:
        sys.path.insert(0, root)


class plan_mode:
    """VXG_PLAN_BATCH for the plans created inside (capi.hip reads it at every vxg_plan_create):
    "0" unbatched, "1" batched, "mixed", None = the default (plain create: the batched
    candidate; measure=True: both recorded, vxg_plan_select keeps one)."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        import os
        self.old = os.environ.get("VXG_PLAN_BATCH")
        if self.mode is None:
            os.environ.pop("VXG_PLAN_BATCH", None)
        else:
            os.environ["VXG_PLAN_BATCH"] = self.mode

    def __exit__(self, *exc):
        import os
        if self.old is None:
            os.environ.pop("VXG_PLAN_BATCH", None)
        else:
            os.environ["VXG_PLAN_BATCH"] = self.old


def test_plan_graph_replay_matches_direct(ctx):
    """vxg_plan: the recorded HIP graph reproduces vxg_canonicalize's bytes on every replay,
    and a replay reads the CURRENT contents of the input buffers (new batch, same buffers)."""
    import torch
    rng = np.random.default_rng(31)
    vals = rng.integers(0, 1 << 11, 70_000, dtype=np.uint64).astype(np.uint32)
    prices = np.round(rng.uniform(0, 1000, 50_000), 2)
    strings = [None if i % 17 == 0 else b"row-%d-" % i * (1 + i % 5) for i in range(20_000)]
    arrs = [E.encode_bitpacked(vals, bit_width=11, allow_patches=False), E.encode_alp(prices),
            A.chunked([E.encode_fsst(strings[:9000]), E.encode_fsst(strings[9000:])])]
    dev = [a.to(torch.device("cuda", 0)) for a in arrs]
    plan = V.Plan(dev, ctx)
    for _ in range(3):
        res = plan.launch(sync=True)
        assert res[0].numpy().tobytes() == vals.tobytes()
        assert res[1].numpy().tobytes() == prices.tobytes()
        views, _ = res[2].numpy()
        (rviews, rheap), rvalid = canon(arrs[2])
        assert views.tobytes() == rviews.tobytes()
        assert [b.tobytes() for b in res[2].buffers()] == [b.tobytes() for b in rheap]
        assert np.array_equal(res[2].validity_mask(), rvalid)
    # new batch in place: same shapes, different packed values
    vals2 = rng.integers(0, 1 << 11, 70_000, dtype=np.uint64).astype(np.uint32)
    new = E.encode_bitpacked(vals2, bit_width=11, allow_patches=False)
    dev[0].buffers[0].copy_(torch.from_numpy(np.ascontiguousarray(new.buffers[0]).view(np.uint8).reshape(-1).copy()))
    assert plan.launch(sync=True)[0].numpy().tobytes() == vals2.tobytes()
    plan.close()


@contextlib.contextmanager
def env_set(**kv):
    """Environment variables set for the block (the planner reads these at plan recording)."""
    import os
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update({k: str(v) for k, v in kv.items()})
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("fuse,prepass", [("1", "ingrid"), ("1", "separate"), ("0", "separate")])
def test_plan_fused_fsst_k1g(ctx, fuse, prepass):
    """A batched plan decodes one FSST accessor group's tiles inside its K1g launch
    (fsst_k1g_kernel, the tiles spread between the K1g workgroups): lineitem columns (Dict(VarBin)
    strings, RunEnd, numeric cascades -- K1g jobs) beside chunked FSST columns with FastLanes-
    packed offsets/lengths (the fused group), plain i32 offsets/lengths (a second group: its own
    launch), nulls and ragged chunk sizes, and a FSST-only plan (a K1g launch with no K1g jobs).
    `ingrid` (round 6, the default for groups of <= 8,192 tiles): the group's length pre-pass runs
    as the fused launch's first workgroups, 32 tiles each (a 31,000-string chunk is 4 such scan
    blocks), publishing tagged records the tiles wait for; `separate`: its own kernel before.
    VXG_PLAN_FUSE=0 records the unfused form; all equal the oracle on every replay."""
    import torch
    sys_path_bench()
    from tools import lineitem as L
    rows, cr = 5 * 4096 + 11, 4096
    cols, plain_vals = L.lineitem_columns(range(L.n_chunks(rows, cr)), rows=rows, chunk_rows=cr)
    rng = np.random.default_rng(505)
    strs = _comment_strings(rng, 60_000, vocab=80)
    strs = [None if i % 23 == 5 else x for i, x in enumerate(strs)]
    cuts = [0, 6, 9_000, 9_257, 40_000, 60_000]  # every chunk holds a null (one nullable dtype)
    packed = A.chunked([E.encode_fsst(strs[a:b]) for a, b in zip(cuts, cuts[1:])])
    plain = A.chunked([E.encode_fsst(strs[a:b], compress_children=False) for a, b in zip(cuts[:3], cuts[1:4])])
    arrs = [cols[name] for name, _ in L.COLUMNS] + [packed, plain]
    kinds = [kind for _, kind in L.COLUMNS] + ["utf8", "utf8"]
    with env_set(VXG_PLAN_FUSE=fuse, VXG_FUSED_PREPASS_MAX_TILES=8192 if prepass == "ingrid" else 0):
        with plan_mode("1"):
            plans = [V.Plan([a.to(torch_dev()) for a in arrs], ctx), V.Plan([packed.to(torch_dev())], ctx)]
    assert all(p.info()["batched"] for p in plans)
    want = [canon(a) if k == "utf8" else np.concatenate(plain_vals[n]) for a, k, n in
            zip(arrs, kinds, [name for name, _ in L.COLUMNS] + ["", ""])]
    for _ in range(3):
        for plan, idx in zip(plans, ([*range(len(arrs))], [len(arrs) - 2])):
            res = plan.launch(sync=True)
            for r, i in zip(res, idx):
                if kinds[i] == "utf8":
                    (rviews, rbufs), rvalid = want[i]
                    assert r.numpy()[0].tobytes() == rviews.tobytes(), i
                    assert [b.tobytes() for b in r.buffers()] == [b.tobytes() for b in rbufs], i
                    assert np.array_equal(r.validity_mask(), rvalid), i
                else:
                    assert r.numpy().tobytes() == want[i].tobytes(), i
    for p in plans:
        p.close()


def test_plan_fused_prepass_length_widths(ctx):
    """The in-grid pre-pass's FastLanes length body at the edges of its shapes: a chunk of
    constant-length strings (FoR lengths of bit width 0: no words staged), a chunk whose lengths
    need ~18 bits (a 200 KB string every 97 rows: those tiles take the direct per-string path),
    and chunks of exactly one 32-tile scan block (8,192 strings) and one string more (a second
    block of one tile), with nulls; three replays equal the oracle."""
    rng = np.random.default_rng(1818)
    const = [b"abcdefgh!" for _ in range(3_000)]
    longs = _comment_strings(rng, 2_000, vocab=40)
    longs = [bytes(rng.integers(97, 123, 200_000).astype(np.uint8)) if i % 97 == 13 else x for i, x in enumerate(longs)]
    b1 = _comment_strings(rng, 8_192, vocab=60)
    b2 = [None if i % 31 == 7 else x for i, x in enumerate(_comment_strings(rng, 8_193, vocab=60))]
    chunks = [E.encode_fsst(c) for c in (const, longs, b1, b2)]
    lw = [c.children[-1].children[0].meta["bit_width"] if c.children[-1].children else None for c in chunks]
    fs = A.chunked(chunks)
    with env_set(VXG_FUSED_PREPASS_MAX_TILES=8192), plan_mode("1"):
        plan = V.Plan([fs.to(torch_dev())], ctx)
    (rv, rb), rvalid = canon(fs)
    for _ in range(3):
        r = plan.launch(sync=True)[0]
        assert r.numpy()[0].tobytes() == rv.tobytes(), lw
        assert [b.tobytes() for b in r.buffers()] == [b.tobytes() for b in rb], lw
        assert np.array_equal(r.validity_mask(), rvalid)
    plan.close()


def test_plan_fused_prepass_graph_replay(ctx):
    """A plan that replays as a HIP graph (VXG_PLAN_DIRECT=0) gives its fused launch's in-grid
    pre-pass a new record tag per replay through hipGraphExecKernelNodeSetParams: replays of
    lineitem-like columns beside a chunked FSST column equal the oracle, with no device error."""
    rng = np.random.default_rng(4711)
    strs = _comment_strings(rng, 20_000, vocab=50)
    strs = [None if i % 17 == 3 else x for i, x in enumerate(strs)]
    fs = A.chunked([E.encode_fsst(strs[a:b]) for a, b in ((0, 7_000), (7_000, 7_001), (7_001, 20_000))])
    codes = A.chunked([E.encode_bitpacked(rng.integers(0, 1000, 9_000).astype(np.uint32), bit_width=10,
                                          allow_patches=False) for _ in range(3)])
    with env_set(VXG_PLAN_DIRECT=0, VXG_FUSED_PREPASS_MAX_TILES=8192), plan_mode("1"):
        plan = V.Plan([fs.to(torch_dev()), codes.to(torch_dev())], ctx)
    info = plan.info()
    assert info["batched"] and info["direct_nodes"] == 0, info
    (rv, rb), rvalid = canon(fs)
    for _ in range(4):
        r = plan.launch(sync=True)[0]
        assert r.numpy()[0].tobytes() == rv.tobytes() and [b.tobytes() for b in r.buffers()] == [b.tobytes() for b in rb]
        assert np.array_equal(r.validity_mask(), rvalid)
    plan.close()


def test_plan_fused_prepass_tag_wraps(ctx):
    """The in-grid pre-pass's record tag (1-65535) is advanced by every vxg_plan_launch: 65,600
    back-to-back replays of a small fused plan (a FSST column beside a K1g job) wrap it.  Every
    replay's tiles find records carrying their own tag (a wait that never ends reports
    kErrPlanSync, which the synchronising launch would raise) and the last replay equals the
    oracle."""
    rng = np.random.default_rng(65600)
    s1 = _comment_strings(rng, 3_000, vocab=30)
    codes = A.chunked([E.encode_bitpacked(rng.integers(0, 100, 5_000).astype(np.uint32), bit_width=7,
                                          allow_patches=False) for _ in range(2)])
    f1 = A.chunked([E.encode_fsst(s1[:1_000]), E.encode_fsst(s1[1_000:])])
    with env_set(VXG_FUSED_PREPASS_MAX_TILES=8192), plan_mode("1"):
        d1 = f1.to(torch_dev())
        plan = V.Plan([d1, codes.to(torch_dev())], ctx)
    assert plan.info()["batched"]
    for _ in range(65_600):
        plan.launch(sync=False)
    ctx.sync()
    (rv, rb), _ = canon(f1)
    r = plan.launch(sync=True)[0]
    assert r.numpy()[0].tobytes() == rv.tobytes() and [b.tobytes() for b in r.buffers()] == [b.tobytes() for b in rb]
    plan.close()


@pytest.mark.parametrize("rows,cr", [(3 * 8192 + 99, 8192), (100 * 1024 + 77, 1024)])
def test_plan_lineitem_columns(ctx, rows, cr):
    """vxg_plan over the lineitem columns (RunEnd, Dict strings, FSST chunks: planner
    temporaries live with the plan) equals the oracle on every replay.  101 chunks per column
    exceed every kernel-argument table (K1 32, FSST 24, RunEnd/VarBin 48): the plan records
    one launch per kernel group over a device-resident chunk table."""
    import sys
    import torch
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from tools import lineitem as L
    cols, plain = L.lineitem_columns(range(L.n_chunks(rows, cr)), rows=rows, chunk_rows=cr)
    arrs = [cols[name] for name, _ in L.COLUMNS]
    plan = V.Plan([a.to(torch.device("cuda", 0)) for a in arrs], ctx)
    for _ in range(2):
        res = plan.launch(sync=True)
        for (name, kind), a, r in zip(L.COLUMNS, arrs, res):
            if kind == "utf8":
                (rviews, rbufs), _ = canon(a)
                assert r.numpy()[0].tobytes() == rviews.tobytes(), name
                assert [b.tobytes() for b in r.buffers()] == [b.tobytes() for b in rbufs], name
            else:
                assert r.numpy().tobytes() == np.concatenate(plain[name]).tobytes(), name
    plan.close()


def _k1g_columns(rng):
    """Chunked columns covering every K1g body (k1g.hip): T = 8..64 bits plain / FoR / ZigZag,
    ALP f32 / f64, Dict with 1/2/4/8-byte values and string dictionaries (16-byte views), with
    ragged chunk lengths, an empty chunk and sliced BitPacked chunks (offset > 0)."""
    lens = [1000, 2500, 1024, 0, 3, 7000]
    cols = []

    def chunked(make):
        arrs, exp = [], []
        for n in lens:
            a, v = make(n)
            arrs.append(a)
            exp.append(v)
        return A.chunked(arrs), np.concatenate(exp)

    for dt in (np.uint8, np.uint16, np.uint32, np.uint64):
        bits = np.iinfo(dt).bits
        for W in (1, bits // 2 + 1, bits - 1):
            def mk(n, dt=dt, W=W):
                v = rng.integers(0, 1 << W, n, dtype=np.uint64).astype(dt)
                off = int(rng.integers(1, 1000)) if n > 2000 else 0  # sliced chunk
                return E.encode_bitpacked(v, bit_width=W, allow_patches=False, offset=off), v
            cols.append(chunked(mk))
    for dt in (np.int8, np.int16, np.int32, np.int64):
        lo = int(np.iinfo(dt).min) // 2
        cols.append(chunked(lambda n, dt=dt, lo=lo: (lambda v: (E.encode_for_bitpacked(v, allow_patches=False), v))(
            (lo + 3 * rng.integers(0, 40, n)).astype(dt))))
        cols.append(chunked(lambda n, dt=dt: (lambda v: (E.encode_zigzag(v), v))(
            (rng.integers(-60, 60, n)).astype(dt))))
    for ft in (np.float64, np.float32):
        cols.append(chunked(lambda n, ft=ft: (lambda v: (E.encode_alp(v), v))(
            (np.round(rng.uniform(0, 1000, n) * 100) / 100).astype(ft))))
    for vdt in (np.uint8, np.int16, np.uint32, np.int64):
        pool = np.unique(rng.integers(0, 100, 64).astype(vdt))
        cols.append(chunked(lambda n, pool=pool: (lambda v: (E.encode_dict(v), v))(pool[rng.integers(0, pool.size, n)])))
    return cols


def test_plan_k1g_every_kind(ctx):
    """A plan of small chunked columns: their K1 decodes are batched across columns onto one graph
    branch and run as ONE K1g launch (runtime T / W / epilogue per chunk table entry); every
    column equals the oracle, string dictionaries included."""
    import torch
    rng = np.random.default_rng(77)
    cols = _k1g_columns(rng)
    words = [b"DELIVER IN PERSON", b"NONE", b"TAKE BACK RETURN", b"COLLECT COD"]
    strs = [[words[i] for i in rng.integers(0, 4, n)] for n in (3000, 1, 5000)]
    sarr = A.chunked([E.encode_dict_strings(s) for s in strs])
    arrs = [c for c, _ in cols] + [sarr]
    with plan_mode("1"):
        plan = V.Plan([a.to(torch.device("cuda", 0)) for a in arrs], ctx)
    for _ in range(2):
        res = plan.launch(sync=True)
        for k, ((a, exp), r) in enumerate(zip(cols, res)):
            got = r.numpy()
            ref, _ = canon(a)
            assert got.tobytes() == ref.tobytes() == exp.tobytes(), (k, a.children[1].encoding)
        (rviews, rbufs), _ = canon(sarr)
        assert res[-1].numpy()[0].tobytes() == rviews.tobytes()
        assert [b.tobytes() for b in res[-1].buffers()] == [b.tobytes() for b in rbufs]
    plan.close()


@pytest.mark.parametrize("sizes", [[8192] * 6 + [5000], [8192] * 5 + [12288], [8192], [8192, 4096, 8192]])
def test_plan_string_dict_job_lookup(ctx, sizes):
    """Unbatched plans run each chunked Dict(VarBin) column as one K1g launch whose workgroups
    find their chunk directly when every chunk but the last spans the same workgroups (last chunk
    smaller: direct; a larger last chunk, a single chunk or unequal chunks: the fallback count).
    Every view and byte equals the oracle."""
    import torch
    rng = np.random.default_rng(88)
    words = [b"DELIVER IN PERSON", b"NONE", b"TAKE BACK RETURN", b"COLLECT COD", b"x" * 30]
    strs = [[words[i] for i in rng.integers(0, len(words), n)] for n in sizes]
    sarr = A.chunked([E.encode_dict_strings(s) for s in strs])
    with plan_mode("0"):
        plan = V.Plan([sarr.to(torch.device("cuda", 0))], ctx)
    res = plan.launch(sync=True)[0]
    (rviews, rbufs), _ = canon(sarr)
    assert res.numpy()[0].tobytes() == rviews.tobytes()
    assert [b.tobytes() for b in res.buffers()] == [b.tobytes() for b in rbufs]
    plan.close()


@pytest.mark.parametrize("mode", ["0", "1"])
@pytest.mark.parametrize("n_words,wlen", [(300, 20), (1000, 20)], ids=["bytes_gt_2k", "views_bytes_gt_16k"])
def test_plan_string_dict_large_dictionary(ctx, mode, n_words, wlen):
    """K1g builds a Dict(VarBin) column's views from LDS only when the dictionary
    bytes fit (<= 2 KiB beside the views in 16 KiB); larger dictionaries take the global-memory
    branch (views read their bytes from HBM).  300 distinct 20-byte words (6 KB of bytes) and
    1000 (views + bytes > 16 KiB), unbatched (one K1g per column) and batched: every view and
    byte equals the oracle."""
    import torch
    rng = np.random.default_rng(89 + n_words)
    words = [(b"w%05d-" % i + bytes(rng.integers(97, 123, wlen - 7, dtype=np.uint8))) for i in range(n_words)]
    strs = [[words[i] for i in rng.integers(0, n_words, n)] for n in (70_000, 65_536, 1234)]
    sarr = A.chunked([E.encode_dict_strings(s) for s in strs])
    with plan_mode(mode):
        plan = V.Plan([sarr.to(torch.device("cuda", 0))], ctx)
    res = plan.launch(sync=True)[0]
    (rviews, rbufs), _ = canon(sarr)
    assert res.numpy()[0].tobytes() == rviews.tobytes()
    assert [b.tobytes() for b in res.buffers()] == [b.tobytes() for b in rbufs]
    plan.close()


@pytest.mark.parametrize("mode", ["0", "1"])
@pytest.mark.parametrize("n_words", [5, 300])
def test_plan_string_dict_bad_offsets(ctx, mode, n_words):
    """A Dict(VarBin) dictionary whose offsets run past its bytes is reported by the plan's
    replay as 'VarBin offsets out of range' (LDS and global-memory K1g branches)."""
    import torch
    rng = np.random.default_rng(90)
    words = [b"word-%04d-abcdefghij" % i for i in range(n_words)]
    chunks = []
    for n in (40_000, 5_000):
        d = E.encode_dict_strings([words[i] for i in rng.integers(0, n_words, n)])
        vb = d.children[0]
        offs = np.ascontiguousarray(vb.children[0].buffers[0]).view(A.NP_OF_PTYPE[vb.children[0].ptype]).copy()
        offs[len(offs) // 2] = offs[-1] + 5000  # past the end of the bytes
        vb.children[0] = A.primitive(offs)
        chunks.append(d)
    with plan_mode(mode):
        plan = V.Plan([A.chunked(chunks).to(torch.device("cuda", 0))], ctx)
    with pytest.raises(V.VortexGpuError, match="VarBin offsets out of range"):
        plan.launch(sync=True)
    ctx.sync()
    plan.close()


def test_plan_mixed_large_and_small_arrays(ctx):
    """A plan with a 21 MB chunked array (22 K1 chunks) next to small columns of every K1g body:
    batched together (K1 launch groups for the large group, one K1g launch for the rest), every
    replay equal to the oracle."""
    import torch
    rng = np.random.default_rng(91)
    big = rng.integers(0, 1 << 13, 5_300_000, dtype=np.uint64).astype(np.uint32)  # 21 MB of u32
    big_arr = A.chunked([E.encode_bitpacked(big[i:i + (1 << 20)], bit_width=13, allow_patches=False)
                         for i in range(0, big.size, 1 << 20)])
    cols = _k1g_columns(rng)[:6]
    arrs = [big_arr] + [c for c, _ in cols]
    with plan_mode("1"):
        plan = V.Plan([a.to(torch.device("cuda", 0)) for a in arrs], ctx)
    for _ in range(2):
        res = plan.launch(sync=True)
        assert res[0].numpy().tobytes() == big.tobytes()
        for (a, exp), r in zip(cols, res[1:]):
            assert r.numpy().tobytes() == exp.tobytes()
    plan.close()


def _nested_chunked_arrays(rng):
    """Trees whose ChunkedArray is NOT the root: a consumer kernel reads its decoded output right
    after it (Dict values, FoR / ZigZag / ALP children, RunEnd ends and values, Sparse indices,
    a string dictionary's values).  Under PlanBatch only a root ChunkedArray may defer its
    launches to the end of the plan (nested deferral read unwritten temporaries)."""
    def bp_chunks(v, W, sizes):
        out, at = [], 0
        for n in sizes:
            out.append(E.encode_bitpacked(v[at:at + n], bit_width=W, allow_patches=False))
            at += n
        return A.chunked(out)

    cases = []
    # Dict(values = Chunked[u32], codes = BitPacked u16)
    dv = rng.integers(0, 1 << 20, 3000, dtype=np.uint64).astype(np.uint32)
    codes = rng.integers(0, dv.size, 40_000).astype(np.uint16)
    cases.append((A.dict_array(bp_chunks(dv, 20, [1000, 1500, 500]),
                               E.encode_bitpacked(codes, bit_width=12, allow_patches=False)), dv[codes]))
    # FoR(i64) over Chunked[BitPacked u64]
    raw = rng.integers(0, 1 << 9, 50_000, dtype=np.uint64)
    ref = -123_456_789
    cases.append((A.frame_of_reference(bp_chunks(raw, 9, [20_000, 1024, 28_976]), ref, 0, "i64"),
                  raw.view(np.int64) + ref))
    # ZigZag(i32) over Chunked[BitPacked u32]
    zz = rng.integers(-500, 500, 30_000).astype(np.int32)
    zu = ((zz.astype(np.int64) << 1) ^ (zz.astype(np.int64) >> 63)).astype(np.uint32)
    cases.append((A.zigzag(bp_chunks(zu, 10, [10_000, 20_000])), zz))
    # ALP(f64) over Chunked[FoR(BitPacked)] encoded ints
    prices = np.round(rng.uniform(0, 1000, 20_000) * 100) / 100
    e, f, enc, _, _ = E.alp_encode(prices)
    assert enc.size == prices.size
    enc = enc.astype(np.int64)
    cases.append((A.alp(A.chunked([E.encode_for_bitpacked(enc[:7000], allow_patches=False),
                                   E.encode_for_bitpacked(enc[7000:], allow_patches=False)]), e, f), None))
    # RunEnd(ends = Chunked, values = Chunked)
    runs = rng.integers(1, 9, 4000)
    ends = np.cumsum(runs).astype(np.uint64)
    rvals = rng.integers(0, 1 << 30, runs.size, dtype=np.uint64).astype(np.uint32)
    cases.append((A.run_end(bp_chunks(ends, 15, [1500, 2500]), bp_chunks(rvals, 30, [2000, 2000]), int(ends[-1])),
                  np.repeat(rvals, runs)))
    # Sparse(u16) with Chunked indices
    idx = np.sort(rng.choice(60_000, 700, replace=False)).astype(np.uint64)
    sv = rng.integers(1, 1 << 16, idx.size, dtype=np.uint64).astype(np.uint16)
    expect = np.zeros(60_000, np.uint16)
    expect[idx] = sv
    cases.append((A.sparse(bp_chunks(idx, 16, [300, 400]), A.primitive(sv), 60_000), expect))
    return cases


def test_plan_nested_chunked_not_deferred(ctx):
    """A plan with a root ChunkedArray (batching on) and trees holding NESTED ChunkedArrays:
    every replay equals the oracle and vxg_canonicalize, for primitive and string trees."""
    import torch
    rng = np.random.default_rng(2024)
    cases = _nested_chunked_arrays(rng)
    root = A.chunked([E.encode_bitpacked(rng.integers(0, 1 << 7, n, dtype=np.uint64).astype(np.uint32),
                                         bit_width=7, allow_patches=False) for n in (5000, 3000)])
    words = [b"DELIVER IN PERSON", b"NONE", b"TAKE BACK RETURN", b"COLLECT COD", b"x" * 40]
    sdict = A.chunked([E.encode_dict_strings([words[i] for i in rng.integers(0, 5, n)]).children[0]
                       for n in (3, 4)])  # Chunked[VarBin] dictionary values
    scodes = rng.integers(0, sdict.len, 9000).astype(np.uint8)
    sarr = A.dict_array(sdict, E.encode_bitpacked(scodes, bit_width=3, allow_patches=False))
    arrs = [root] + [a for a, _ in cases] + [sarr]
    with plan_mode("1"):
        plan = V.Plan([a.to(torch.device("cuda", 0)) for a in arrs], ctx)
    for _ in range(3):
        res = plan.launch(sync=True)
        assert res[0].numpy().tobytes() == canon(root)[0].tobytes()
        for k, ((a, exp), r) in enumerate(zip(cases, res[1:-1])):
            got = r.numpy()
            ref, _ = canon(a)
            assert got.tobytes() == ref.tobytes(), k
            assert got.tobytes() == gpu(a, ctx).numpy().tobytes(), k
            if exp is not None:
                assert got.tobytes() == np.ascontiguousarray(exp).tobytes(), k
        (rviews, rbufs), _ = canon(sarr)
        assert res[-1].numpy()[0].tobytes() == rviews.tobytes()
        assert [b.tobytes() for b in res[-1].buffers()] == [b.tobytes() for b in rbufs]
    plan.close()


def test_varbin_bad_offsets_is_an_error(ctx):
    """VarBin offsets that run backwards or past the bytes are rejected (zero view + error),
    on the direct path and through a plan's batched dictionary views."""
    import torch
    heap = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", np.uint8).copy()
    offs = np.array([0, 5, 3, 20, 36, 40], np.int32)  # 5 -> 3 backwards; 36 -> 40 past the end
    vb = A.varbin(A.primitive(offs), A.primitive(heap))
    with pytest.raises(V.VortexGpuError, match="VarBin offsets"):
        gpu(vb, ctx)
    codes = np.array([0, 1, 2, 3, 4] * 100, np.uint8)
    d = A.dict_array(vb, E.encode_bitpacked(codes, bit_width=3, allow_patches=False))
    arr = A.chunked([d, d])
    plan = V.Plan([arr.to(torch.device("cuda", 0))], ctx)
    with pytest.raises(V.VortexGpuError, match="VarBin offsets"):
        plan.launch(sync=True)
    plan.close()


# ------------------------------------------------------------------ edge cases: empty inputs
def test_empty_arrays_every_encoding(ctx):
    """len = 0 through every encoding and container (the reference canonicalizes empty arrays
    to empty canonical arrays): no launch may touch memory, outputs are empty."""
    empty_u32 = np.zeros(0, np.uint32)
    cases = [
        E.encode_bitpacked(empty_u32, bit_width=5, allow_patches=False),
        E.encode_for_bitpacked(np.zeros(0, np.int64)),
        E.encode_zigzag(np.zeros(0, np.int32)),
        E.encode_alp(np.zeros(0, np.float64), cascade=False),
        A.dict_array(A.primitive(np.array([7, 9], np.uint16)), A.primitive(np.zeros(0, np.uint32))),
        A.constant(5, 0, "i64"),
        A.chunked([E.encode_bitpacked(np.arange(3000, dtype=np.uint32) % 64, bit_width=6),
                   A.primitive(np.zeros(0, np.uint32)),
                   E.encode_bitpacked(np.arange(100, dtype=np.uint32) % 64, bit_width=6)]),
    ]
    for arr in cases:
        assert_primitive_parity(arr, ctx)
    heap, offs, _ = E.strings_to_heap([])
    assert_string_parity(A.varbin(A.primitive(offs.astype(np.int32)), A.primitive(heap)), ctx, [])
    assert_string_parity(A.chunked([E.encode_fsst([b"only one string here!"]), E.encode_varbinview([])]), ctx,
                         [b"only one string here!"])


def test_ragged_single_element_chunks(ctx):
    """Chunks of 1, 2, 1023, 1025 values (ragged FastLanes tails) in one grouped launch."""
    rng = np.random.default_rng(77)
    chunks, expect = [], []
    for n in [1, 2, 1023, 1024, 1025, 1, 7, 4097]:
        v = rng.integers(0, 1 << 9, n, dtype=np.uint64).astype(np.uint16)
        chunks.append(E.encode_bitpacked(v, bit_width=9, allow_patches=False))
        expect.append(v)
    assert_primitive_parity(A.chunked(chunks), ctx, np.concatenate(expect))


# ------------------------------------------------------------------ Bool canonical + compressed validity
def _bool_case(ctx, arr):
    got = A.canonicalize(arr.to(torch_dev()), ctx)
    want, wvalid = canon(arr)
    assert got.kind == "bool"
    assert np.array_equal(got.numpy(), want)
    gv = got.validity_mask()
    if wvalid is None:
        assert gv is None or gv.all()
    else:
        assert np.array_equal(gv, wvalid)


def torch_dev():
    import torch
    return torch.device("cuda", 0)


@pytest.mark.parametrize("n", [1, 31, 32, 33, 8191, 8192, 8193, 100_003, 1 << 20])
@pytest.mark.parametrize("kind", ["random", "long", "alternating"])
def test_runend_bool(ctx, n, kind):
    """RunEndBool -> BoolArray (runend-bool/src/compress.rs:46-93): flips at run ends inside
    8192-bit workgroup spans; runs shorter than, equal to and much longer than a span."""
    rng = np.random.default_rng(n)
    if kind == "random":
        m = rng.integers(0, 2, n).astype(bool)
    elif kind == "long":
        m = np.repeat(rng.integers(0, 2, n // 5000 + 2).astype(bool), 5000)[:n]
    else:
        m = (np.arange(n) % 2).astype(bool)
    for bp in (False, True):
        _bool_case(ctx, E.encode_runend_bool(m, bitpack_ends=bp))


def test_runend_bool_sliced_and_zero_length_runs(ctx):
    # the reference's slice KAT (compute.rs:72-84): ends [5,6,7,10] start false offset 2 len 6
    _bool_case(ctx, A.run_end_bool(A.primitive(np.array([5, 6, 7, 10], np.uint32)), False, length=6, offset=2))
    # slices of a long random array at many offsets, u16/u32/u64 ends
    rng = np.random.default_rng(9)
    m = rng.integers(0, 2, 50_000).astype(bool)
    ends, start = E.runend_bool_encode(m)
    for lo, hi in [(0, 50_000), (3, 49_000), (8191, 8193 * 3), (20_000, 20_001)]:
        b = int(np.searchsorted(ends, lo, side="right"))
        e = int(np.searchsorted(ends, hi, side="right"))
        st = start if b % 2 == 0 else (not start)
        for pt in (np.uint32, np.uint64):
            arr = A.run_end_bool(A.primitive(ends[b:e + 1].astype(pt)), st, length=hi - lo, offset=lo)
            _bool_case(ctx, arr)
    # zero-length runs (repeated ends) flip twice
    _bool_case(ctx, A.run_end_bool(A.primitive(np.array([0, 3, 3, 7, 7, 7, 40], np.uint64)), True, length=40))


def test_bool_encodings(ctx):
    rng = np.random.default_rng(3)
    m = rng.integers(0, 2, 70_001).astype(bool)
    _bool_case(ctx, A.bool_array(m))
    _bool_case(ctx, A.bool_array(m, bit_offset=3))
    _bool_case(ctx, A.byte_bool(m.astype(np.uint8) * rng.integers(1, 255, m.size).astype(np.uint8)))
    _bool_case(ctx, A.constant_bool(True, 1000))
    _bool_case(ctx, A.constant_bool(False, 1000))
    for fill in (None, True, False):
        idx = np.sort(rng.choice(m.size, 500, replace=False)).astype(np.uint64) + 7
        _bool_case(ctx, A.sparse_bool(A.primitive(idx), A.bool_array(rng.integers(0, 2, 500).astype(bool)),
                                      m.size, indices_offset=7, fill=fill))


def test_chunked_bools_ragged(ctx):
    """pack_bools (chunked/canonical.rs:154-163) at bit offsets that are not word aligned."""
    rng = np.random.default_rng(4)
    chunks = []
    for i, n in enumerate([5, 33, 1, 8192, 9000, 31, 100_000, 64, 3]):
        m = rng.integers(0, 2, n).astype(bool)
        k = i % 4
        chunks.append([A.bool_array(m, bit_offset=i % 8), A.byte_bool(m), E.encode_runend_bool(m),
                       A.constant_bool(bool(i % 2), n)][k])
    _bool_case(ctx, A.chunked(chunks))


def test_compressed_validity_children(ctx):
    """A validity child may be any Bool array (validity.rs:25-110): RunEndBool, ByteBool,
    Constant, Chunked; values and nulls both match the oracle."""
    rng = np.random.default_rng(6)
    n = 30_000
    vals = rng.integers(0, 1 << 12, n).astype(np.uint32)
    m = np.repeat(rng.integers(0, 2, n // 100 + 1).astype(bool), 100)[:n]
    for v in (E.encode_runend_bool(m), A.byte_bool(m), A.chunked([E.encode_runend_bool(m[:777]), A.byte_bool(m[777:])])):
        for arr in (A.primitive(vals, validity=v), E.encode_bitpacked(vals, bit_width=12, allow_patches=False, validity=v)):
            got = A.canonicalize(arr.to(torch_dev()), ctx)
            want, wvalid = canon(arr)
            assert got.numpy()[:n].tobytes() == want.tobytes()
            assert np.array_equal(got.validity_mask(), wvalid)
    # strings with a RunEndBool validity
    strs = [b"s%d" % i * (i % 7) for i in range(n)]
    heap, offs, _ = E.strings_to_heap(strs)
    sv = A.varbin(A.primitive(offs.astype(np.int32)), A.primitive(heap), validity=E.encode_runend_bool(m))
    got = A.canonicalize(sv.to(torch_dev()), ctx)
    (rv, rh), rvalid = canon(sv)
    assert got.numpy()[0].tobytes() == rv.tobytes() and np.array_equal(got.validity_mask(), rvalid)


def test_plan_with_bool_columns(ctx):
    rng = np.random.default_rng(8)
    m = rng.integers(0, 2, 200_000).astype(bool)
    arrs = [E.encode_runend_bool(m), A.byte_bool(m), A.primitive(np.arange(m.size, dtype=np.uint32),
                                                                  validity=E.encode_runend_bool(~m))]
    plan = V.Plan([a.to(torch_dev()) for a in arrs], ctx)
    for _ in range(2):
        res = plan.launch(sync=True)
        assert np.array_equal(res[0].numpy(), m) and np.array_equal(res[1].numpy(), m)
        assert np.array_equal(res[2].validity_mask(), ~m)
    plan.close()


@pytest.mark.parametrize("mode", ["0", "1", "mixed", None])
def test_plan_modes_non_c5_mix(ctx, mode):
    """A plan over a table that is not C5's shape -- a C3-like shard (Chunked[Dict(codes=BitPacked
    u64 W=10, u64 values)], 6 chunks), a C4-like FSST column, bool columns (RunEndBool, ByteBool,
    a primitive with a RunEndBool validity) and one large chunked u32 column -- recorded unbatched,
    batched, mixed (arrays <= VXG_PLAN_BATCH_MAX_BYTES batched) and by default (both recorded, the
    faster kept unless within 3 %, then the smaller graph, measure=True): every replay
    byte-identical to the oracle in every mode."""
    import torch
    sys_path_bench()
    import bench
    rng = np.random.default_rng(303)
    dvals = rng.integers(0, 1 << 62, 1024, dtype=np.uint64)
    c3, c3_plain = [], []
    for k in range(6):
        codes = rng.integers(0, 1024, 64 * 1024 + 37 * k, dtype=np.uint64)
        c3.append(A.dict_array(A.primitive(dvals), E.encode_bitpacked(codes, bit_width=10, allow_patches=False)))
        c3_plain.append(dvals[codes])
    c3_arr = A.chunked(c3)
    heap, offs = bench.c4_heap(rng, 60_000)
    c4_arr = E.encode_fsst_from_heap(heap, offs)
    m = rng.integers(0, 2, 150_000).astype(bool)
    big = rng.integers(0, 1 << 13, 3 * (1 << 20), dtype=np.uint64).astype(np.uint32)  # 12 MB out
    big_arr = A.chunked([E.encode_bitpacked(big[i:i + (1 << 20)], bit_width=13, allow_patches=False)
                         for i in range(0, big.size, 1 << 20)])
    arrs = [c3_arr, c4_arr, E.encode_runend_bool(m), A.byte_bool(m),
            A.primitive(np.arange(m.size, dtype=np.uint32), validity=E.encode_runend_bool(~m)), big_arr]
    env = {} if mode is None else {"VXG_PLAN_BATCH_MAX_BYTES": str(4 << 20)}  # mixed: big_arr unbatched
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        with plan_mode(mode):
            plan = V.Plan([a.to(torch_dev()) for a in arrs], ctx, measure=mode is None)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    (rviews, rheap), _ = canon(c4_arr)  # one data buffer (not chunked)
    for _ in range(2):
        res = plan.launch(sync=True)
        assert res[0].numpy().tobytes() == np.concatenate(c3_plain).tobytes()
        assert res[1].numpy()[0].tobytes() == rviews.tobytes()
        assert [b.tobytes() for b in res[1].buffers()] == [rheap.tobytes()]
        assert np.array_equal(res[2].numpy(), m) and np.array_equal(res[3].numpy(), m)
        assert np.array_equal(res[4].validity_mask(), ~m)
        assert res[5].numpy().tobytes() == big.tobytes()
    plan.close()


def _validity_nodes(host, dev):
    """(host Bool node, device Bool node) of every ARRAY validity child in two parallel trees."""
    out = []
    if host.validity == A.VALIDITY["ARRAY"] and host.children and host.children[-1].encoding == A.ENC["BOOL"]:
        out.append((host.children[-1], dev.children[-1]))
    for h, d in zip(host.children, dev.children):
        out += _validity_nodes(h, d)
    return out


def test_plan_mixed_nullable_chunked_fsst_validity_changes(ctx):
    """in a mixed plan the batch runs on its own graph branch, and a chunked FSST
    column's deferred decode reads the per-chunk validity bitmaps its array branch wrote; the
    batch branch now joins every array branch first.  A nullable chunked FSST column (batched)
    beside a large unbatched column, replayed, then its validity changed IN PLACE between replays:
    every replay equals the oracle of the current validity."""
    import copy
    import os
    import torch
    rng = np.random.default_rng(606)
    strs = _comment_strings(rng, 50_000, vocab=60)
    strs = [None if i % 17 == 3 else x for i, x in enumerate(strs)]
    cuts = [0, 5, 7_000, 7_301, 30_000, 50_000]
    fsst = A.chunked([E.encode_fsst(strs[a:b]) for a, b in zip(cuts, cuts[1:])])
    big = rng.integers(0, 1 << 13, 3 * (1 << 20), dtype=np.uint64).astype(np.uint32)
    big_arr = A.chunked([E.encode_bitpacked(big[i:i + (1 << 20)], bit_width=13, allow_patches=False)
                         for i in range(0, big.size, 1 << 20)])
    dev = fsst.to(torch_dev())
    pairs = _validity_nodes(fsst, dev)
    assert len(pairs) == len(cuts) - 1
    old = os.environ.get("VXG_PLAN_BATCH_MAX_BYTES")
    os.environ["VXG_PLAN_BATCH_MAX_BYTES"] = str(4 << 20)  # the FSST column batched, big_arr not
    try:
        with plan_mode("mixed"):
            plan = V.Plan([dev, big_arr.to(torch_dev())], ctx)
    finally:
        if old is None:
            os.environ.pop("VXG_PLAN_BATCH_MAX_BYTES", None)
        else:
            os.environ["VXG_PLAN_BATCH_MAX_BYTES"] = old
    info = plan.info()
    assert info["batched"] and info["branches"] == 2

    def check(host):
        (rviews, rbufs), rvalid = canon(host)
        for _ in range(2):
            res = plan.launch(sync=True)
            assert res[0].numpy()[0].tobytes() == rviews.tobytes()
            assert [b.tobytes() for b in res[0].buffers()] == [b.tobytes() for b in rbufs]
            assert np.array_equal(res[0].validity_mask(), rvalid)
            assert res[1].numpy().tobytes() == big.tobytes()

    check(fsst)
    for rnd in range(2):  # more rows become null, in place on the device
        host = copy.deepcopy(fsst)
        for (h, d), (h2, _) in zip(pairs, _validity_nodes(host, host)):
            m = np.unpackbits(np.asarray(h.buffers[0]), bitorder="little")[: h.len].astype(bool)
            m &= rng.random(m.size) > 0.3
            bits = np.packbits(m, bitorder="little")
            h2.buffers[0] = bits
            d.buffers[0][: bits.size].copy_(torch.from_numpy(bits).to(torch_dev()))
        torch.cuda.synchronize()
        check(host)
        fsst = host
        pairs = [(h2, d) for (h2, _), (_, d) in zip(_validity_nodes(host, host), pairs)]
    plan.close()


def test_dict_nullable_values(ctx):
    """Dict over nullable values: canonical = take(values, codes) with the values' validity
    taken by the codes (dict/array.rs:68-73, primitive/compute/take.rs:58-67)."""
    rng = np.random.default_rng(12)
    n, d = 50_000, 300
    dv = rng.integers(0, 1 << 30, d).astype(np.uint32)
    dmask = rng.random(d) > 0.2
    codes = rng.integers(0, d, n).astype(np.uint64)
    for values in (A.primitive(dv, validity=dmask), A.primitive(dv, validity=E.encode_runend_bool(dmask))):
        for c in (A.primitive(codes), E.encode_bitpacked(codes, allow_patches=False)):
            arr = A.dict_array(values, c)
            got = A.canonicalize(arr.to(torch_dev()), ctx)
            want, wvalid = canon(arr)
            assert got.numpy().tobytes() == want.tobytes()
            assert np.array_equal(got.validity_mask(), wvalid)
    # strings: Dict(VarBin with nulls)
    strs = [None if i % 5 == 0 else b"value-%d" % i * (1 + i % 3) for i in range(d)]
    heap, offs, valid = E.strings_to_heap(strs)
    sv = A.varbin(A.primitive(offs.astype(np.int32)), A.primitive(heap), validity=valid)
    arr = A.dict_array(sv, E.encode_bitpacked(codes, allow_patches=False))
    got = A.canonicalize(arr.to(torch_dev()), ctx)
    (rv, rh), rvalid = canon(arr)
    assert got.numpy()[0].tobytes() == rv.tobytes()
    assert np.array_equal(got.validity_mask(), rvalid)
    # chunked dicts with nullable values
    ch = A.chunked([A.dict_array(A.primitive(dv, validity=dmask), A.primitive(codes[:1234])),
                    A.dict_array(A.primitive(dv), A.primitive(codes[1234:]))])
    got = A.canonicalize(ch.to(torch_dev()), ctx)
    want, wvalid = canon(ch)
    assert got.numpy().tobytes() == want.tobytes() and np.array_equal(got.validity_mask(), wvalid)


# ------------------------------------------------------------------ compute::take on compressed arrays
def _take_case(ctx, arr, idx):
    got = A.take(arr.to(torch_dev()), idx, ctx)
    vals, valid = canon(arr)
    ii = np.asarray(idx).astype(np.int64)
    want = np.ascontiguousarray(vals[ii])
    assert got.numpy().tobytes() == want.tobytes()
    if valid is None:
        assert got.validity is None or got.validity_mask().all()
    else:
        assert np.array_equal(got.validity_mask(), valid[ii])


@pytest.mark.parametrize("T,W", [(8, 3), (16, 11), (32, 7), (32, 31), (64, 1), (64, 24), (64, 63)])
def test_take_bitpacked(ctx, T, W):
    """bitpacking/compute/take.rs:21-125: unpack_single of the taken positions only (few
    indices) and the canonicalize-then-take path (many indices, take.rs:23-31)."""
    rng = np.random.default_rng(T * 100 + W)
    n = 70_001
    dt = {8: np.uint8, 16: np.uint16, 32: np.uint32, 64: np.uint64}[T]
    vals = (rng.integers(0, 1 << 62, n, dtype=np.uint64) & np.uint64((1 << W) - 1 if W < 64 else (1 << 64) - 1)).astype(dt)
    arr = E.encode_bitpacked(vals, bit_width=W, allow_patches=False)
    for k in (0, 1, 17, 5000, 40_000):
        _take_case(ctx, arr, rng.integers(0, n, k).astype(np.uint32))
    _take_case(ctx, arr, np.array([0, n - 1, 1023, 1024, 1025], np.int64))


def test_take_cascades(ctx):
    rng = np.random.default_rng(77)
    n = 100_000
    idx = rng.integers(0, n, 3000).astype(np.uint64)
    # patches (inner): a few wide outliers
    v = rng.integers(0, 1 << 9, n).astype(np.uint32)
    v[rng.choice(n, 300, replace=False)] = rng.integers(1 << 20, 1 << 31, 300).astype(np.uint32)
    bp = E.encode_bitpacked(v, allow_patches=True)
    assert bp.meta["has_patches"]
    _take_case(ctx, bp, idx)
    _take_case(ctx, bp, np.sort(rng.choice(n, 500, replace=False)).astype(np.int32))
    # sliced offset
    _take_case(ctx, E.encode_bitpacked(v[:5000] & 511, bit_width=9, allow_patches=False, offset=300),
               rng.integers(0, 5000 - 300, 200).astype(np.uint16))
    # FoR / ZigZag / ALP (+ patches) / Dict
    s = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    _take_case(ctx, E.encode_for_bitpacked(s), idx)
    _take_case(ctx, E.encode_zigzag(rng.integers(-5000, 5000, n).astype(np.int32)), idx)
    prices = np.round(rng.uniform(1, 100_000, n) * 100) / 100
    prices[rng.choice(n, 100, replace=False)] = rng.uniform(0, 1, 100) * np.pi
    _take_case(ctx, E.encode_alp(prices), idx)
    _take_case(ctx, E.encode_alp(np.round(rng.uniform(0, 100, n), 1).astype(np.float32)), idx)
    dv = rng.integers(0, 1 << 40, 300).astype(np.uint64)
    _take_case(ctx, A.dict_array(A.primitive(dv), E.encode_bitpacked(rng.integers(0, 300, n).astype(np.uint64),
                                                                     allow_patches=False)), idx)
    # anything else: canonicalize + gather (chunked, runend)
    _take_case(ctx, A.chunked([E.encode_bitpacked(v[:40_000] & 511, bit_width=9, allow_patches=False),
                               A.primitive(v[40_000:])]), idx)
    _take_case(ctx, E.encode_runend(np.repeat(np.arange(1000, dtype=np.int32), 100)), idx)


def test_take_validity_and_errors(ctx):
    rng = np.random.default_rng(78)
    n = 50_000
    v = rng.integers(0, 1 << 12, n).astype(np.uint32)
    m = rng.random(n) > 0.3
    idx = rng.integers(0, n, 2000).astype(np.int64)
    _take_case(ctx, E.encode_bitpacked(v, bit_width=12, allow_patches=False, validity=m), idx)
    _take_case(ctx, A.primitive(v, validity=E.encode_runend_bool(m)), idx)
    _take_case(ctx, E.encode_bitpacked(v, bit_width=12, allow_patches=False), np.zeros(0, np.uint32))
    # out-of-bounds index -> OutOfBounds at the next sync (compute/take.rs bounds)
    with pytest.raises(V.VortexGpuError) as ei:
        A.take(E.encode_bitpacked(v, bit_width=12, allow_patches=False).to(torch_dev()),
               np.array([1, n], np.uint32), ctx)
    assert ei.value.kind == "OutOfBounds"


@pytest.mark.parametrize("dt", [np.int8, np.int16, np.int32, np.int64])
def test_take_negative_index_is_out_of_bounds(ctx, dt):
    """A negative signed index is a huge usize in the reference (`as usize`): OutOfBounds on
    every path - unpack_single (few indices), canonicalize-then-take (many indices or other
    encodings), the Dict codes take, and the validity gather."""
    rng = np.random.default_rng(5)
    n = 1000  # longer than 255 so a zero-extended i8 -1 would be a valid row
    v = rng.integers(0, 1 << 12, n).astype(np.uint32)
    m = rng.random(n) > 0.3
    trees = [E.encode_bitpacked(v, bit_width=12, allow_patches=False),                  # packed path
             A.primitive(v),                                                             # fallback
             E.encode_dict(rng.integers(0, 5, n).astype(np.uint32) * 7),                 # Dict codes
             A.primitive(v, validity=m)]                                                 # validity gather
    for t in trees:
        for idx in (np.array([-1], dt), np.array([3, -1, 5] + [1] * 200, dt)):
            with pytest.raises(V.VortexGpuError) as ei:
                A.take(t.to(torch_dev()), idx, ctx)
            assert ei.value.kind == "OutOfBounds", (t.encoding, idx[:3])


def test_take_index_dtypes(ctx):
    import torch
    v = np.arange(100, dtype=np.uint32)
    t = A.primitive(v).to(torch_dev())
    for tdt in ("uint16", "uint32", "uint64"):
        if hasattr(torch, tdt):
            idx = torch.tensor([3, 7], dtype=torch.int64).to(getattr(torch, tdt))
            assert A.take(t, idx, ctx).numpy().tolist() == [3, 7]
    with pytest.raises(V.VortexGpuError):
        A.take(t, np.array([1.0]), ctx)


# ------------------------------------------------------------------ compute::filter (stream compaction)
def _filter_case(ctx, arr, pred):
    from oracle_tree import filter_canon
    got = A.filter(arr.to(torch_dev()), pred.to(torch_dev()), ctx)
    want, wvalid = filter_canon(arr, pred)
    if arr.dtype == A.DTYPE["PRIMITIVE"]:
        assert got.len == len(want) and got.numpy().tobytes() == want.tobytes()
    elif arr.dtype == A.DTYPE["BOOL"]:
        assert got.len == len(want) and np.array_equal(got.numpy(), want)
        nb = (got.len + 7) // 8
        assert got.values.cpu().numpy()[:nb].tobytes() == np.packbits(want, bitorder="little").tobytes()
    else:
        wv, wh = want
        gv, gh = got.numpy()
        assert got.len == len(wv) and gv.tobytes() == wv.tobytes()  # same views byte for byte
        assert gh.tobytes() == wh.tobytes() and got.data_buffers == [(0, len(wh))]
    if wvalid is None:
        assert got.validity is None
    else:
        assert np.array_equal(got.validity_mask(), wvalid)
    return got


def _preds(rng, n):
    yield A.bool_array(rng.random(n) < 0.5)
    yield A.bool_array(rng.random(n) < 0.01)
    yield A.bool_array(np.ones(n, bool))
    yield A.bool_array(np.zeros(n, bool))
    m = np.zeros(n, bool)
    m[:: 4097] = True
    yield E.encode_runend_bool(m | (np.arange(n) % 9000 < 3000))
    yield A.constant_bool(True, n)


@pytest.mark.parametrize("n", [0, 1, 63, 64, 4095, 4097, 70_001])
def test_filter_primitive_sizes(ctx, n):
    """primitive/compute/filter.rs:15-50: selected rows in order, at tile edges (64, 4096)."""
    rng = np.random.default_rng(n + 5)
    v = rng.integers(0, 1 << 30, n).astype(np.uint32)
    for pred in _preds(rng, n):
        _filter_case(ctx, A.primitive(v), pred)


def test_filter_compressed_cascades(ctx):
    """filter.rs:41-49 fallback (canonicalize, then filter) on every primitive encoding."""
    rng = np.random.default_rng(91)
    n = 100_000
    pred = A.bool_array(rng.random(n) < 0.3)
    v = rng.integers(0, 1 << 9, n).astype(np.uint32)
    v[rng.choice(n, 300, replace=False)] = rng.integers(1 << 20, 1 << 31, 300).astype(np.uint32)
    _filter_case(ctx, E.encode_bitpacked(v, allow_patches=True), pred)
    _filter_case(ctx, E.encode_for_bitpacked(rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)), pred)
    _filter_case(ctx, E.encode_zigzag(rng.integers(-5000, 5000, n).astype(np.int16)), pred)
    prices = np.round(rng.uniform(1, 100_000, n) * 100) / 100
    _filter_case(ctx, E.encode_alp(prices), pred)
    _filter_case(ctx, E.encode_dict(rng.integers(0, 50, n).astype(np.uint8) * 3), pred)
    _filter_case(ctx, E.encode_runend(np.repeat(np.arange(1000, dtype=np.int64), 100)), pred)
    _filter_case(ctx, E.encode_delta(np.cumsum(rng.integers(0, 5, n)).astype(np.uint64)), pred)
    _filter_case(ctx, A.chunked([E.encode_bitpacked(v[:40_000] & 511, bit_width=9, allow_patches=False),
                                 A.primitive(v[40_000:])]), pred)
    # 16-byte-free widths: u8 / u16 / f32
    _filter_case(ctx, A.primitive(rng.integers(0, 255, n).astype(np.uint8)), pred)
    _filter_case(ctx, A.primitive(rng.standard_normal(n).astype(np.float32)), pred)


def test_filter_validity_and_bools(ctx):
    """validity.filter(predicate) and BoolArray filter (bool/compute/filter.rs:15-60)."""
    rng = np.random.default_rng(92)
    n = 77_777
    m = rng.random(n) > 0.3
    v = rng.integers(0, 1 << 12, n).astype(np.uint32)
    for pred in _preds(rng, n):
        _filter_case(ctx, E.encode_bitpacked(v, bit_width=12, allow_patches=False, validity=m), pred)
        _filter_case(ctx, A.bool_array(rng.random(n) < 0.5, validity=E.encode_runend_bool(m)), pred)
    _filter_case(ctx, E.encode_runend_bool(rng.random(n) < 0.001), A.bool_array(rng.random(n) < 0.7))


def test_filter_strings(ctx):
    """VarBin / FSST filter (varbin/compute/filter.rs:19-200, fsst/compute.rs:147-160): the
    canonical of the result is one heap of the selected strings, null rows empty."""
    rng = np.random.default_rng(93)
    n = 20_000
    strs = [None if i % 7 == 3 else (b"comment %d " % i) * (1 + i % 4) for i in range(n)]
    strs[5] = b""
    strs[6] = b"x" * 12
    strs[8] = b"y" * 13
    heap, offs, valid = E.strings_to_heap(strs)
    pred = A.bool_array(rng.random(n) < 0.4)
    _filter_case(ctx, A.varbin(A.primitive(offs.astype(np.int32)), A.primitive(heap), validity=valid), pred)
    _filter_case(ctx, E.encode_fsst(strs), pred)
    _filter_case(ctx, E.encode_fsst([s or b"" for s in strs]), A.bool_array(np.ones(n, bool)))
    _filter_case(ctx, E.encode_dict_strings([b"alpha", b"a-much-longer-value", b"z"] * 1000),
                 A.bool_array(rng.random(3000) < 0.5))
    _filter_case(ctx, A.chunked([E.encode_fsst(strs[:9000]), E.encode_fsst(strs[9000:])]), pred)
    _filter_case(ctx, E.encode_varbinview(strs), pred)


def test_filter_errors(ctx):
    arr = A.primitive(np.arange(100, dtype=np.uint32)).to(torch_dev())
    with pytest.raises(V.VortexGpuError) as ei:
        A.filter(arr, A.bool_array(np.ones(99, bool)).to(torch_dev()), ctx)
    assert ei.value.kind == "InvalidArgument"
    with pytest.raises(V.VortexGpuError) as ei:
        A.filter(arr, A.bool_array(np.ones(100, bool), validity=np.ones(100, bool)).to(torch_dev()), ctx)
    assert ei.value.kind == "InvalidArgument"
    with pytest.raises(V.VortexGpuError):
        A.filter(arr, A.primitive(np.ones(100, np.uint8)).to(torch_dev()), ctx)
