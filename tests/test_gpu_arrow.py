"""GPU: the canonical outputs are valid Arrow arrays.

The reference's boundary ends in Canonical::into_arrow (vortex-array/src/canonical.rs:71-85;
varbinview_as_arrow, varbinview/mod.rs:518): Primitive -> PrimitiveArray, Bool -> BooleanArray,
VarBinView -> StringViewArray / BinaryViewArray over the same buffers.  Here the engine's device
buffers (values / LSB bits / 16-byte views + data buffers, LSB validity) are copied to the host
unchanged and wrapped by pyarrow's from_buffers (Canonical.to_arrow); `validate(full=True)` runs
Arrow's own checks (view lengths, inline zero padding, prefixes equal to the data bytes,
buffer_index / offset inside the buffers, UTF-8) and to_pylist() must equal the plain data.
"""
import numpy as np
import pytest

import vortex_amd.arrays as A
import vortex_amd.encode as E

pytestmark = pytest.mark.gpu
pa = pytest.importorskip("pyarrow")


def _dev():
    import torch
    return torch.device("cuda", 0)


def _arrow(arr, ctx):
    out = A.canonicalize(arr.to(_dev()), ctx).to_arrow()
    out.validate(full=True)
    return out


def test_primitive_with_nulls_is_valid_arrow(ctx):
    rng = np.random.default_rng(21)
    n = 70_001
    for dt in (np.int8, np.uint16, np.int32, np.uint64, np.float32, np.float64):
        vals = (rng.integers(0, 40, n) * 3).astype(dt)
        mask = rng.random(n) < 0.8
        for arr in (A.primitive(vals, validity=mask),
                    E.encode_bitpacked(vals.astype(A.NP_OF_PTYPE["u" + A.PTYPE_OF_NP[np.dtype(dt)][1:]]), validity=mask)
                    if np.dtype(dt).kind in "ui" else E.encode_alp(vals)):
            got = _arrow(arr, ctx)
            want = [v if (m or not arr.nullable) else None for v, m in zip(vals.tolist(), mask)]
            if got.type != pa.from_numpy_dtype(dt):  # bitpacked form of a signed type is its unsigned twin
                got = got.cast(pa.from_numpy_dtype(dt))
            assert got.to_pylist() == want


def test_bool_encodings_are_valid_arrow(ctx):
    rng = np.random.default_rng(22)
    n = 10_007
    bits = rng.random(n) < 0.4
    mask = rng.random(n) < 0.9
    for arr in (A.bool_array(bits, validity=mask, bit_offset=5), E.encode_runend_bool(np.repeat(bits[:100], 100)),
                E.encode_roaring_bool(bits), A.byte_bool(bits)):
        got = _arrow(arr, ctx)
        plain = np.repeat(bits[:100], 100) if arr.len == 10_000 else bits
        valid = mask if arr.nullable else np.ones(arr.len, bool)
        assert got.to_pylist() == [bool(b) if v else None for b, v in zip(plain, valid)]


def _strings(rng, n, nulls=True):
    out = []
    for i in range(n):
        k = int(rng.integers(0, 40))
        if nulls and i % 7 == 3:
            out.append(None)
        elif i % 11 == 0:
            out.append(("x" * 12).encode())          # exactly inline
        elif i % 13 == 0:
            out.append(("y" * 13).encode())          # first non-inline length
        else:
            out.append(("word%d " % i * 9)[:k].encode())
    return out


def test_varbinview_single_and_chunked_are_valid_arrow(ctx):
    rng = np.random.default_rng(23)
    s1 = _strings(rng, 5000)
    s2 = _strings(rng, 3000)
    s3 = _strings(rng, 4000, nulls=False)
    heap, offs, valid = E.strings_to_heap(s1)
    cases = [
        (E.encode_fsst(s1), s1),
        (A.varbin(A.primitive(offs.astype(np.int32)), A.primitive(heap), validity=valid), s1),
        (E.encode_varbinview(s2), s2),
        (E.encode_dict_strings_nullable(s2), s2),
        (A.chunked([E.encode_fsst(s1), E.encode_varbinview(s2), E.encode_fsst(s3)]), s1 + s2 + s3),
        (A.chunked([E.encode_dict_strings([s for s in s3]), E.encode_fsst(s3)]), s3 + s3),
    ]
    for arr, plain in cases:
        got = _arrow(arr, ctx)
        assert got.type == pa.string_view()
        assert got.to_pylist() == [None if s is None else s.decode() for s in plain]
    # the 12 / 13-byte inline boundary (varbin/flatten.rs:28-57): inline vs referenced views
    got = _arrow(E.encode_varbinview([None, None, b"123456789012", b"1234567890123"]), ctx)
    assert got.to_pylist() == [None, None, "123456789012", "1234567890123"]


def test_c4_full_size_is_valid_arrow(ctx):
    """BASELINE C4 at full size (6,001,215 FSST strings) through Canonical.to_arrow."""
    import bench
    rng = np.random.default_rng(42)
    arr, info = bench.make_c4(rng, 1, 0)
    got = _arrow(arr, ctx)
    assert len(got) == info["values"] == 6_001_215 and got.null_count == 0
    heap, offs = bench.c4_heap(np.random.default_rng(42), info["values"])
    for i in (0, 1, 12345, 3_000_000, 6_001_214):
        assert got[i].as_py() == heap[offs[i]: offs[i + 1]].tobytes().decode()


def test_lineitem_string_columns_are_valid_arrow(ctx, lineitem_file_bytes):
    """The lineitem scan's string columns (4 Dict(VarBin) + l_comment FSST, chunked) read from
    file bytes and canonicalized by one plan: every column validates and equals the generator's
    strings."""
    import torch
    import bench
    from tools import lineitem as L
    from vortex_amd.file import DeviceColumns, VortexFile
    f = VortexFile(torch.from_numpy(lineitem_file_bytes).pin_memory())
    chunks = range(0, 4)
    dc = DeviceColumns(f, ctx, None, chunks.start, chunks.stop)
    plan = A.Plan(dc.nodes, ctx)
    res = plan.launch(sync=True)
    plain = [L.chunk_values(c) for c in chunks]
    n_checked = 0
    for (name, kind), r in zip(L.COLUMNS, res):
        got = r.to_arrow()
        got.validate(full=True)
        want = np.concatenate([p[name] for p in plain])
        if kind == "utf8":
            assert got.type == pa.string_view()
            assert got.to_pylist() == [s.decode() if isinstance(s, bytes) else s for s in want.tolist()]
            n_checked += 1
        else:
            assert np.array_equal(got.to_numpy(zero_copy_only=False), want)
    assert n_checked == 5
    plan.close()
    f.close()
