"""CPU: the Vortex file reader (include/vortex_file.h, vortex_amd/csrc/serde.cpp) against files
written by tools/vxfile.py (the reference LayoutWriter's layout restated).

No device is needed: with region = NULL the reader's buffer pointers are file offsets, so every
reconstructed tree is compared node by node with the tree that was written - encoding ids,
lengths, dtypes and nullability derived the way the reference accessors derive them, the
per-encoding metadata decoded from flexbuffers, and every buffer's bytes - and malformed files
must fail with InvalidSerde, never crash.  Parity of the written BYTES with the Rust writer is
unpinned (no reference-written file exists in the reference tree and it cannot be built here);
the flexbuffer/flatbuffer decoders are checked against hand-built buffers of the published
formats instead.
"""
import ctypes as C
import struct

import numpy as np
import pytest

import vortex_amd._lib as L
import vortex_amd.arrays as A
import vortex_amd.encode as E
from tools import lineitem as LI
from tools import vxfile as X
from vortex_amd.file import VortexFile


def _check_tree(node, a, data: np.ndarray, path="root"):
    if a.encoding == X.ENC_EXTENSION:
        a = a.children[0]
    assert node.encoding == a.encoding, path
    assert node.len == a.len, path
    assert node.dtype == a.dtype, path
    if a.dtype == L.DTYPE["PRIMITIVE"]:
        assert L.PTYPES[node.ptype] == a.ptype, path
    assert bool(node.nullable) == bool(a.nullable), path
    assert node.validity == a.validity, path
    m = L.VxgMeta()
    A._fill_meta(m, a)
    assert bytes(m) == bytes(node.meta), (path, a.encoding, a.meta)
    if a.buffers:
        want = np.ascontiguousarray(a.buffers[0]).view(np.uint8).reshape(-1)
        assert node.n_buffers == 1, path
        off, n = int(node.buffers[0].ptr or 0), int(node.buffers[0].len)
        assert off % 64 == 0, path  # 64-byte aligned in the file (lib.rs:15)
        assert n == want.size, path
        assert data[off: off + n].tobytes() == want.tobytes(), path
    else:
        assert node.n_buffers == 0, path
    assert node.n_children == len(a.children), path
    for i, c in enumerate(a.children):
        _check_tree(node.children[i], c, data, f"{path}/{i}")


def _lineitem(rows=5000, chunk_rows=2048):
    cols, plain = LI.lineitem_columns(range(LI.n_chunks(rows, chunk_rows)), rows=rows, chunk_rows=chunk_rows)
    out = []
    for name, kind in LI.COLUMNS:
        chunks = cols[name].children[1:]
        if name in ("l_shipdate", "l_commitdate", "l_receiptdate"):
            chunks = [X.date_column(c) for c in chunks]
        out.append((name, chunks))
    return out, plain


def test_flex_roundtrip_shapes():
    """flexbuffer decoding of every shape the metadata uses (maps, nested maps, vectors,
    strings, bools, null, ints of every width and sign, floats) via the reader's metadata
    path: a Constant / Sparse / ALPRD / VarBinView metadata written by the builder and read
    back through a one-column file."""
    for v, p in ((0, "u8"), (255, "u8"), (-1, "i64"), (-(2 ** 40), "i64"), (2 ** 63 + 5, "u64"),
                 (1.5, "f64"), (-2.25, "f32"), (7, "i16")):
        a = A.constant(v, 10, p)
        data = X.write_file([("c", [a])])
        f = VortexFile(data)
        node = f.column_tree(0, 0, 1)
        _check_tree(node.children[1], a, np.frombuffer(data, np.uint8))
        f.close()


def test_lineitem_file_roundtrip():
    cols, plain = _lineitem()
    data = X.write_file(cols)
    raw = np.frombuffer(data, np.uint8)
    assert data[-4:] == b"VRTX" and struct.unpack("<H", data[-8:-6])[0] == 1
    f = VortexFile(data)
    assert f.row_count == 5000
    assert [c.name for c in f.columns] == [n for n, _ in LI.COLUMNS]
    for ci, (name, chunks) in enumerate(cols):
        info = f.columns[ci]
        assert info.n_chunks == len(chunks) == 3 and info.rows == 5000
        if name.endswith("date"):
            assert info.is_extension and info.extension_id == "vortex.date" and info.extension_metadata == b"\x04"
            assert info.dtype == L.DTYPE["PRIMITIVE"] and info.ptype == "i32"
        else:
            assert not info.is_extension
        row = 0
        for k, ch in enumerate(chunks):
            c = f.chunk(ci, k)
            assert c.row_offset == row and c.rows == ch.len
            assert c.message_begin % 64 == 0 and c.buffers_begin % 64 == 0 and c.message_end % 64 == 0
            row += ch.len
        # consecutive messages: the column's chunks are one contiguous byte range
        for k in range(1, len(chunks)):
            assert f.chunk(ci, k).message_begin == f.chunk(ci, k - 1).message_end
        assert list(f.chunk_offsets(ci, 0, 3)) == [0, 2048, 4096, 5000]
        node = f.column_tree(ci, 0, 3)
        assert node.encoding == L.ENC["CHUNKED"] and node.len == 5000 and node.meta.chunked.nchunks == 3
        for k, ch in enumerate(chunks):
            _check_tree(node.children[1 + k], ch, raw, f"{name}[{k}]")
        sub = f.column_tree(ci, 1, 3)
        assert sub.len == 5000 - 2048 and sub.n_children == 3
        _check_tree(sub.children[1], chunks[1], raw)
    f.close()


@pytest.mark.parametrize("typed", [True, False])
def test_every_encoding_roundtrip(typed, monkeypatch):
    monkeypatch.setattr(X, "TYPED_VECTORS", typed)
    rng = np.random.default_rng(3)
    n = 3000
    arrays = {
        "delta": E.encode_delta(np.cumsum(rng.integers(0, 9, n)).astype(np.uint32)),
        "zigzag": E.encode_zigzag(rng.integers(-500, 500, n).astype(np.int32)),
        "alprd": E.encode_alprd(rng.standard_normal(n)),
        "alp_patched": E.encode_alp(np.concatenate([np.round(rng.uniform(0, 100, n - 3), 2), [np.pi, np.e, 1e300]])),
        "bitpacked_patched": E.encode_bitpacked(np.where(rng.random(n) < 0.01, 1 << 40, rng.integers(0, 100, n)).astype(np.uint64)),
        "runend": E.encode_runend(np.repeat(rng.integers(0, 50, 300), 10).astype(np.int64), compress_values=True),
        "dict_prim": E.encode_dict(rng.integers(0, 7, n).astype(np.uint16) * 1000),
        "fsst": E.encode_fsst([None if i % 17 == 0 else b"hello world %d" % i for i in range(n)]),
        "varbinview": E.encode_varbinview([None if i % 5 == 0 else b"x" * (i % 30) for i in range(n)]),
        "nullable_prim": A.primitive(rng.integers(0, 9, n).astype(np.int16), validity=rng.random(n) < 0.7),
        "bool": A.bool_array(rng.random(n) < 0.5, validity=rng.random(n) < 0.9, bit_offset=3),
        "runend_bool": E.encode_runend_bool(np.repeat(rng.random(30) < 0.5, 100), bitpack_ends=True),
        "bytebool": A.byte_bool(rng.random(n) < 0.5),
        "roaring_bool": E.encode_roaring_bool(rng.random(n) < 0.3),
        "roaring_validity": A.primitive(rng.integers(0, 9, n).astype(np.int16),
                                        validity=E.encode_roaring_bool(rng.random(n) < 0.9)),
        "sparse": A.sparse(A.primitive(np.array([3, 70, 999], np.uint64)), A.primitive(np.array([1, 2, 3], np.int32)),
                           1000, fill=-7),
        "constant_null": A.constant(None, 500, "f64"),
        "compressed_validity": E.encode_bitpacked(rng.integers(0, 100, n).astype(np.uint32),
                                                  validity=E.encode_runend_bool(np.repeat(rng.random(30) < 0.8, 100))),
    }
    # columns of different lengths cannot share a file: one file per array
    for name, a in arrays.items():
        data = X.write_file([(name, [a])])
        f = VortexFile(data)
        node = f.column_tree(0, 0, 1)
        _check_tree(node.children[1], a, np.frombuffer(data, np.uint8), name)
        f.close()


def _expect_serde_error(data):
    with pytest.raises(L.VortexGpuError) as ei:
        f = VortexFile(data)
        for ci in range(len(f.columns)):
            f.column_tree(ci, 0, f.columns[ci].n_chunks)
    assert ei.value.kind in ("InvalidSerde", "NotImplemented"), ei.value


def test_malformed_files_fail_cleanly():
    cols, _ = _lineitem(rows=3000, chunk_rows=1024)
    data = bytearray(X.write_file(cols))
    _expect_serde_error(bytes(data[:-1]))                      # truncated EOF
    bad_magic = bytearray(data)
    bad_magic[-1] ^= 0xFF
    _expect_serde_error(bytes(bad_magic))
    bad_ver = bytearray(data)
    bad_ver[-8] = 9
    _expect_serde_error(bytes(bad_ver))
    _expect_serde_error(bytes(40))
    # corrupt every byte of the postscript / a region of the footer / a message in turn: never a
    # crash, either a clean error or (when the byte is not load-bearing) a successful parse
    rng = np.random.default_rng(0)
    n = len(data)
    for pos in list(range(n - 40, n - 8)) + list(rng.integers(0, n - 40, 300)):
        d = bytearray(data)
        d[int(pos)] ^= 0x5A
        try:
            f = VortexFile(bytes(d))
            for ci in range(len(f.columns)):
                f.column_tree(ci, 0, f.columns[ci].n_chunks)
            f.close()
        except L.VortexGpuError as e:
            assert e.kind in ("InvalidSerde", "NotImplemented", "OutOfBounds", "InvalidArgument"), e


def test_region_must_cover_the_chunks():
    cols, _ = _lineitem(rows=3000, chunk_rows=1024)
    data = X.write_file(cols)
    f = VortexFile(data)
    b, e = f.byte_range(2, 0, 3)
    node = f.column_tree(2, 0, 3, region=1 << 40, region_offset=b, region_len=e - b)
    # pointers are rebased into the region
    assert node.children[1].children[0].buffers[0].ptr is not None
    with pytest.raises(L.VortexGpuError) as ei:
        f.column_tree(2, 0, 3, region=1 << 40, region_offset=b + 64, region_len=e - b)
    assert ei.value.kind == "InvalidArgument"
    with pytest.raises(L.VortexGpuError):
        f.column_tree(99, 0, 1)
    f.close()


def test_region_must_cover_every_chunk():
    """Chunk messages out of file order (a malformed or foreign writer): a region spanning the
    first chunk's begin and the last chunk's end does not cover a middle chunk written elsewhere,
    and no buffer pointer may leave the region."""
    cols, _ = _lineitem(rows=3000, chunk_rows=1024)
    cols = cols[:2]
    order = [(0, 0), (0, 2), (1, 0), (1, 1), (1, 2), (0, 1)]
    data = X.write_file(cols, message_order=order)
    f = VortexFile(data)
    c0, c1, c2 = (f.chunk(0, k) for k in range(3))
    assert c0.message_begin < c2.message_begin < c1.message_begin
    b, e = c0.message_begin, c2.message_end
    with pytest.raises(L.VortexGpuError) as ei:
        f.column_tree(0, 0, 3, region=1 << 40, region_offset=b, region_len=e - b)
    assert ei.value.kind in ("InvalidArgument", "InvalidSerde")
    # covering all three messages is fine, and the out-of-order file still reads correctly
    node = f.column_tree(0, 0, 3, region=1 << 40, region_offset=b, region_len=c1.message_end - b)
    lo, hi = 1 << 40, (1 << 40) + c1.message_end - b
    for k in range(3):
        for leaf in _leaf_buffers(node.children[1 + k]):
            assert lo <= leaf[0] and leaf[0] + leaf[1] <= hi
    raw = np.frombuffer(data, np.uint8)
    node = f.column_tree(0, 0, 3)
    for k, ch in enumerate(cols[0][1]):
        _check_tree(node.children[1 + k], ch, raw)
    f.close()


def _leaf_buffers(node):
    out = [(int(node.buffers[i].ptr or 0), int(node.buffers[i].len)) for i in range(node.n_buffers)]
    for i in range(node.n_children):
        out += _leaf_buffers(node.children[i])
    return out


def test_flatbuffer_postscript_is_32_bytes():
    # writer.rs:248-262 postscript_size: a Postscript flatbuffer is exactly 32 bytes
    fbb = X.FBB()
    fbb.start(2)
    fbb.field(1, "Q", 1100000)
    fbb.field(0, "Q", 1000000)
    ps = fbb.finish(fbb.end())
    assert len(ps) == 32
