"""GPU: BASELINE C5 "via vortex-serde" at reduced size — a lineitem Vortex file's bytes are parsed
by the engine's reader (vxg_file_*), each column's message range is copied to HBM once, and the
reader's trees are canonicalized by the HIP engine; every output byte must equal the oracle's
canonicalize of the arrays that were written (tests/oracle_tree.py), and the plain values."""
import ctypes as C

import numpy as np
import pytest

import vortex_amd as V
import vortex_amd._lib as L
import vortex_amd.arrays as A
from oracle_tree import canon
from tools import lineitem as LI
from tools import vxfile as X
from vortex_amd.file import DeviceColumns, VortexFile, scan

pytestmark = pytest.mark.gpu


def _file(rows, chunk_rows):
    import torch
    cols, plain = LI.lineitem_columns(range(LI.n_chunks(rows, chunk_rows)), rows=rows, chunk_rows=chunk_rows)
    written = []
    for name, _ in LI.COLUMNS:
        chunks = cols[name].children[1:]
        if name in ("l_shipdate", "l_commitdate", "l_receiptdate"):
            chunks = [X.date_column(c) for c in chunks]
        written.append((name, chunks))
    data = X.write_file(written)
    host = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).pin_memory()
    return VortexFile(host), written, plain


def _storage(chunks):
    return [c.children[0] if c.encoding == X.ENC_EXTENSION else c for c in chunks]


def _compare(res, chunks, plain_vals):
    arr = A.chunked(_storage(chunks))
    ref, rvalid = canon(arr)
    if res.kind == "primitive":
        got = res.numpy()
        assert got.tobytes() == ref.tobytes()
        assert got.tobytes() == np.concatenate(plain_vals).astype(got.dtype).tobytes()
    else:
        views, _ = res.numpy()
        rviews, rheap = ref
        assert views.tobytes() == rviews.tobytes()
        bufs = res.buffers()
        assert len(bufs) == len(rheap)
        for g, r in zip(bufs, rheap):
            assert g.tobytes() == r.tobytes()
    assert res.validity_mask() is None and rvalid is None


def test_lineitem_file_scan_matches_oracle(ctx):
    f, written, plain = _file(rows=20_000, chunk_rows=4096)
    assert f.row_count == 20_000
    res = scan(f, ctx)
    assert len(res) == 16
    for (name, chunks), r in zip(written, res):
        assert r.len == 20_000, name
        _compare(r, chunks, plain[name])
    f.close()


def test_lineitem_file_chunk_range_and_plan(ctx):
    """A rank's chunk range (what bench C5 decodes at N > 1) through a vxg_plan, replayed after
    the device region was refreshed from the file bytes."""
    f, written, plain = _file(rows=30_000, chunk_rows=4096)
    dc = DeviceColumns(f, ctx, None, 2, 6)
    plan = A.Plan(dc.nodes, ctx)
    for rep in range(2):
        dc.refresh()
        res = plan.launch(sync=True)
        for (name, chunks), r in zip(written, res):
            _compare(r, chunks[2:6], plain[name][2:6])
    plan.close()
    f.close()


def test_file_reader_rejects_uncovered_region(ctx):
    f, _, _ = _file(rows=5000, chunk_rows=2048)
    import torch
    region = torch.empty(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(L.VortexGpuError) as ei:
        f.column_tree(0, 0, 2, region.data_ptr(), 0, 64)
    assert ei.value.kind == "InvalidArgument"
    f.close()


def test_c5_full_size_plan(ctx, lineitem_file_bytes):
    """BASELINE C5 at full size through the exact path the bench times: all
    92 chunks x 16 columns read from the file's bytes, one H2D per column region
    (DeviceColumns), one measuring vxg_plan (its kept graph) replayed twice; plus the same
    columns recorded unbatched (device-table K1 launches of >= 128 workgroups take K1w) and
    batched (K1g).  Every numeric column's bytes and every string row equal the generator's
    plain values (bench.c5_verify); three chunks also equal the oracle's canonicalize of the
    written arrays; the forced modes' outputs equal the verified ones byte for byte."""
    import time
    import torch
    import bench
    from test_gpu_parity import plan_mode
    t0 = time.perf_counter()
    f = VortexFile(torch.from_numpy(lineitem_file_bytes).pin_memory())
    n = LI.n_chunks()
    dc = DeviceColumns(f, ctx, None, 0, n)
    plan = A.Plan(dc.nodes, ctx, measure=True)
    plan.launch()
    res = plan.launch(sync=True)
    assert bench.c5_verify(res, range(n)) == f.row_count
    def content(r):  # the canonical's bytes: values, or views + each data buffer's used bytes
        if r.kind == "primitive":
            return [bytes(r.values.cpu().numpy())]
        return [bytes(r.views.cpu().numpy())] + [b.tobytes() for b in r.buffers()]

    ref = [content(r) for r in res]
    # oracle on a sample of chunks: each column's chunk arrays as written, canonicalized on the CPU
    from oracle_tree import view_bytes
    sample = (0, 45, n - 1)
    cols, _ = LI.lineitem_columns(sample)
    for (name, kind), r in zip(LI.COLUMNS, res):
        for j, c in enumerate(sample):
            chunk = cols[name].children[1 + j]
            o, _ = canon(chunk)
            row0 = c * LI.CHUNK_ROWS
            if r.kind == "primitive":
                assert r.numpy()[row0: row0 + chunk.len].tobytes() == o.tobytes(), (name, c)
            else:
                views, bufs = r.numpy()[0], r.buffers()
                rv, rh = o
                for i in range(0, chunk.len, 97):
                    assert view_bytes(views, bufs, row0 + i) == view_bytes(rv, rh, i), (name, c, i)
    plan.close()
    for mode in ("0", "1"):
        with plan_mode(mode):
            p = A.Plan(dc.nodes, ctx)
        out = p.launch(sync=True)
        assert p.info()["batched"] == (mode == "1")
        for (name, _), want, r in zip(LI.COLUMNS, ref, out):
            assert content(r) == want, (mode, name)
        p.close()
    f.close()
    assert time.perf_counter() - t0 < 120
