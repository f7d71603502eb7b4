"""Reading Vortex files into the decode engine (host side of include/vortex_file.h).

The reference scans a file with vortex-serde's LayoutReaderBuilder -> LayoutBatchStream
(layouts/read/builder.rs, stream.rs:91-227): the footer is read from the tail (read/footer.rs:
140-187), every column's Chunked layout yields its Flat chunks, each chunk's bytes become an
Array through ArrayBufferReader (message_reader.rs:249-348) + ArrayView (view.rs:45-83), and
the bench collects the batches into a ChunkedArray and canonicalizes it (bench-vortex/benches/
compress_noci.rs:124-145).

Here the file's bytes stay in (pinned) host memory; the native reader (vxg_file_*, serde.cpp)
parses footer, layouts, messages and flexbuffer metadata, and a column's chunk range - its
messages are contiguous in the file - is copied to HBM with ONE H2D copy; the reader then
builds that column's ChunkedArray tree with buffer pointers into the device copy, and the trees
go to vxg_canonicalize / vxg_plan like any other arrays.  No CPU decode anywhere.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import PTYPES

REGION_SLACK = 256  # kernels may read a few bytes past a buffer's end (aligned 16-byte loads)


@dataclass
class ColumnInfo:
    name: str
    dtype: int
    ptype: str
    nullable: bool
    is_extension: bool
    extension_id: Optional[str]
    extension_metadata: bytes
    n_chunks: int
    rows: int


@dataclass
class ChunkInfo:
    row_offset: int
    rows: int
    message_begin: int
    message_end: int
    buffers_begin: int


class VortexFile:
    """A parsed Vortex file over host bytes (numpy uint8 array, bytes, or a CPU torch uint8
    tensor - pinned for fast H2D).  The bytes must stay alive and unchanged while open."""

    def __init__(self, data):
        self.lib = _lib.gpu_lib()
        if isinstance(data, (bytes, bytearray)):
            data = np.frombuffer(bytes(data), dtype=np.uint8).copy()
        self._data = data
        if hasattr(data, "data_ptr"):
            ptr, n = data.data_ptr(), data.numel()
        else:
            arr = np.ascontiguousarray(data, dtype=np.uint8)
            self._data = arr
            ptr, n = arr.ctypes.data, arr.size
        self.nbytes = int(n)
        h = C.c_void_p()
        _lib.check(self.lib.vxg_file_open(C.c_void_p(ptr), n, C.byref(h)))
        self.handle = h
        rc, nc = C.c_uint64(), C.c_uint32()
        _lib.check(self.lib.vxg_file_info(h, C.byref(rc), C.byref(nc)))
        self.row_count = int(rc.value)
        self.columns: list[ColumnInfo] = []
        for i in range(nc.value):
            ci = _lib.VxgFileColumn()
            _lib.check(self.lib.vxg_file_column_info(h, i, C.byref(ci)))
            em = bytes(ci.extension_metadata[: ci.extension_metadata_len]) if ci.extension_metadata_len else b""
            self.columns.append(ColumnInfo(ci.name.decode(), int(ci.dtype), PTYPES[ci.ptype] if ci.ptype < 11 else "u8",
                                           bool(ci.nullable), bool(ci.is_extension),
                                           ci.extension_id.decode() if ci.extension_id else None, em,
                                           int(ci.n_chunks), int(ci.rows)))

    def column_index(self, name: str) -> int:
        for i, c in enumerate(self.columns):
            if c.name == name:
                return i
        raise KeyError(name)

    def chunk(self, col: int, i: int) -> ChunkInfo:
        ch = _lib.VxgFileChunk()
        _lib.check(self.lib.vxg_file_chunk_info(self.handle, col, i, C.byref(ch)))
        return ChunkInfo(int(ch.row_offset), int(ch.rows), int(ch.message_begin), int(ch.message_end),
                         int(ch.buffers_begin))

    def byte_range(self, col: int, c0: int, c1: int) -> tuple[int, int]:
        """File bytes [begin, end) of chunks [c0, c1) of a column (contiguous messages)."""
        return self.chunk(col, c0).message_begin, self.chunk(col, c1 - 1).message_end

    def chunk_offsets(self, col: int, c0: int, c1: int) -> np.ndarray:
        out = np.zeros(c1 - c0 + 1, dtype=np.uint64)
        _lib.check(self.lib.vxg_file_chunk_offsets(self.handle, col, c0, c1,
                                                    out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out

    def column_tree(self, col: int, c0: int, c1: int, region: int = 0, region_offset: int = 0,
                    region_len: Optional[int] = None, chunk_offsets_dev: int = 0) -> _lib.VxgArray:
        """The ChunkedArray node of chunks [c0, c1) of column `col` (vxg_file_column_array);
        buffer pointers = region + (file offset - region_offset).  The node (and its subtree)
        is owned by the file."""
        out = C.POINTER(_lib.VxgArray)()
        rl = self.nbytes - region_offset if region_len is None else region_len
        _lib.check(self.lib.vxg_file_column_array(self.handle, col, c0, c1, C.c_void_p(region), region_offset, rl,
                                                  C.c_void_p(chunk_offsets_dev), C.byref(out)))
        return out.contents

    def close(self):
        if getattr(self, "handle", None):
            self.lib.vxg_file_close(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceColumns:
    """Chunks [c0, c1) of the given columns of `f` uploaded to HBM - one H2D copy of each
    column's contiguous message range (plus its chunk offsets) - and the reader's trees over
    them.  `refresh()` re-copies the bytes into the same device buffers (the next batch of a
    scan), leaving the trees valid."""

    def __init__(self, f: VortexFile, ctx, columns: Optional[Sequence[int]] = None, c0: int = 0,
                 c1: Optional[int] = None, stream=None):
        import torch
        self.f, self.ctx = f, ctx
        dev = torch.device("cuda", ctx.device)
        self.columns = list(range(len(f.columns))) if columns is None else list(columns)
        self.ranges, self.regions, self.offsets, self.nodes = [], [], [], []
        host = f._data if hasattr(f._data, "data_ptr") else torch.from_numpy(f._data)
        self._host = host
        for col in self.columns:
            n = f.columns[col].n_chunks
            e1 = n if c1 is None else min(c1, n)
            b, e = f.byte_range(col, c0, e1)
            region = torch.empty(e - b + REGION_SLACK, dtype=torch.uint8, device=dev)
            offs = torch.from_numpy(f.chunk_offsets(col, c0, e1).view(np.uint8).copy()).to(dev)
            self.ranges.append((b, e, c0, e1))
            self.regions.append(region)
            self.offsets.append(offs)
        self.refresh(stream)
        for col, region, offs, (b, e, s0, s1) in zip(self.columns, self.regions, self.offsets, self.ranges):
            self.nodes.append(f.column_tree(col, s0, s1, region.data_ptr(), b, e - b, offs.data_ptr()))

    def refresh(self, stream=None):
        """H2D of every column's byte range (non-blocking from pinned memory)."""
        for region, (b, e, _, _) in zip(self.regions, self.ranges):
            region[: e - b].copy_(self._host[b:e], non_blocking=True)

    def nbytes(self) -> int:
        return sum(e - b for b, e, _, _ in self.ranges)


def scan(f: VortexFile, ctx, columns: Optional[Sequence[int]] = None, c0: int = 0, c1: Optional[int] = None):
    """Canonicalize chunks [c0, c1) of the given columns (all by default): one H2D per column
    range, then one vxg_canonicalize per column -> [arrays.Canonical] (device tensors)."""
    from . import arrays as A
    dc = DeviceColumns(f, ctx, columns, c0, c1)
    outs = []
    for node in dc.nodes:
        keep: list = []
        o, res = A.alloc_canonical(ctx, node, keep)
        _lib.check(ctx.lib.vxg_canonicalize(ctx.handle, C.byref(node), C.byref(o), ctx.stream_ptr()))
        if res.validity is not None and not o.validity:
            res.validity = None
        res._keep = (keep, dc)
        outs.append(res)
    ctx.sync()
    return outs
