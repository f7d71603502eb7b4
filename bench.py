"""bench.py — device-resident decode throughput of the Vortex canonicalize hot path on MI355X.

Contract:
  python bench.py --gpus N --steps K --warmup W
  * one process per GPU over RCCL.  Run without torchrun and with N > 1, this script launches
    `python -m torch.distributed.run --nproc-per-node N ... bench.py` as a CHILD before it
    touches a GPU and exits with the child's status; every worker asserts WORLD_SIZE == N;
  * a "step" = one vxg_canonicalize (the drop-in C-ABI path) of one array whose buffers are
    already in HBM;
  * headline workload = BASELINE config C1 (FastLanes BitPacked u32, W=7, 64 Mi values) —
    the configuration the north-star target (>=70 % of HBM roofline) is quoted on; chunked
    arrays shard one chunk per GPU, so every rank decodes its own 64 Mi-value chunk
    (weak scaling, no data-path collective);
  * `value` = decoded bytes written by ALL ranks / max-over-ranks time (GB/s, whole job);
    `value_per_gpu` = value / N;
  * `roofline` = algorithmic bytes (packed read + decoded write) per launch / mean kernel
    time from HIP events on the decode stream, against 8.0 TB/s;
  * `cpu_baseline` = the oracle (C restatement of the reference's single-threaded
    canonicalize) on bounded samples of every config, rank 0 at N = 1 only: median of >= 20
    repetitions, 1 core, and all cores chunk-parallel for the chunked configs (C3, C5);
  * the other configs (C2 ALP f64; C3 the fixed 256-chunk Dict->BitPacked u64 table, split
    over the ranks = strong scaling; C4 FSST; C5 the TPC-H lineitem scan: 16 chunked columns,
    this rank's chunk range, read from a Vortex file's bytes) are measured the same way and
    reported under "encodings".
Inputs are rotated across several HBM copies so every step reads from HBM, not from the
256 MiB Infinity Cache; every copy decodes into its own outputs (plans and direct calls alike),
so no step rewrites the buffer the previous one wrote.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "decoded GB/s/GPU (device-resident) per encoding; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
C3_CHUNKS, C3_CHUNK_VALUES = 256, (128 << 20) // 256  # BASELINE C3: 128 Mi values in 256 chunks


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------ inputs
def c2_values(rng, n):
    """C2 data: 2-decimal prices + 0.1% random full-precision exceptions in the same range
    (never 2-decimal, so always ALP patches)."""
    vals = np.round(rng.uniform(1, 100000, n) * 100) / 100
    k = n // 1000
    vals[rng.choice(n, k, replace=False)] = rng.uniform(1, 100000, k) + 1e-7
    return vals


def c3_chunk_plain(c: int):
    """Plain data of chunk c of the C3 table (seeded by c so every rank agrees without
    communicating): 1024 random u64 dictionary values and Zipf(1.1) codes."""
    r = np.random.default_rng(1000 + c)
    dv = r.integers(0, 2 ** 63, 1024, dtype=np.uint64)
    codes = (r.zipf(1.1, C3_CHUNK_VALUES) - 1) % 1024
    return dv, codes.astype(np.uint64)


def c3_chunk(c: int, plain=None):
    """Chunk c of the C3 table: Dict(codes = BitPacked u64 W=10, values = Primitive u64[1024])."""
    import vortex_amd.arrays as A
    import vortex_amd.encode as E
    dv, codes = c3_chunk_plain(c) if plain is None else plain
    return A.dict_array(A.primitive(dv), A.bitpacked(E.bitpack_buffer(codes, 10), "u64", 10, C3_CHUNK_VALUES))


def c3_shard(world: int, rank: int) -> range:
    from vortex_amd.shard import plan_shards
    packed_bytes = (C3_CHUNK_VALUES // 1024) * 128 * 10 + 1024 * 8
    return plan_shards([packed_bytes] * C3_CHUNKS, world)[rank]


def c5_shard(world: int, rank: int) -> range:
    from tools import lineitem as L
    from vortex_amd.shard import plan_shards
    return plan_shards([1] * L.n_chunks(), world)[rank]


WORDS = (b"furiously regular deposits sleep carefully final accounts ironic packages blithely "
         b"quickly express requests pending theodolites slyly even instructions bold foxes "
         b"unusual asymptotes special platelets silent pinto beans fluffily careful dependencies "
         b"daring ideas close courts blithe dolphins quiet excuses ruthless warthogs").split()


def c4_heap(rng, n):
    """n synthetic TPC-H l_comment strings (10..43 chars cut from a word stream; dbgen is
    unavailable offline) -> (heap u8, offsets i64[n+1])."""
    lens = rng.integers(10, 44, n)
    total = int(lens.sum())
    wl = np.array([len(w) + 1 for w in WORDS])
    nw = int(total / wl.mean() * 1.1) + 16
    ids = rng.integers(0, len(WORDS), nw)
    mat = np.zeros((len(WORDS), wl.max()), dtype=np.uint8)
    for i, w in enumerate(WORDS):
        mat[i, : len(w)] = np.frombuffer(w, np.uint8)
        mat[i, len(w)] = 32
    rows = mat[ids]
    keep = np.arange(mat.shape[1])[None, :] < wl[ids][:, None]
    stream = rows[keep][:total]
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    return stream, offs


# ------------------------------------------------------------------------------ output checks
# Every timed workload's full-size output is checked after the timed region (never inside it):
# against the generator's plain values (C1, C2, C3: xxh3 of the exact bytes; C4: the exact views
# and heap, built here in numpy from the plain strings; C5: every numeric column's bytes and
# every string row's logical value) - no oracle involved.  Rotated copies must produce the same
# output bytes as the checked copy.
def _xxh(*bufs) -> int:
    import xxhash
    h = xxhash.xxh3_64()
    for b in bufs:
        h.update(memoryview(np.ascontiguousarray(b)).cast("B"))
    return h.intdigest()


def expected_views(heap: np.ndarray, offs: np.ndarray, bidx: int = 0) -> np.ndarray:
    """arrow-array 53.2 make_view over one data buffer: len <= 12 inline and
    zero padded, else {len, 4-byte prefix, buffer_index, offset} -> u8[n, 16]."""
    n = offs.size - 1
    lens = np.diff(offs).astype(np.uint32)
    starts = offs[:-1].astype(np.int64)
    pad = np.concatenate([heap, np.zeros(16, np.uint8)])
    first = pad[starts[:, None] + np.arange(12)[None, :]]
    first[np.arange(12)[None, :] >= lens[:, None]] = 0
    v = np.zeros((n, 16), np.uint8)
    v[:, :4] = lens.view(np.uint8).reshape(n, 4)
    inl = lens <= 12
    v[inl, 4:16] = first[inl]
    ni = ~inl
    v[ni, 4:8] = first[ni, :4]
    v[ni, 8:12] = np.frombuffer(np.uint32(bidx).tobytes(), np.uint8)
    v[ni, 12:16] = starts[ni].astype(np.uint32).view(np.uint8).reshape(-1, 4)
    return v


def strings_of(views: np.ndarray, data: np.ndarray, bufs, width: int):
    """Logical strings of canonical views (u8[n, 16]) over the data buffers (offset, len) in
    `data`: (lengths, u8[n, width] zero padded)."""
    n = views.shape[0]
    lens = views[:, :4].copy().view(np.uint32).reshape(n).astype(np.int64)
    if lens.size and lens.max() > width:
        raise AssertionError(f"string longer than {width}")
    out = np.zeros((n, width), np.uint8)
    inl = lens <= 12
    out[inl, : min(12, width)] = views[inl, 4: 4 + min(12, width)]
    ni = np.nonzero(~inl)[0]
    if ni.size:
        bidx = views[ni, 8:12].copy().view(np.uint32).reshape(-1).astype(np.int64)
        off = views[ni, 12:16].copy().view(np.uint32).reshape(-1).astype(np.int64)
        base = np.array([o for o, _ in bufs], np.int64)[bidx]
        blen = np.array([n_ for _, n_ in bufs], np.int64)[bidx]
        if np.any(off + lens[ni] > blen):
            raise AssertionError("view points past its data buffer")
        idx = np.minimum(base[:, None] + off[:, None] + np.arange(width)[None, :], data.size - 1)
        g = data[idx]
        g[np.arange(width)[None, :] >= lens[ni][:, None]] = 0
        out[ni] = g
        if not np.array_equal(views[ni, 4:8], g[:, :4]):
            raise AssertionError("view prefix differs from its bytes")
    out[np.arange(width)[None, :] >= lens[:, None]] = 0
    return lens, out


def plain_strings(strs, width: int):
    a = np.array(strs, dtype=f"S{width}")
    return np.char.str_len(a).astype(np.int64), np.frombuffer(a.tobytes(), np.uint8).reshape(len(strs), width)


def _host(t) -> np.ndarray:
    return t.cpu().numpy() if t is not None else None


def expect_hash(digest: int, what: str):
    def check(results):
        got = _xxh(_host(results[0].values))
        if got != digest:
            raise AssertionError(f"{what}: decoded bytes differ from the plain values")
    return check


def make_c1(rng, world, rank):
    """C1: 64 Mi u32 uniform in [0,128) -> BitPacked W=7, no patches (one chunk per GPU)."""
    import vortex_amd.encode as E
    vals = rng.integers(0, 128, 64 << 20, dtype=np.uint32)
    return E.encode_bitpacked(vals, bit_width=7, allow_patches=False), dict(
        name="C1", encoding="fastlanes.bitpacked u32 W=7", values=vals.size,
        read_bytes=vals.size * 7 // 8, write_bytes=vals.nbytes, dtype="u32",
        expect=expect_hash(_xxh(vals), "C1"))


def make_c2(rng, world, rank):
    """C2: 64 Mi f64 prices -> ALP->FoR->BitPacked(u64, W=24) + Sparse patches (one chunk per GPU)."""
    import vortex_amd.encode as E
    n = 64 << 20
    vals = c2_values(rng, n)
    arr = E.encode_alp(vals)
    return arr, dict(name="C2", encoding="vortex.alp(fastlanes.for(fastlanes.bitpacked u64)) f64",
                     values=n, read_bytes=arr.nbytes(), write_bytes=n * 8, dtype="f64",
                     expect=expect_hash(_xxh(vals), "C2"))


def make_c3(rng, world, rank):
    """C3: BASELINE's fixed table, Chunked x256 [Dict(codes=BitPacked u64 W=10, values=Primitive
    u64[1024])], 512 Ki values per chunk = 128 Mi values.  The table is the same at every N
    (strong scaling): this rank decodes the contiguous chunk range vortex_amd.shard.plan_shards
    gives it (balanced by compressed bytes; chunk_offsets, chunked/mod.rs:54-70), all 256 at N=1."""
    import xxhash
    import vortex_amd.arrays as A
    mine = c3_shard(world, rank)
    chunks, h = [], xxhash.xxh3_64()
    for c in mine:
        dv, codes = c3_chunk_plain(c)
        chunks.append(c3_chunk(c, (dv, codes)))
        h.update(memoryview(dv[codes]).cast("B"))  # take(values, codes), dict/array.rs:68-73
    arr = A.chunked(chunks)
    return arr, dict(expect=expect_hash(h.intdigest(), "C3"),name="C3", encoding="vortex.chunked[vortex.dict(codes=fastlanes.bitpacked u64 W=10)] u64",
                     values=len(mine) * C3_CHUNK_VALUES, read_bytes=arr.nbytes() - 8 * (len(mine) + 1),
                     write_bytes=len(mine) * C3_CHUNK_VALUES * 8, dtype="u64", chunks_per_gpu=len(mine),
                     chunk_range=[mine.start, mine.stop], global_chunks=C3_CHUNKS, strong_scaling=True)


def make_c4(rng, world, rank):
    """C4: 6 001 215 synthetic l_comment strings -> FSST (codes VarBin i32 offsets FoR/BitPacked,
    lengths FoR/BitPacked); one column per GPU (replicas)."""
    import vortex_amd.encode as E
    n = 6_001_215
    heap, offs = c4_heap(rng, n)
    arr = E.encode_fsst_from_heap(heap, offs)
    want_views, want_heap = _xxh(expected_views(heap, offs)), _xxh(heap)

    def check(results):
        r = results[0]
        if _xxh(_host(r.views)) != want_views:
            raise AssertionError("C4: views differ from make_view over the plain strings")
        if len(r.data_buffers) != 1 or _xxh(_host(r.data)[: r.data_buffers[0][1]]) != want_heap:
            raise AssertionError("C4: data buffer differs from the plain strings' bytes")
    return arr, dict(name="C4", encoding="vortex.fsst utf8 -> varbinview", values=n,
                     read_bytes=arr.nbytes(), write_bytes=int(offs[-1]) + 16 * n, dtype="u8", expect=check)


def c5_file(dist, rank: int) -> np.ndarray:
    """BASELINE C5's file: the whole synthetic SF1 lineitem table (tools/lineitem.py: 16 columns,
    92 chunks of 64 Ki rows, each chunk compressed with the sampling compressor's cascade; the
    three date columns as vortex.date extension arrays) written the way bench-vortex writes it
    (LayoutWriter::write_array_columns over a StructArray of ChunkedArrays, tpch/mod.rs:249-307;
    tools/vxfile.py).  Rank 0 writes it once to /tmp, the others read it after a barrier."""
    import tempfile
    from tools import lineitem as L
    from tools import vxfile as X
    path = Path(tempfile.gettempdir()) / f"vxg_lineitem_{os.environ.get('MASTER_PORT', 'single')}.vortex"
    if rank == 0:
        cols, _ = L.lineitem_columns(range(L.n_chunks()))
        written = []
        for name, _ in L.COLUMNS:
            chunks = cols[name].children[1:]
            if name in L.DATE_COLUMNS:
                chunks = [X.date_column(c) for c in chunks]
            written.append((name, chunks))
        data = X.write_file(written)
        del cols, written
        path.write_bytes(data)
    if dist is not None:
        dist.barrier()
    out = np.fromfile(path, dtype=np.uint8)
    if dist is not None:
        dist.barrier()
    if rank == 0:
        path.unlink(missing_ok=True)
    return out


def _tree_buffer_bytes(node) -> int:
    tot = sum(int(node.buffers[i].len) for i in range(node.n_buffers))
    return tot + sum(_tree_buffer_bytes(node.children[i]) for i in range(node.n_children))


class FileWorkload:
    """C5 "via vortex-serde": the lineitem file's bytes sit in pinned host memory; the engine's
    reader (vxg_file_*) parses footer, layouts and this rank's chunk messages; each column's
    message range is copied to HBM once (DeviceColumns); a step = one replay of the vxg_plan
    that canonicalizes the 16 reader-built ChunkedArray trees (struct_to_arrow,
    canonical.rs:169-187: one canonicalize per field).  `copies` device copies of the regions
    (each with its own plan) are replayed in turn so the inputs come from HBM."""

    def __init__(self, host, ctx, c0: int, c1: int, copies: int = 1):
        import torch
        import vortex_amd.arrays as A
        from vortex_amd.file import DeviceColumns, VortexFile
        self.ctx = ctx
        self.host = torch.from_numpy(host).pin_memory()
        t0 = time.perf_counter()
        self.f = VortexFile(self.host)
        self.dcs = [DeviceColumns(self.f, ctx, None, c0, c1)]
        torch.cuda.synchronize()
        self.setup_s = time.perf_counter() - t0
        self.dcs += [DeviceColumns(self.f, ctx, None, c0, c1) for _ in range(copies - 1)]
        # replayed many times: each plan measures its candidates (VXG_PLAN_MEASURE)
        self.plans = [A.Plan(dc.nodes, ctx, measure=True) for dc in self.dcs]
        self.n_copies = copies
        self.read_bytes = sum(_tree_buffer_bytes(n) for n in self.dcs[0].nodes)
        self.region_bytes = self.dcs[0].nbytes()
        self.input_bytes = self.region_bytes
        self.write_bytes = 0
        for r in self.plans[0].results:
            for t in (r.values, r.views, r.data):
                if t is not None:
                    self.write_bytes += int(t.numel())
        self.rows = int(self.dcs[0].nodes[0].len)
        self.i = 0

    def step(self):
        k = self.i
        self.i += 1
        self.plans[k % len(self.plans)].launch()

    def results(self, k: int):
        return self.plans[k].results

    def run_copy(self, k: int):
        self.i = k
        self.step()

    def nodes0(self):
        return list(self.dcs[0].nodes)

    def close(self):
        for p in self.plans:
            p.close()
        self.f.close()


def run_file_e2e(host, ctx, c0: int, c1: int, reps: int = 5) -> dict:
    """File bytes in (pinned host memory) -> Arrow buffers out (pinned host memory): reader
    parse (footer + layouts + this range's messages) + one H2D per column range + canonicalize
    (direct vxg_canonicalize per column) + D2H of every canonical buffer.  Median of `reps`."""
    import torch
    import vortex_amd.arrays as A
    from vortex_amd import _lib
    from vortex_amd.file import DeviceColumns, VortexFile
    hostt = torch.from_numpy(host).pin_memory()
    outs_h, times, parts = None, [], []
    for r in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f = VortexFile(hostt)
        dc = DeviceColumns(f, ctx, None, c0, c1)
        t1 = time.perf_counter()
        keep: list = []
        res = []
        for node in dc.nodes:
            o, rr = A.alloc_canonical(ctx, node, keep)
            _lib.check(ctx.lib.vxg_canonicalize(ctx.handle, C.byref(node), C.byref(o), ctx.stream_ptr()))
            res.append(rr)
        bufs = [t for rr in res for t in (rr.values, rr.views, rr.data, rr.validity) if t is not None]
        if outs_h is None:
            outs_h = [torch.empty(t.numel(), dtype=torch.uint8).pin_memory() for t in bufs]
        for hbuf, t in zip(outs_h, bufs):
            hbuf.copy_(t, non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ctx.sync()
        f.close()
        times.append(t2 - t0)
        parts.append((t1 - t0, t2 - t1))
    i = int(np.argsort(times[1:])[len(times[1:]) // 2]) + 1
    out_bytes = sum(int(h.numel()) for h in outs_h)
    return dict(e2e_ms=round(times[i] * 1e3, 3), parse_and_h2d_ms=round(parts[i][0] * 1e3, 3),
                decode_and_d2h_ms=round(parts[i][1] * 1e3, 3), file_bytes=int(host.size),
                h2d_bytes=int(dc.nbytes()), d2h_bytes=out_bytes,
                e2e_decoded_GBps=round(out_bytes / times[i] / 1e9, 2))


def c5_verify(results, chunks):
    """C5 outputs (the 16 lineitem columns' canonicals, in L.COLUMNS order) of the chunk range
    `chunks`, column by column against the generator's plain values: numeric columns byte for
    byte, string columns row by row (logical value of each view), row counts exact, no nulls."""
    from tools import lineitem as L
    host_res = []
    for r in results:
        if r.kind == "primitive":
            host_res.append(("p", _host(r.values)))
        else:
            host_res.append(("s", _host(r.views).reshape(-1, 16), _host(r.data), r.data_buffers))
        if r.validity is not None and not _host(r.validity).all():
            raise AssertionError("C5: unexpected nulls")
    row = 0
    for c in chunks:
        vals = L.chunk_values(c)
        n = vals["l_orderkey"].size
        for (name, _), hr in zip(L.COLUMNS, host_res):
            v = vals[name]
            if hr[0] == "p":
                w = v.dtype.itemsize
                if hr[1][row * w: (row + n) * w].tobytes() != v.tobytes():
                    raise AssertionError(f"C5 {name}: chunk {c} differs")
            else:
                width = max(len(x) for x in v)
                gl, gs = strings_of(hr[1][row: row + n], hr[2], hr[3], max(width, 1))
                el, es = plain_strings(v, max(width, 1))
                if not (np.array_equal(gl, el) and np.array_equal(gs, es)):
                    raise AssertionError(f"C5 {name}: chunk {c} strings differ")
        row += n
    for (name, kind), hr in zip(L.COLUMNS, host_res):
        n_out = hr[1].size // {"i64": 8, "f64": 8, "i32": 4}[kind] if hr[0] == "p" else hr[1].shape[0]
        if n_out != row:
            raise AssertionError(f"C5 {name}: {n_out} rows out, {row} expected")
    return row


def make_c5(rng, world, rank, dist=None):
    """C5: bench-vortex's TPC-H lineitem scan -> canonicalize "via vortex-serde": the table is
    read from a Vortex file's bytes (c5_file) by the engine's reader.  The table is fixed
    (strong scaling): the 92 chunks are split into contiguous ranges, one per rank, and a step
    canonicalizes every column of this rank's range."""
    from tools import lineitem as L
    mine = c5_shard(world, rank)
    host = c5_file(dist, rank)

    def check(results):
        c5_verify(results, mine)

    return ("file", host, mine.start, mine.stop), dict(expect=check,
        name="C5", encoding="lineitem scan from Vortex file bytes: 16 x vortex.chunked[<per-column cascades>] -> canonical",
        values=0, read_bytes=0, write_bytes=0, dtype="mixed", chunks_per_gpu=len(mine),
        chunk_range=[mine.start, mine.stop], global_chunks=L.n_chunks(), strong_scaling=True)


# ------------------------------------------------------------------------------ timing
class Workload:
    """One or more arrays (C5: the 16 lineitem columns) with preallocated canonical outputs; a
    step canonicalizes each of them once through the C ABI, on one stream.  By default a step
    is one replay of a vxg_plan (the planner's launches recorded once as a HIP graph: every
    kernel runs every step, without per-step host planning and per-kernel submission);
    graph=False calls vxg_canonicalize per array per step instead."""

    def __init__(self, arrs, info, ctx, copies: int, graph: bool = True):
        import torch
        import vortex_amd.arrays as A
        self.info, self.ctx, self.graph = info, ctx, graph
        arrs = arrs if isinstance(arrs, list) else [arrs]
        dev = torch.device("cuda", ctx.device)
        self.copies = [[arr.to(dev) for arr in arrs] for _ in range(copies)]
        self.n_copies = copies
        if graph:
            self.plans = [A.Plan(trees, ctx, measure=True) for trees in self.copies]
        else:
            # every rotated copy decodes into its own outputs too: rewriting one output buffer
            # step after step would let the Infinity Cache absorb part of the writes
            self.keep = []
            self.cols = []
            self.outs = [[] for _ in range(copies)]
            for j, arr in enumerate(arrs):
                nodes = [A.flatten(trees[j], self.keep) for trees in self.copies]
                outs = []
                for k in range(copies):
                    o, res = A.alloc_canonical(ctx, nodes[k], self.keep)
                    outs.append(o)
                    self.outs[k].append(res)
                self.cols.append((nodes, outs))
        self.i = 0
        self.input_bytes = sum(a.nbytes() for a in arrs)

    def results(self, k: int):
        """Canonical outputs of copy k."""
        return self.plans[k].results if self.graph else self.outs[k]

    def run_copy(self, k: int):
        self.i = k
        self.step()

    def step(self):
        k = self.i
        self.i += 1
        if self.graph:
            self.plans[k % len(self.plans)].launch()
            return
        for nodes, outs in self.cols:
            chk(self.ctx.lib.vxg_canonicalize(self.ctx.handle, C.byref(nodes[k % len(nodes)]),
                                              C.byref(outs[k % len(outs)]), self.ctx.stream_ptr()))

    def nodes0(self):
        self.keep0 = []
        return [A_flatten(t, self.keep0) for t in self.copies[0]]

    def close(self):
        for p in getattr(self, "plans", []):
            p.close()


def chk(st):
    from vortex_amd import _lib
    _lib.check(st)


def A_flatten(tree, keep):
    import vortex_amd.arrays as A
    return A.flatten(tree, keep)


def plan_report(wl, steps: int) -> dict:
    """What the replayed plan hides: the kept graph's mode and its measured
    candidates (vxg_plan_get_info of copy 0's plan), and what a ONE-SHOT scan of copy 0 pays
    instead: vxg_plan_create without measurement + its first replay (device time by HIP events,
    create by host wall clock), and direct vxg_canonicalize calls of every array per step (no
    graph; host wall time per step over `steps` back-to-back steps, outputs preallocated)."""
    import torch
    import vortex_amd.arrays as A
    ctx = wl.ctx
    info = wl.plans[0].info()
    nodes = wl.nodes0()
    p = A.Plan(nodes, ctx)
    create_ms = p.info()["create_ms"]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    p.launch()
    e1.record()
    torch.cuda.synchronize()
    first_wall = (time.perf_counter() - t0) * 1e3
    ctx.sync()
    first_dev = e0.elapsed_time(e1)
    one_shot_mode = p.info()
    p.close()
    keep: list = []
    outs = [A.alloc_canonical(ctx, n, keep)[0] for n in nodes]

    def direct():
        for n, o in zip(nodes, outs):
            chk(ctx.lib.vxg_canonicalize(ctx.handle, C.byref(n), C.byref(o), ctx.stream_ptr()))
    for _ in range(3):
        direct()
    ctx.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        direct()
    torch.cuda.synchronize()
    direct_ms = (time.perf_counter() - t0) * 1e3 / steps
    ctx.sync()
    del keep, outs
    return {"plan_mode": {"batched": info["batched"], "branches": info["branches"],
                          "direct_launch_nodes": info["direct_nodes"]},
            "plan_candidates": info["candidates"], "plan_create_ms_measured": info["create_ms"],
            "one_shot": {"plan_create_ms": create_ms, "batched": one_shot_mode["batched"],
                         "first_replay_device_ms": round(first_dev, 4), "first_replay_wall_ms": round(first_wall, 4),
                         "create_plus_first_replay_ms": round(create_ms + first_wall, 4),
                         "no_graph_ms_per_step": round(direct_ms, 4)}}


def run_workload(wl, steps: int, warmup: int, dist):
    """Warmup, then exactly `steps` back-to-back steps between barrier + synchronize.  Two HIP
    events on the decode stream (torch's current stream, the stream the engine is given) bracket
    the timed steps: (end - start) / steps is the mean device time per step (per launch for a
    one-kernel step like C1).  No event sits between the timed steps: a timing event between two
    kernels waits for the first one's memory release and stretches each interval by ~2-3 us on a
    60 us kernel (rocprofv3's average of the same launches agrees with the two-event mean, not
    with per-step events).  A second, untimed pass with an event after every step gives the
    per-step median."""
    import torch
    for _ in range(warmup):
        wl.step()
    wl.ctx.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for s in range(steps):
        wl.step()
    e1.record()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    wl.ctx.sync()  # surfaces device-side errors (OOB codes, ...)
    kmean = e0.elapsed_time(e1) / steps
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    evs[0].record()
    for s in range(steps):
        wl.step()
        evs[s + 1].record()
    torch.cuda.synchronize()
    wl.ctx.sync()
    kmed = float(np.median([evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]))
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, kmean, kmed


def verify_workload(wl, expect) -> dict:
    """After the timed region: replay every rotated copy once and check its output - copy 0
    against the plain values (`expect`), every other copy byte-equal to copy 0."""
    ref = None
    for k in range(wl.n_copies):
        wl.run_copy(k)
        wl.ctx.sync()
        res = wl.results(k)
        hs = []
        for r in res:
            hs += [_xxh(_host(t)) for t in (r.values, r.views, r.validity) if t is not None]
            if r.data is not None:  # each data buffer's bytes (the 16-byte alignment gaps are never written)
                d = _host(r.data)
                hs += [_xxh(d[o: o + n]) for o, n in r.data_buffers]
        if k == 0:
            expect(res)
            ref = hs
        elif hs != ref:
            raise AssertionError(f"{wl.info['name'] if hasattr(wl, 'info') else 'C5'}: copy {k} output differs")
    return {"verified": True, "copies_checked": wl.n_copies}


def run_e2e(arr, info, ctx, reps: int = 5):
    """Host -> host rate: compressed buffers in pinned host memory are copied H2D, decoded,
    and the canonical output copied D2H into pinned host memory (PCIe Gen5 x16 both ways).
    Returns decoded GB/s over the whole round trip and the H2D/D2H byte counts."""
    import torch
    import vortex_amd.arrays as A
    dev = torch.device("cuda", ctx.device)

    def pin(a):
        return A.Array(a.encoding, a.len, a.dtype, a.ptype, a.nullable, a.validity, dict(a.meta),
                       [torch.from_numpy(np.ascontiguousarray(b).view(np.uint8).reshape(-1).copy()).pin_memory()
                        for b in a.buffers], [pin(c) for c in a.children])

    host = pin(arr)
    dev_tree = host.to(dev)  # allocate device buffers once (shapes fixed)

    def h2d(src, dst):
        for s, d in zip(src.buffers, dst.buffers):
            if s.numel():
                d.copy_(s, non_blocking=True)
        for s, d in zip(src.children, dst.children):
            h2d(s, d)

    keep = []
    node = A.flatten(dev_tree, keep)
    vb, db = C.c_uint64(), C.c_uint64()
    chk(ctx.lib.vxg_canonical_size(ctx.handle, C.byref(node), C.byref(vb), C.byref(db)))
    out = A._lib.VxgCanonical()
    prim = arr.dtype == A.DTYPE["PRIMITIVE"]
    if prim:
        dv = torch.empty(vb.value, dtype=torch.uint8, device=dev)
        out.values = dv.data_ptr()
        hv = torch.empty(vb.value, dtype=torch.uint8).pin_memory()
    else:
        dv = torch.empty(vb.value, dtype=torch.uint8, device=dev)
        dd = torch.empty(db.value + 16, dtype=torch.uint8, device=dev)
        out.views, out.data, out.data_bytes = dv.data_ptr(), dd.data_ptr(), db.value
        hv = torch.empty(vb.value, dtype=torch.uint8).pin_memory()
        hd = torch.empty(db.value + 16, dtype=torch.uint8).pin_memory()
    times = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h2d(host, dev_tree)
        chk(ctx.lib.vxg_canonicalize(ctx.handle, C.byref(node), C.byref(out), ctx.stream_ptr()))
        hv.copy_(dv, non_blocking=True)
        if not prim:
            hd.copy_(dd, non_blocking=True)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    ctx.sync()
    t = float(np.median(times[1:]))
    d2h = vb.value + (0 if prim else db.value)
    return dict(e2e_ms=round(t * 1e3, 3), e2e_decoded_GBps=round(info["write_bytes"] / t / 1e9, 2),
                h2d_bytes=arr.nbytes(), d2h_bytes=int(d2h),
                pcie_GBps_effective=round((arr.nbytes() + d2h) / t / 1e9, 2))


def pmc_traffic(name: str):
    """Per-launch HBM bytes of the dominant kernel from committed rocprofv3 PMC summaries
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py: FETCH_SIZE*2 + WRITE_SIZE,
    KiB -> bytes, gfx950 read correction per MI355X_MICROARCH.md §HBM).  Not measured by this
    run: the PMC passes need their own rocprofv3 runs (see `roofline.traffic_source`)."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d.get(name, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


# ------------------------------------------------------------------------------ CPU baseline
def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_cores() -> int:
    """Host cores this process may use (the GPU box's share is 16 per GPU; the affinity mask
    may show the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


_POOL_ITEMS: list = []


def _pool_decode(idxs):
    """Worker: canonicalize the given items through the oracle; returns decoded bytes."""
    from oracle_tree import canon
    tot = 0
    for i in idxs:
        for a in _POOL_ITEMS[i]:
            v, _ = canon(a)
            tot += v.nbytes if hasattr(v, "nbytes") else 0
    return tot


def _median_time(fn, reps: int, budget_s: float):
    ts = []
    t_start = time.perf_counter()
    for r in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        if r >= 4 and time.perf_counter() - t_start > budget_s:
            break
    return float(np.median(ts)), len(ts)


def cpu_baselines(budget_s: float, reps: int = 20) -> dict:
    """The oracle ("port": the reference is Rust and cannot be built here) timed on this box's
    host cores, in the reference's structure (per-block unpack, one materialised buffer per
    cascade level, serial pack_primitives; fresh outputs like the reference allocates per call),
    median of `reps` repetitions on a bounded sample of each config.  C1 is also timed with a
    pre-faulted output.  The chunked configs (C3, C5) are also timed chunk-parallel over all
    cores (fork pool; each worker canonicalizes whole chunks, outputs stay in the worker).
    Runs before anything touches the GPU, so the pool forks a GPU-free process."""
    import multiprocessing as mp
    sys.path.insert(0, str(ROOT / "tests"))
    from oracle import oracle as O
    from oracle_tree import canon
    import vortex_amd.encode as E
    from tools import lineitem as L
    cores = _cpu_cores()
    per_budget = budget_s / 7
    out = {"nproc": os.cpu_count(), "cores_all": cores, "reps": reps, "kind": "port", "cpu_model": cpu_model()}
    Lb = O.lib()
    # C1 full array, 1 core
    rng = np.random.default_rng(42)
    vals = rng.integers(0, 128, 64 << 20, dtype=np.uint32)
    packed = np.zeros((vals.size // 1024) * 128 * 7, np.uint8)
    Lb.vxo_bitpack(O.PT["u32"], 7, O.p(vals), vals.size, O.p(packed))
    pre = np.empty_like(vals)
    pre.fill(1)

    def c1(fresh):
        o = np.empty_like(vals) if fresh else pre
        assert Lb.vxo_unpack(O.PT["u32"], 7, 0, vals.size, O.p(packed), packed.size, O.p(o)) == 0
    t_fresh, n1 = _median_time(lambda: c1(True), reps, per_budget)
    t_pre, _ = _median_time(lambda: c1(False), reps, per_budget)
    assert np.array_equal(pre, vals)
    out["C1"] = {"sample": "full C1 (64 Mi u32 W=7)", "1core_GBps": round(vals.nbytes / t_fresh / 1e9, 3),
                 "1core_prefaulted_GBps": round(vals.nbytes / t_pre / 1e9, 3), "reps": n1}
    # C2: 8 Mi values of the C2 distribution
    n2 = 8 << 20
    a2 = E.encode_alp(c2_values(np.random.default_rng(43), n2))
    t2, r2 = _median_time(lambda: canon(a2), reps, per_budget)
    out["C2"] = {"sample": "8 Mi f64 of the C2 distribution, ALP->FoR->BitPacked + patches",
                 "1core_GBps": round(n2 * 8 / t2 / 1e9, 3), "reps": r2}
    # C3: 16 of the 256 chunks (8 Mi values)
    c3 = [[c3_chunk(c)] for c in range(16)]
    # C4: 1 Mi strings
    heap, offs = c4_heap(np.random.default_rng(44), 1 << 20)
    a4 = E.encode_fsst_from_heap(heap, offs)
    t4, r4 = _median_time(lambda: canon(a4), reps, per_budget)
    out["C4"] = {"sample": "1 Mi synthetic l_comment strings, FSST",
                 "1core_GBps": round((int(offs[-1]) + 16 * (1 << 20)) / t4 / 1e9, 3), "reps": r4}
    # C5: 16 of the 92 lineitem chunks x 16 columns (>= the 16 cores of the all-core run)
    n5 = max(16, cores)
    cols, plain = L.lineitem_columns(range(n5))
    c5 = [[cols[name].children[1 + i] for name, _ in L.COLUMNS] for i in range(n5)]
    c5_bytes = sum(L.canonical_bytes(v) for vs in plain.values() for v in vs)
    c3_bytes = 16 * C3_CHUNK_VALUES * 8
    global _POOL_ITEMS
    for key, items, nbytes, sample in (("C3", c3, c3_bytes, "16 of the 256 C3 chunks (8 Mi u64)"),
                                       ("C5", c5, c5_bytes, f"{n5} of the 92 lineitem chunks x 16 columns")):
        _POOL_ITEMS = items
        t1, r1 = _median_time(lambda: _pool_decode(range(len(items))), reps, per_budget)
        ent = {"sample": sample, "1core_GBps": round(nbytes / t1 / 1e9, 3), "reps": r1}
        if cores > 1:
            ctx = mp.get_context("fork")
            with ctx.Pool(min(cores, len(items))) as pool:
                parts = [list(range(i, len(items), cores)) for i in range(min(cores, len(items)))]
                pool.map(_pool_decode, parts)  # warm the workers
                tp, rp = _median_time(lambda: pool.map(_pool_decode, parts), reps, per_budget)
            ent.update({"all_core_GBps": round(nbytes / tp / 1e9, 3), "all_core_reps": rp,
                        "cores": min(cores, len(items))})
        out[key] = ent
    _POOL_ITEMS = []
    return out


# ------------------------------------------------------------------------------ launch
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_workers(n: int) -> int:
    """`--gpus N` without torchrun: start N workers through torch.distributed.run as a child
    process (nothing here has touched a GPU) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "bench.py")] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"[bench] launching {n} workers: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


def launcher_selftest(world: int, rank: int) -> None:
    """--launcher-selftest (CPU, gloo): every worker reports its rank and the C3/C5 chunk ranges
    it would decode; rank 0 gathers them and prints one JSON line."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    assert dist.get_world_size() == world and dist.get_rank() == rank
    mine = [rank, world, c3_shard(world, rank).start, c3_shard(world, rank).stop,
            c5_shard(world, rank).start, c5_shard(world, rank).stop]
    parts = [torch.zeros(6, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(parts, torch.tensor(mine, dtype=torch.int64))
    t = torch.tensor([float(rank)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"selftest": True, "world": world, "max_rank": t.item(),
                          "ranks": [p.tolist() for p in parts]}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workloads", default="c1,c2,c3,c4,c5",
                    help="comma list; c1 is the headline, others go under 'encodings'")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true",
                    help="call vxg_canonicalize per array per step instead of replaying a vxg_plan graph")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="diagnostic: with one process, build rank 0's shard of an N-GPU run of C3/C5")
    ap.add_argument("--e2e", action="store_true",
                    help="also measure host->host (H2D + decode + D2H over PCIe); never the headline value")
    ap.add_argument("--copies", type=int, default=0,
                    help="diagnostic: rotated input copies for every workload (default: per config, > 256 MiB)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the post-timing check of every output against the plain values")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="CPU check of the multi-process launch (gloo): print every rank's chunk ranges")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_workers(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        log(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={world}")
        sys.exit(2)
    if args.launcher_selftest:
        launcher_selftest(world, rank)
        return

    # the CPU baseline runs first: its fork pool must not inherit an initialised GPU runtime
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        t0 = time.perf_counter()
        cpu = cpu_baselines(args.cpu_seconds)
        log(f"[bench] cpu baseline: {time.perf_counter() - t0:.1f}s")

    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus

    import vortex_amd as V
    ctx = V.Context(local)
    rng = np.random.default_rng(42 + rank)
    # --simulate-world N (diagnostic, single process): rank 0's shard of an N-GPU run of the
    # sharded configs, to read one GPU's share of the N-GPU work before an N-GPU node is used
    shard_world = args.simulate_world if args.simulate_world and world == 1 else world
    makers = {"c1": make_c1, "c2": make_c2, "c3": make_c3, "c4": make_c4, "c5": make_c5}
    # Rotated HBM copies of every input, so the rotated total exceeds the 256 MiB Infinity Cache
    # (MI355X_MICROARCH.md): C1 8 x 58.7 MB, C2 2 x 202 MB, C3 2 x 170 MB, C4 4 x 77 MB,
    # C5 2 x 180 MB of file regions (one plan per copy)
    copies = {"c1": 8, "c2": 2, "c3": 2, "c4": 4, "c5": 2}
    if args.copies:
        copies = {k: args.copies for k in copies}
    results = {}
    for key in [w.strip() for w in args.workloads.split(",") if w.strip()]:
        t0 = time.perf_counter()
        arr, info = makers[key](rng, shard_world, rank, dist) if key == "c5" else makers[key](rng, shard_world, rank)
        if isinstance(arr, tuple) and arr[0] == "file":
            _, host, c0, c1 = arr
            e2e = run_file_e2e(host, ctx, c0, c1) if args.e2e else None
            wl = FileWorkload(host, ctx, c0, c1, copies[key])
            info.update(values=wl.rows, read_bytes=wl.read_bytes, write_bytes=wl.write_bytes,
                        h2d_region_bytes=wl.region_bytes, reader_setup_ms=round(wl.setup_s * 1e3, 2))
        else:
            e2e = run_e2e(arr, info, ctx) if args.e2e and not isinstance(arr, list) else None
            # one-array steps are one or two back-to-back kernel launches: direct calls overlap
            # the next submission with the running kernel (a graph replay measured 2-6 us slower
            # per step on C1, C2, C4); multi-array steps and C3's 256-chunk table (one launch over
            # a device chunk table instead of 8 kernel-argument tables) replay a plan
            wl = Workload(arr, info, ctx, copies[key], graph=(isinstance(arr, list) or key == "c3") and not args.no_graph)
        del arr
        if rank == 0:
            log(f"[bench] {info['name']}: built in {time.perf_counter() - t0:.1f}s; timing...")
        # every config: >= 20 timed steps after >= 3 warm-ups (median of >= 20 reps)
        steps = args.steps if key == "c1" else max(20, args.steps)
        warm = args.warmup if key == "c1" else max(3, args.warmup)
        elapsed, kmean, kmed = run_workload(wl, steps, warm, dist)
        check = None
        if not args.no_verify:
            t1 = time.perf_counter()
            check = verify_workload(wl, info.pop("expect"))
            check["verify_s"] = round(time.perf_counter() - t1, 1)
            if rank == 0:
                log(f"[bench] {info['name']}: output verified ({wl.n_copies} copies, {check['verify_s']} s)")
        info.pop("expect", None)
        rotation = {"copies": wl.n_copies, "input_bytes_per_copy": int(wl.input_bytes),
                    "rotated_input_bytes": int(wl.n_copies * wl.input_bytes),
                    "exceeds_infinity_cache": bool(wl.n_copies * wl.input_bytes > 256 * 2 ** 20)}
        per_step = elapsed / steps
        algo = info["read_bytes"] + info["write_bytes"]
        total_write = world * info["write_bytes"]
        if info.get("strong_scaling") and dist is not None:  # ranks hold different shares of one table
            t = torch.tensor([float(info["write_bytes"])], dtype=torch.float64, device="cuda")
            dist.all_reduce(t)
            total_write = float(t.item())
        plan = plan_report(wl, steps) if getattr(wl, "plans", None) else None
        results[key] = dict(info=info, elapsed=elapsed, ms_per_step=per_step * 1e3, kernel_ms_mean=kmean,
                            kernel_ms_median=kmed, algo_bytes=algo, steps=steps, warmup=warm, plan=plan,
                            value=total_write * steps / elapsed / 1e9, e2e=e2e, check=check, rotation=rotation)
        wl.close()
        del wl
        torch.cuda.empty_cache()

    if rank == 0:
        head_key = "c1" if "c1" in results else next(iter(results))
        h = results[head_key]
        info = h["info"]
        achieved = h["algo_bytes"] / (h["kernel_ms_mean"] / 1e3) / 1e9
        line = {
            "metric": METRIC,
            "value": round(h["value"], 2),
            "unit": "GB/s",
            "value_per_gpu": round(h["value"] / world, 2),
            "value_aggregate": round(h["value"], 2),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(h["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": info["dtype"],
            "data": "synthetic (seeded; inputs resident in HBM, rotated across copies)",
            "launch": "headline (C1), C2, C4: direct vxg_canonicalize per step; C3 (256-chunk table) and C5 (16 columns): vxg_plan replay (HIP graph, or direct launches of a short kernel chain)"
                      + (" disabled (--no-graph)" if args.no_graph else ""),
            "config": {"workload": f"{info['name']}: {info['encoding']}, {info['values']} values per GPU, "
                                   f"one chunk per GPU", "values_per_gpu": info["values"],
                       "parallelism": f"chunk-per-GPU x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic("fl_unpack_u32_w7") if head_key == "c1" else None,
                         "traffic_source": "profiles/pmc_traffic.json (committed rocprofv3 --pmc FETCH_SIZE / "
                                           "WRITE_SIZE passes of this workload; not this run)",
                         "kernel_ms_mean": round(h["kernel_ms_mean"], 5),
                         "kernel_ms_median": round(h["kernel_ms_median"], 5),
                         "algorithmic_bytes_per_launch": h["algo_bytes"]},
            "verified": bool(h["check"] and h["check"]["verified"]),
            "host": {"cpu_model": cpu_model(), "nproc": os.cpu_count(), "cores_used_max": _cpu_cores()},
            "encodings": {},
        }
        for k, r in results.items():
            i = r["info"]
            ent = {
                "encoding": i["encoding"], "values_per_gpu": i["values"],
                "scaling": "strong" if i.get("strong_scaling") else "weak",
                "decoded_GBps_total": round(r["value"], 2),
                "decoded_GBps_per_gpu": round(r["value"] / world, 2),
                "decoded_GBps_per_gpu_kernel": round(i["write_bytes"] / (r["kernel_ms_mean"] / 1e3) / 1e9, 1),
                "hbm_frac_algorithmic": round(r["algo_bytes"] / (r["kernel_ms_mean"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "kernel_ms_mean": round(r["kernel_ms_mean"], 5), "kernel_ms_median": round(r["kernel_ms_median"], 5),
                "ms_per_step": round(r["ms_per_step"], 5), "steps": r["steps"], "warmup": r["warmup"],
                "read_bytes": i["read_bytes"], "write_bytes": i["write_bytes"]}
            if r.get("plan"):
                ent.update(r["plan"])
            for extra in ("chunks_per_gpu", "chunk_range", "global_chunks", "h2d_region_bytes", "reader_setup_ms"):
                if extra in i:
                    ent[extra] = i[extra]
            ent["rotation"] = r["rotation"]
            ent["verified"] = bool(r["check"] and r["check"]["verified"])
            if cpu is not None and i["name"] in cpu:
                ent["cpu_baseline"] = cpu[i["name"]]
            if r.get("e2e"):
                ent["host_to_host"] = r["e2e"]
            line["encodings"][i["name"]] = ent
        if cpu is not None:
            c1 = cpu["C1"]
            line["cpu_baseline"] = {
                "value": c1["1core_GBps"], "unit": "GB/s", "cores": 1, "kind": "port",
                "sample": f"C1 full array (64 Mi u32, W=7) decoded by oracle/vx_oracle.c vxo_unpack (-O3 "
                          f"-march=native), fresh output per call, median of {c1['reps']} reps "
                          f"(pre-faulted output: {c1['1core_prefaulted_GBps']} GB/s); {cpu['cpu_model']}, nproc={cpu['nproc']}; "
                          f"C2-C5 (1 core, and all {cpu['cores_all']} cores for C3/C5) under encodings.*.cpu_baseline"}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
