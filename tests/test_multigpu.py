"""N>1 path on CPU: chunk sharding + the max-over-ranks timing reduction with gloo, world 2 and 4.

Each rank builds the same seeded ChunkedArray, takes its contiguous chunk range
(vortex_amd/shard.py), decodes it with the oracle into its output slice, and the gathered slices
must equal the single-process decode of the whole array.  The GPU version of the same code path
runs in bench.py (RCCL barrier instead of gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import vortex_amd.arrays as A
import vortex_amd.encode as E
from vortex_amd.shard import plan_shards, rank_shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def build_chunked(seed=0, n_chunks=13):
    rng = np.random.default_rng(seed)
    chunks = []
    for c in range(n_chunks):
        n = int(rng.integers(500, 5000))
        kind = c % 3
        if kind == 0:
            dv = rng.integers(0, 2 ** 40, 64, dtype=np.uint64)
            vals = dv[rng.integers(0, 64, n)]
            chunks.append(E.encode_dict(vals))
        elif kind == 1:
            chunks.append(E.encode_bitpacked(rng.integers(0, 1 << 11, n, dtype=np.uint64)))
        else:
            chunks.append(E.encode_delta(np.cumsum(rng.integers(0, 4, n)).astype(np.uint64)))
    return A.chunked(chunks)


def test_plan_shards_covers_all_chunks_contiguously():
    for n in (0, 1, 5, 256):
        for world in (1, 2, 3, 8):
            w = np.random.default_rng(n).integers(1, 100, n)
            rs = plan_shards(w, world)
            assert len(rs) == world
            flat = [i for r in rs for i in r]
            assert flat == list(range(n))
            if n >= world * 4:
                tot = w.sum()
                assert max(w[list(r)].sum() for r in rs) <= tot / world + w.max()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle_tree import canon
    arr = build_chunked()
    sub, first, length = rank_shard(arr, rank, world)
    part = canon(sub)[0] if sub is not None else np.zeros(0, np.uint64)
    assert part.size == length
    # gather variable-size slices (pad to max)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([length], dtype=torch.int64))
    mx = int(max(s.item() for s in sizes))
    buf = torch.zeros(mx, dtype=torch.int64)
    buf[:length] = torch.from_numpy(part.view(np.int64))
    bufs = [torch.zeros(mx, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(bufs, buf)
    firsts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(firsts, torch.tensor([first], dtype=torch.int64))
    # the bench's max-over-ranks timing reduction
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        out = np.zeros(arr.len, np.int64)
        for r in range(world):
            n = int(sizes[r].item())
            f = int(firsts[r].item())
            out[f:f + n] = bufs[r][:n].numpy()
        full = canon(arr)[0].view(np.int64)
        q.put((bool(np.array_equal(out, full)), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_decode_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok
    assert tmax == float(world)
