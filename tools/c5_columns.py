"""Per-column isolation of BASELINE C5 (the lineitem scan read from Vortex file bytes).

Every column of the file is canonicalized ALONE (one vxg_canonicalize per step on one stream,
so a rocprofv3 --kernel-trace of this script gives each kernel its own duration), timed with
HIP events over `reps` back-to-back steps; prints one JSON line per column with its kernel
time, algorithmic bytes (compressed buffers read + canonical bytes written) and fraction of the
8 TB/s HBM roofline, then the sum.  Usage:
  python tools/c5_columns.py [--world N --rank R] [--reps 20] [--mark]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rotate", type=int, default=1,
                    help="device copies of the file regions the plan-mode steps rotate through")
    ap.add_argument("--mark", action="store_true",
                    help="launch a torch kernel before every column (segments a rocprofv3 --pmc trace; tools/c5_traffic.py)")
    args = ap.parse_args()
    import torch
    import bench
    import vortex_amd as V
    import vortex_amd.arrays as A
    from vortex_amd import _lib
    from vortex_amd.file import DeviceColumns, VortexFile
    mine = bench.c5_shard(args.world, args.rank)
    host = torch.from_numpy(bench.c5_file(None, 0)).pin_memory()
    ctx = V.Context(0)
    f = VortexFile(host)
    dc = DeviceColumns(f, ctx, None, mine.start, mine.stop)
    # --rotate K: K device copies of the column regions, the plan-mode steps cycle through them
    # (one plan per copy) so a column's inputs come from HBM, not from the Infinity Cache
    rot = [dc] + [DeviceColumns(f, ctx, None, mine.start, mine.stop) for _ in range(args.rotate - 1)]
    tot_t = tot_p = tot_b = 0.0
    marker = torch.zeros(1, device="cuda")
    for ci, (col, node) in enumerate(zip(dc.columns, dc.nodes)):
        keep: list = []
        o, res = A.alloc_canonical(ctx, node, keep)
        if args.mark:  # after the output sizing (its length readback is not a decode step)
            torch.cuda.synchronize()
            marker.add_(1)
            torch.cuda.synchronize()

        def step():
            _lib.check(ctx.lib.vxg_canonicalize(ctx.handle, C.byref(node), C.byref(o), ctx.stream_ptr()))
        for _ in range(3):
            step()
        ctx.sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        # the same column as its own vxg_plan (device chunk tables: one launch per kernel group)
        plans = [A.Plan([r.nodes[ci]], ctx, measure=True) for r in rot]
        for k in range(3):
            plans[k % len(plans)].launch()
        ctx.sync()
        e0.record()
        for k in range(args.reps):
            plans[k % len(plans)].launch()
        e1.record()
        torch.cuda.synchronize()
        plan_ms = e0.elapsed_time(e1) / args.reps
        for p in plans:
            p.close()
        rb = bench._tree_buffer_bytes(node)
        wb = sum(int(t.numel()) for t in (res.values, res.views, res.data) if t is not None)
        tot_t += ms
        tot_p += plan_ms
        tot_b += rb + wb
        print(json.dumps({"column": f.columns[col].name, "chunks": len(mine), "rotate": args.rotate, "ms": round(ms, 4),
                          "plan_ms": round(plan_ms, 4), "read_bytes": rb, "write_bytes": wb,
                          "hbm_frac": round((rb + wb) / ms / 1e6 / 8000, 3),
                          "plan_hbm_frac": round((rb + wb) / plan_ms / 1e6 / 8000, 3)}), flush=True)
    print(json.dumps({"column": "SUM (sequential)", "ms": round(tot_t, 4), "plan_ms": round(tot_p, 4),
                      "bytes": tot_b, "hbm_frac": round(tot_b / tot_t / 1e6 / 8000, 3),
                      "plan_hbm_frac": round(tot_b / tot_p / 1e6 / 8000, 3)}), flush=True)
    f.close()
    ctx.close()


if __name__ == "__main__":
    main()
