"""Per-phase cycle split of the FSST decode kernel (profiling build, -DVXG_FSST_STAMPS).

  make -C vortex_amd/csrc stamps
  VXG_GPU_LIB=vortex_amd/libvortex_gpu_stamps.so python tools/fsst_stamps.py [--workload c4|l_comment]

Runs the C4 column (or C5's l_comment) through a plan `reps` times and prints, per decode
workgroup, the mean s_memtime ticks thread 0 spent in each phase of the staged path (phases
end at workgroup barriers, so they include the wait for the slowest wave), plus the kernel's
event time for scale.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

PHASES = ["prologue+length scan", "code staging+zero image", "pass1+segment scan", "pass2 image ORs",
          "copy-out+views"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    if "stamps" not in os.environ.get("VXG_GPU_LIB", ""):
        sys.exit("set VXG_GPU_LIB to the stamps build (make -C vortex_amd/csrc stamps)")
    import numpy as np
    import torch
    import bench
    import vortex_amd as V
    import vortex_amd.arrays as A
    ctx = V.Context(0)
    fn = ctx.lib.vxg_debug_fsst_stamps
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int]
    rng = np.random.default_rng(0)
    if a.workload == "c4":
        arr, _ = bench.make_c4(rng, 1, 0)
        node_arr = arr.to(torch.device("cuda", 0))
        plan = A.Plan([node_arr], ctx)
    else:
        from vortex_amd.file import DeviceColumns, VortexFile
        host = torch.from_numpy(bench.c5_file(None, 0)).pin_memory()
        f = VortexFile(host)
        ci = [c.name for c in f.columns].index("l_comment")
        dc = DeviceColumns(f, ctx, [ci], 0, f.columns[ci].n_chunks)
        plan = A.Plan(dc.nodes, ctx)
    for _ in range(3):
        plan.launch()
    ctx.sync()
    fn(None, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        plan.launch()
    e1.record()
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 16)()
    fn(buf, 0)
    wgs = buf[15]
    out = {"workload": a.workload, "step_ms": round(e0.elapsed_time(e1) / a.reps, 4), "workgroups": wgs // a.reps,
           "ticks_per_wg": {p: round(buf[i] / max(wgs, 1), 1) for i, p in enumerate(PHASES)}}
    tot = sum(out["ticks_per_wg"].values())
    out["share"] = {p: round(v / tot, 3) for p, v in out["ticks_per_wg"].items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
