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
    ap.add_argument("--ablate", default="", help="comma list of ablation masks to time (output wrong)")
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
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_uint64, C.c_int]
    rng = np.random.default_rng(0)
    if a.workload == "c4":
        arr, _ = bench.make_c4(rng, 1, 0)
        plan = A.Plan([arr.to(torch.device("cuda", 0))], ctx)
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        plan.launch()
    e1.record()
    torch.cuda.synchronize()
    if a.ablate:
        ab = ctx.lib.vxg_debug_fsst_ablate
        ab.restype, ab.argtypes = C.c_int, [C.c_uint32]
        res = {}
        for mask in [int(x) for x in a.ablate.split(",")]:
            ab(mask)
            for _ in range(3):
                plan.launch()
            ctx.sync()
            e0.record()
            for _ in range(a.reps):
                plan.launch()
            e1.record()
            torch.cuda.synchronize()
            res[mask] = round(e0.elapsed_time(e1) / a.reps, 4)
        ab(0)
        print(json.dumps({"workload": a.workload, "ablation_step_ms": res,
                          "bits": "1=pass2 2=pass1+scan 4=views 8=copy-out 16=code loads"}), flush=True)
    n = 1 << 18
    rec = np.zeros((n, 8), np.uint64)
    fn(fn.argtypes[0](rec.ctypes.data), n, 1)  # the last replay's records, then reset
    plan.launch()
    ctx.sync()
    fn(fn.argtypes[0](rec.ctypes.data), n, 0)  # one clean replay
    r = rec[rec[:, 7] == 1].astype(np.int64)
    d = np.diff(r[:, :6], axis=1)
    dur = r[:, 5] - r[:, 0]
    span = int(r[:, 5].max() - r[:, 0].min())
    out = {"workload": a.workload, "step_ms_stamped": round(e0.elapsed_time(e1) / a.reps, 4),
           "staged_workgroups": int(r.shape[0]), "span_ticks": span,
           "mean_wg_ticks": round(float(dur.mean()), 1), "concurrency": round(float(dur.sum()) / max(span, 1), 1),
           "phase_mean_ticks": {p: round(float(d[:, k].mean()), 1) for k, p in enumerate(PHASES)},
           "phase_median_ticks": {p: int(np.median(d[:, k])) for k, p in enumerate(PHASES)}}
    out["share"] = {p: round(float(d[:, k].sum() / dur.sum()), 3) for k, p in enumerate(PHASES)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
