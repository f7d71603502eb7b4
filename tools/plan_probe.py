"""Diagnostic: is a C5 step bound by host-side submission or by the device?

Builds C5 (this GPU's whole lineitem table), records it as a vxg_plan, and reports
  * host time of vxg_plan_launch alone (no sync), per call,
  * device time per replay (HIP events around back-to-back replays),
Run on the GPU box: python tools/plan_probe.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    import vortex_amd as V
    import vortex_amd.arrays as A

    world = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    ctx = V.Context(0)
    (_, host, c0, c1), info = bench.make_c5(np.random.default_rng(42), world, 0)
    wl = bench.FileWorkload(host, ctx, c0, c1)  # C5 as bench runs it: reader-built trees, one plan
    plan = wl.plans[0]
    for _ in range(5):
        plan.launch()
    ctx.sync()
    n = 100
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dev_us, host_us = [], []
    for trial in range(5):
        host = []
        torch.cuda.synchronize()
        e0.record()
        for _ in range(n):
            t = time.perf_counter()
            plan.launch()
            host.append(time.perf_counter() - t)
        e1.record()
        torch.cuda.synchronize()
        dev_us.append(e0.elapsed_time(e1) / n * 1e3)
        host_us.append(np.median(host) * 1e6)
    print(f"plan[{os.environ.get('VXG_GPU_LIB', 'in-tree')}] world={world}: host launch {min(host_us):.1f} us, "
          f"device us/replay min {min(dev_us):.1f} median {np.median(dev_us):.1f}")
    wl.close()


if __name__ == "__main__":
    main()
