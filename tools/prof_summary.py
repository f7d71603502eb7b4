"""Summarise a rocprofv3 kernel trace (run_kernel_trace.csv) per kernel: all dispatches, and the
steady state after the first `--skip` dispatches of each kernel (bench warmup), so the average
duration can be compared with bench.py's live HIP-event measurement of the timed region.
Optionally summarise SQ PMC counters (run_counter_collection.csv) per kernel.

  python tools/prof_summary.py --trace gpurun_out/prof_r01d --skip 5 [--pmc gpurun_out/pmc_sq_r01d]
"""
from __future__ import annotations

import argparse
import collections
import csv
from pathlib import Path


def short(name: str) -> str:
    return name.replace("(anonymous namespace)::", "").split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--skip", type=int, default=5)
    ap.add_argument("--pmc", default=None)
    a = ap.parse_args()
    f = next(Path(a.trace).rglob("*kernel_trace.csv"))
    per = collections.defaultdict(list)
    with f.open() as fh:
        rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Start_Timestamp"]))
    for r in rows:
        per[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    print(f"{'kernel':90s} {'calls':>5s} {'avg_us':>9s} {'steady_avg_us':>13s} {'steady_min_us':>13s}")
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        st = v[a.skip:] if len(v) > a.skip else v
        print(f"{k:90s} {len(v):5d} {sum(v) / len(v):9.2f} {sum(st) / len(st):13.2f} {min(st):13.2f}")
    if a.pmc:
        g = next(Path(a.pmc).rglob("*counter_collection.csv"))
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        with g.open() as fh:
            for r in csv.DictReader(fh):
                acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print("\nPMC (mean per dispatch)")
        for k, cs in acc.items():
            print(k)
            for c, v in sorted(cs.items()):
                print(f"    {c:24s} {sum(v) / len(v):16.1f}")
            if "SQ_WAVES" in cs and "SQ_INSTS_VALU" in cs:
                w = sum(cs["SQ_WAVES"]) / len(cs["SQ_WAVES"])
                print(f"    {'VALU instr per wave':24s} {sum(cs['SQ_INSTS_VALU']) / len(cs['SQ_INSTS_VALU']) / w:16.1f}")


if __name__ == "__main__":
    main()
