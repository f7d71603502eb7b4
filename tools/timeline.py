"""Timeline of a rocprofv3 kernel trace: for the last K replays of a repeated step (split at
gaps longer than --gap us), report per replay the wall span, the union of kernel busy time,
the sum of kernel durations (concurrency = sum / union) and the idle time inside the span, and
the kernels on the replay's critical path candidates (longest first).
Usage: python tools/timeline.py <run_kernel_trace.csv> [--gap 50] [--last 3] [--min-kernels 5]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap", type=float, default=50.0)
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--min-kernels", type=int, default=5)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3, r["Kernel_Name"],
                  int(r["Grid_Size_X"])) for r in rows), key=lambda k: k[0])
    groups, cur, end = [], [], None
    for k in ks:
        if cur and k[0] - end > a.gap:
            groups.append(cur)
            cur = []
        cur.append(k)
        end = max(end, k[1]) if end is not None and cur[:-1] else k[1]
    if cur:
        groups.append(cur)
    groups = [g for g in groups if len(g) >= a.min_kernels]
    for g in groups[-a.last:]:
        t0 = min(k[0] for k in g)
        t1 = max(k[1] for k in g)
        iv = sorted((k[0], k[1]) for k in g)
        busy, s, e = 0.0, None, None
        for x, y in iv:
            if s is None or x > e:
                if s is not None:
                    busy += e - s
                s, e = x, y
            else:
                e = max(e, y)
        busy += e - s
        tot = sum(k[1] - k[0] for k in g)
        print(f"replay: {len(g)} kernels span {t1 - t0:8.1f} us busy(union) {busy:8.1f} us "
              f"sum {tot:8.1f} us concurrency {tot / busy:4.2f} idle {t1 - t0 - busy:6.1f} us")
        agg = defaultdict(lambda: [0, 0.0])
        for k in g:
            short = k[2].split("(")[0][:90]
            agg[short][0] += 1
            agg[short][1] += k[1] - k[0]
        for name, (n, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
            print(f"   {n:3d} x {d / n:7.2f} us = {d:8.1f} us  {name}")
        for k in sorted(g, key=lambda k: k[0]):
            print(f"      +{k[0] - t0:7.1f} .. +{k[1] - t0:7.1f} ({k[1] - k[0]:6.1f}) grid {k[3]:>8} {k[2].split('(')[0][:80]}")


if __name__ == "__main__":
    main()
