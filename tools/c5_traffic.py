"""HBM traffic of BASELINE C5's kernels against their algorithmic bytes (profiles/r03_c5_traffic.json).

Two sources, each a pair of separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE):
  * per column: `tools/c5_columns.py --mark` (every column decoded alone, a torch kernel before each
    column segments the trace; the column's own JSON line gives its algorithmic bytes = compressed
    buffers read + canonical bytes written);  traffic per step = the column's counter sum / its steps;
  * the batched 8-GPU shard: `bench.py --workloads c5 --simulate-world 8` (FSST pre-pass, FSST decode,
    K1g) -- K1g's algorithmic bytes = the shard's minus l_comment's (c5_columns --world 8).
Correction (MI355X_MICROARCH.md §HBM): bytes = (2 * FETCH_SIZE + WRITE_SIZE) KiB x 1024.
  python tools/c5_traffic.py --cols-fetch D --cols-write D --cols-json F [--shard-fetch D --shard-write D
                             --shard-json F --cols8-json F --shard-steps S] --out profiles/r03_c5_traffic.json
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path


def dispatches(d: Path, counter: str):
    """[(dispatch_id, kernel, value)] in dispatch order (rows of one dispatch summed)."""
    acc = defaultdict(float)
    name = {}
    for f in sorted(Path(d).rglob("*counter_collection.csv")):
        with f.open() as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                k = int(r["Dispatch_Id"])
                acc[k] += float(r["Counter_Value"])
                name[k] = r["Kernel_Name"]
    return [(k, name[k], acc[k]) for k in sorted(acc)]


def segments(ds, marker="elementwise"):
    """Split dispatches at marker kernels: list of [(kernel, value)] per column."""
    segs, cur = [], None
    for _, k, v in ds:
        if marker in k:
            cur = []
            segs.append(cur)
        elif cur is not None:
            cur.append((k, v))
    return [g for g in segs if g]  # (torch's own fill kernels also match: empty segments dropped)


def short(k: str) -> str:
    return k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cols-fetch", required=True)
    ap.add_argument("--cols-write", required=True)
    ap.add_argument("--cols-json", required=True)
    ap.add_argument("--cols-reps", type=int, default=3, help="c5_columns --reps of the PMC runs")
    ap.add_argument("--shard-fetch")
    ap.add_argument("--shard-write")
    ap.add_argument("--shard-json")
    ap.add_argument("--cols8-json")
    ap.add_argument("--shard-steps", type=int, default=0, help="plan replays in the shard PMC run")
    ap.add_argument("--out", default="profiles/r03_c5_traffic.json")
    a = ap.parse_args()
    cols = [json.loads(x) for x in Path(a.cols_json).read_text().splitlines() if x.strip().startswith("{")]
    cols = [c for c in cols if not c["column"].startswith("SUM")]
    fseg = segments(dispatches(Path(a.cols_fetch), "FETCH_SIZE"))
    wseg = segments(dispatches(Path(a.cols_write), "WRITE_SIZE"))
    if len(fseg) != len(cols) or len(wseg) != len(cols):
        raise SystemExit(f"{len(cols)} columns but {len(fseg)} / {len(wseg)} marked segments")
    # direct steps + plan replays (warm-ups included) + the plan's selection replays (2 candidates
    # x (1 warm-up + 3 timed), capi.hip vxg_plan_create)
    steps = 2 * (3 + a.cols_reps) + 8
    out = {"correction": "bytes = (2 * FETCH_SIZE + WRITE_SIZE) KiB * 1024 (gfx950, MI355X_MICROARCH.md §HBM)",
           "columns": []}
    for c, fs, ws in zip(cols, fseg, wseg):
        per = defaultdict(lambda: [0.0, 0.0, 0])
        for k, v in fs:
            per[short(k)][0] += v
            per[short(k)][2] += 1
        for k, v in ws:
            per[short(k)][1] += v
        traffic = sum((2 * f + w) * 1024 for f, w, _ in per.values()) / steps
        alg = c["read_bytes"] + c["write_bytes"]
        out["columns"].append({
            "column": c["column"], "algorithmic_bytes": alg, "traffic_bytes_per_step": round(traffic),
            "traffic_over_algorithmic": round(traffic / alg, 4),
            "kernels": {k: {"dispatches_per_step": round(n / steps, 2),
                            "traffic_bytes_per_step": round((2 * f + w) * 1024 / steps)}
                        for k, (f, w, n) in sorted(per.items(), key=lambda kv: -(2 * kv[1][0] + kv[1][1]))}})
    tot_a = sum(c["algorithmic_bytes"] for c in out["columns"])
    tot_t = sum(c["traffic_bytes_per_step"] for c in out["columns"])
    out["columns_total"] = {"algorithmic_bytes": tot_a, "traffic_bytes_per_step": tot_t,
                            "traffic_over_algorithmic": round(tot_t / tot_a, 4)}
    if a.shard_fetch and a.shard_steps:
        f = dispatches(Path(a.shard_fetch), "FETCH_SIZE")
        w = dispatches(Path(a.shard_write), "WRITE_SIZE")
        per = defaultdict(lambda: [0.0, 0.0, 0])
        for _, k, v in f:
            per[short(k)][0] += v
            per[short(k)][2] += 1
        for _, k, v in w:
            per[short(k)][1] += v
        sh = json.loads(Path(a.shard_json).read_text().strip().splitlines()[-1])["encodings"]["C5"]
        c8 = {json.loads(x)["column"]: json.loads(x) for x in Path(a.cols8_json).read_text().splitlines()
              if x.strip().startswith("{")}
        lc = c8["l_comment"]
        fsst_alg = lc["read_bytes"] + lc["write_bytes"]
        shard_alg = sh["read_bytes"] + sh["write_bytes"]
        kern = {}
        for k, (fv, wv, n) in per.items():
            if "elementwise" in k or "rocclr" in k or "sum_kernel" in k:
                continue
            kern[k] = {"launches": n, "traffic_bytes_per_launch": round((2 * fv + wv) * 1024 / max(n, 1))}
        fsst_t = sum(v["traffic_bytes_per_launch"] for k, v in kern.items() if "fsst" in k)
        k1g_t = sum(v["traffic_bytes_per_launch"] for k, v in kern.items() if "k1_generic" in k)
        out["shard8"] = {"kernels": kern, "shard_algorithmic_bytes": shard_alg,
                         "fsst_algorithmic_bytes": fsst_alg, "fsst_traffic_bytes": fsst_t,
                         "fsst_traffic_over_algorithmic": round(fsst_t / fsst_alg, 4),
                         "k1g_algorithmic_bytes": shard_alg - fsst_alg, "k1g_traffic_bytes": k1g_t,
                         "k1g_traffic_over_algorithmic": round(k1g_t / (shard_alg - fsst_alg), 4)}
    Path(a.out).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps({k: v for k, v in out.items() if k != "columns"}, indent=1))
    for c in out["columns"]:
        print(f"{c['column']:18s} alg {c['algorithmic_bytes'] / 1e6:8.2f} MB traffic {c['traffic_bytes_per_step'] / 1e6:8.2f} MB "
              f"ratio {c['traffic_over_algorithmic']:.3f}  top {next(iter(c['kernels']))}")


if __name__ == "__main__":
    main()
