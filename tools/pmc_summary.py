"""Per-kernel summary of rocprofv3 --pmc counter CSVs (one or more pass directories).

  python tools/pmc_summary.py gpurun_out/pmc_r02g_a gpurun_out/pmc_r02g_b ... [--kernel substr]

For every kernel (or the ones matching --kernel) prints the per-dispatch mean of each counter and
the derived rates: instructions per wave, wave-cycle split (SQ_WAVE_CYCLES and the WAIT/ACTIVE
counters count quad-cycles, MI355X_MICROARCH.md), LDS bank-conflict share and HBM bytes per
dispatch ((2 * FETCH_SIZE + WRITE_SIZE) KiB, the gfx950 correction of tools/pmc_traffic.py).
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path


def load(dirs):
    # (kernel, counter) -> list of per-dispatch values (summed over the dispatch's rows)
    per = defaultdict(lambda: defaultdict(float))
    for d in dirs:
        for f in sorted(Path(d).rglob("*counter_collection.csv")):
            with f.open() as fh:
                for row in csv.DictReader(fh):
                    key = (row["Kernel_Name"], row["Counter_Name"], f.parent.name, row.get("Dispatch_Id", ""))
                    per[key[:2]][key[2:]] += float(row["Counter_Value"])
    out = defaultdict(dict)
    for (k, c), disp in per.items():
        vals = list(disp.values())
        out[k][c] = (sum(vals) / len(vals), len(vals))
    return out


def derive(c):
    g = lambda k: c.get(k, (None, 0))[0]
    d = {}
    waves = g("SQ_WAVES")
    if waves:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if g(k) is not None:
                d[k.replace("SQ_INSTS_", "") + "_per_wave"] = round(g(k) / waves, 1)
    wc = g("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS"):
            if g(k) is not None:
                d[k.replace("SQ_", "").lower() + "_frac"] = round(g(k) / wc, 3)
        if waves:
            d["wave_cycles_per_wave"] = round(4 * wc / waves)
    if g("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_frac"] = round((g("SQ_LDS_BANK_CONFLICT") or 0) / g("SQ_LDS_IDX_ACTIVE"), 3)
    if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
        d["hbm_bytes"] = round((2 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    data = load(a.dirs)
    res = {}
    for k, c in sorted(data.items()):
        if a.kernel not in k:
            continue
        res[k] = {"counters": {n: round(v, 1) for n, (v, _) in sorted(c.items())},
                  "dispatches": max(n for _, n in c.values()), "derived": derive(c)}
    if a.json:
        print(json.dumps(res, indent=1))
    else:
        for k, r in res.items():
            print(k[:150])
            print("   ", r["dispatches"], "dispatches", r["derived"])


if __name__ == "__main__":
    main()
