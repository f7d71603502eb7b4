"""Turn rocprofv3 PMC counter CSVs into per-launch HBM traffic (profiles/pmc_traffic.json).

Usage:
  python tools/pmc_traffic.py --fetch <dir with FETCH_SIZE counter_collection.csv>
                              --write <dir with WRITE_SIZE counter_collection.csv>
                              --kernel-substr fl_unpack_kernelILi32ELi7E --name fl_unpack_u32_w7
Correction (MI355X_MICROARCH.md §HBM; cdna_hip_programming.md §7): FETCH_SIZE and WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reports half of the bytes of a wide coalesced streaming read, so
  hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
FETCH_SIZE and WRITE_SIZE are collected in separate --pmc passes (they do not fit one pass).
"""
from __future__ import annotations

import argparse
import csv
import json
from pathlib import Path


def counters(d: Path, counter: str, substr: str, max_grid: bool = False) -> list[float]:
    """Per-dispatch values of `counter` for kernels matching `substr`; max_grid keeps only the
    dispatches of the largest grid (the full-size workload, not the smaller launches of other
    configs -- plan measurements, C5 chunks -- that match the same kernel name)."""
    rows = []
    for f in sorted(d.rglob("*counter_collection.csv")):
        with f.open() as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter and substr in row.get("Kernel_Name", ""):
                    rows.append(row)
    if max_grid and rows:
        g = max(int(r.get("Grid_Size") or 0) for r in rows)
        rows = [r for r in rows if int(r.get("Grid_Size") or 0) == g]
    return [float(r["Counter_Value"]) for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel-substr", required=True)
    ap.add_argument("--name", required=True)
    ap.add_argument("--algorithmic-bytes", type=float, default=None)
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--max-grid", action="store_true", help="only the largest-grid dispatches")
    a = ap.parse_args()
    fetch = counters(Path(a.fetch), "FETCH_SIZE", a.kernel_substr, a.max_grid)
    write = counters(Path(a.write), "WRITE_SIZE", a.kernel_substr, a.max_grid)
    if not fetch or not write:
        raise SystemExit(f"no samples (fetch={len(fetch)}, write={len(write)})")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    rec = {"kernel_substr": a.kernel_substr, "launches_fetch": len(fetch), "launches_write": len(write),
           "FETCH_SIZE_KiB_mean": f_kib, "WRITE_SIZE_KiB_mean": w_kib,
           "read_bytes_corrected": 2 * f_kib * 1024, "write_bytes": w_kib * 1024,
           "hbm_bytes_per_launch": (2 * f_kib + w_kib) * 1024,
           "correction": "gfx950 FETCH_SIZE x2 (MI355X_MICROARCH.md §HBM); KiB -> bytes",
           "dispatches": "largest grid only" if a.max_grid else "all matching"}
    if a.algorithmic_bytes:
        rec["algorithmic_bytes"] = a.algorithmic_bytes
        rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_launch"] / a.algorithmic_bytes
    out = Path(a.out)
    d = json.loads(out.read_text()) if out.exists() else {}
    d[a.name] = rec
    out.write_text(json.dumps(d, indent=1) + "\n")
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
