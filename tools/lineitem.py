"""Synthetic TPC-H lineitem, compressed the way bench-vortex writes it (BASELINE config C5).

dbgen cannot run offline (bench-vortex/src/tpch/dbgen.rs downloads it), so the 16 columns of
bench-vortex/src/tpch/schema.rs:67-84 are generated with TPC-H's value domains at SF1's row
count (6 001 215), rechunked to 64 Ki-row chunks (tpch/mod.rs:38-40, 276-286), and every chunk
is compressed with the cascade the sampling compressor picks for that column's data
(vortex-sampling-compressor/src/compressors/*):
  l_orderkey                 RunEnd (sorted, 1-7 lines per order; ends BitPacked, values FoR/BitPacked)
  l_partkey/suppkey/linenumber   FoR -> BitPacked (i64)
  l_quantity/extendedprice/discount/tax   ALP -> FoR -> BitPacked (f64)
  l_shipdate/commitdate/receiptdate       FoR -> BitPacked (Date32 storage i32)
  l_returnflag/linestatus/shipinstruct/shipmode   Dict(VarBin values, BitPacked codes)
  l_comment                  FSST (per-chunk symbol table; codes VarBin, FoR/BitPacked children)
Chunk c is generated from seed (seed, c), so every rank builds just its own chunk range and all
ranks agree on the table without communicating.
"""
from __future__ import annotations

import numpy as np

SF1_ROWS = 6_001_215
CHUNK_ROWS = 64 * 1024

COLUMNS = [("l_orderkey", "i64"), ("l_partkey", "i64"), ("l_suppkey", "i64"), ("l_linenumber", "i64"),
           ("l_quantity", "f64"), ("l_extendedprice", "f64"), ("l_discount", "f64"), ("l_tax", "f64"),
           ("l_returnflag", "utf8"), ("l_linestatus", "utf8"), ("l_shipdate", "i32"), ("l_commitdate", "i32"),
           ("l_receiptdate", "i32"), ("l_shipinstruct", "utf8"), ("l_shipmode", "utf8"), ("l_comment", "utf8")]

DATE_COLUMNS = ("l_shipdate", "l_commitdate", "l_receiptdate")  # Date32 -> vortex.date extension
RETURNFLAG = [b"A", b"N", b"R"]
LINESTATUS = [b"F", b"O"]
SHIPINSTRUCT = [b"DELIVER IN PERSON", b"COLLECT COD", b"NONE", b"TAKE BACK RETURN"]
SHIPMODE = [b"REG AIR", b"AIR", b"RAIL", b"SHIP", b"TRUCK", b"MAIL", b"FOB"]
# dbgen's text grammar draws from a few hundred words; a subset is enough for FSST's tables
WORDS = (b"furiously regular deposits sleep carefully final accounts ironic packages blithely "
         b"quickly express requests pending theodolites slyly even instructions bold foxes "
         b"unusual asymptotes special platelets silent pinto beans fluffily careful dependencies "
         b"daring ideas close courts blithe dolphins quiet excuses ruthless warthogs across "
         b"about according after against along alongside among around at atop above haggle "
         b"nag wake cajole use detect integrate maintain nod was lose boost affix").split()
STARTDATE = 8035  # 1992-01-01 as days since the epoch


def n_chunks(rows: int = SF1_ROWS, chunk_rows: int = CHUNK_ROWS) -> int:
    return (rows + chunk_rows - 1) // chunk_rows


def chunk_values(c: int, rows: int = SF1_ROWS, chunk_rows: int = CHUNK_ROWS, seed: int = 7) -> dict:
    """Plain values of chunk c: {column: ndarray | list[bytes]}."""
    rng = np.random.default_rng([seed, c])
    n = min(chunk_rows, rows - c * chunk_rows)
    # orders of 1-7 lines; keys increase by 1-4 (dbgen's sparse keys), disjoint per chunk
    runs = rng.integers(1, 8, n)
    starts = np.cumsum(runs) - runs
    runs = runs[starts < n]
    k = runs.size
    order_of_row = np.repeat(np.arange(k), runs)[:n]
    okeys = c * 262_144 + 1 + np.cumsum(rng.integers(1, 5, k)) - 1
    linenumber = (np.arange(n) - np.repeat(np.cumsum(runs) - runs, runs)[:n]) + 1
    orderdate = STARTDATE + rng.integers(0, 2406, k)
    od = orderdate[order_of_row]
    ship = od + rng.integers(1, 122, n)
    commit = od + rng.integers(30, 91, n)
    receipt = ship + rng.integers(1, 31, n)
    qty = rng.integers(1, 51, n)
    partkey = rng.integers(1, 200_001, n)
    retail = (90_000 + (partkey // 10) % 20_001 + 100 * (partkey % 1_000)) / 100.0
    ext = np.round(qty * retail, 2)
    lens = rng.integers(10, 44, n)
    wl = np.array([len(w) + 1 for w in WORDS])
    total = int(lens.sum())
    ids = rng.integers(0, len(WORDS), int(total / wl.mean() * 1.2) + 16)
    stream = b" ".join(WORDS[i] for i in ids)
    offs = np.concatenate([[0], np.cumsum(lens)])
    comment = [stream[offs[i]: offs[i + 1]] for i in range(n)]
    rf = rng.integers(0, 3, n)
    return {
        "l_orderkey": okeys[order_of_row].astype(np.int64),
        "l_partkey": partkey.astype(np.int64),
        "l_suppkey": rng.integers(1, 10_001, n).astype(np.int64),
        "l_linenumber": linenumber.astype(np.int64),
        "l_quantity": qty.astype(np.float64),
        "l_extendedprice": ext,
        "l_discount": rng.integers(0, 11, n) / 100.0,
        "l_tax": rng.integers(0, 9, n) / 100.0,
        "l_returnflag": [RETURNFLAG[i] for i in rf],
        "l_linestatus": [LINESTATUS[i] for i in (ship > STARTDATE + 1260).astype(np.int64)],
        "l_shipdate": ship.astype(np.int32),
        "l_commitdate": commit.astype(np.int32),
        "l_receiptdate": receipt.astype(np.int32),
        "l_shipinstruct": [SHIPINSTRUCT[i] for i in rng.integers(0, 4, n)],
        "l_shipmode": [SHIPMODE[i] for i in rng.integers(0, 7, n)],
        "l_comment": comment,
    }


def encode_column(name: str, v):
    """The sampling compressor's cascade for one chunk of one column."""
    import vortex_amd.encode as E
    if name == "l_orderkey":
        return E.encode_runend(v, compress_values=True)
    if name in ("l_partkey", "l_suppkey", "l_linenumber", "l_shipdate", "l_commitdate", "l_receiptdate"):
        return E.encode_for_bitpacked(v)
    if name in ("l_quantity", "l_extendedprice", "l_discount", "l_tax"):
        return E.encode_alp(v)
    if name == "l_comment":
        heap = np.frombuffer(b"".join(v), dtype=np.uint8).copy()
        offs = np.concatenate([[0], np.cumsum([len(s) for s in v])]).astype(np.int64)
        return E.encode_fsst_from_heap(heap, offs)
    return E.encode_dict_strings(v)


def lineitem_columns(chunk_ids, rows: int = SF1_ROWS, chunk_rows: int = CHUNK_ROWS, seed: int = 7):
    """-> ({column: ChunkedArray of the given chunks}, {column: [plain values per chunk]})."""
    import vortex_amd.arrays as A
    enc = {name: [] for name, _ in COLUMNS}
    plain = {name: [] for name, _ in COLUMNS}
    for c in chunk_ids:
        vals = chunk_values(c, rows, chunk_rows, seed)
        for name, _ in COLUMNS:
            enc[name].append(encode_column(name, vals[name]))
            plain[name].append(vals[name])
    return {k: A.chunked(v) for k, v in enc.items()}, plain


def canonical_bytes(values) -> int:
    """Bytes of the canonical Arrow output of one chunk's plain values (strings: 16-byte views
    + the data buffer bytes a canonical VarBinView holds)."""
    if isinstance(values, list):
        return 16 * len(values) + sum(len(s) for s in values)
    return values.nbytes
