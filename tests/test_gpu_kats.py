"""GPU replay of the reference's known-answer tests (tests/golden/kat.json).

Each KAT the oracle is checked against in tests/test_oracle.py is rebuilt here as the same array
tree, moved to HBM and run through the C ABI: vxg_canonicalize for decodes and slices,
vxg_take_array for take on the compressed (possibly sliced) BitPacked array.  The expected values
are the reference's literals, and every output byte is also compared with the oracle's.
"""
import json
import struct
from pathlib import Path

import numpy as np
import pytest

import vortex_amd.arrays as A
import vortex_amd.encode as E
from oracle_tree import canon, slice_any, view_bytes

pytestmark = pytest.mark.gpu

KATS = {k["name"]: k for k in json.loads((Path(__file__).resolve().parent / "golden" / "kat.json").read_text())}


def _dev():
    import torch
    return torch.device("cuda", 0)


def _gen(k):
    i = np.arange(k["n"], dtype=np.int64)
    return eval(k["gen"], {"i": i}).astype(A.NP_OF_PTYPE[k["ptype"]])  # literal from kat.json


def _gpu(arr, ctx):
    return A.canonicalize(arr.to(_dev()), ctx)


@pytest.mark.parametrize("name", ["bitpacked_take_indices", "bitpacked_take_sliced_indices",
                                  "bitpacked_take_after_slice"])
def test_kat_take_on_compressed_bitpacked(ctx, name):
    """bitpacking/compute/take.rs:227-255, slice.rs:182-206: take on the packed array (sliced by
    metadata where the KAT slices) without canonicalizing it first."""
    k = KATS[name]
    arr = E.encode_bitpacked(_gen(k), bit_width=k["bit_width"])
    if "slice" in k:
        arr = slice_any(arr, *k["slice"])
    idx = np.array(k["indices"], dtype=np.int64)
    got = A.take(arr.to(_dev()), idx, ctx).numpy()
    assert got.tolist() == k["expect_taken"]
    assert got.tobytes() == canon(arr)[0][idx].tobytes()
    # and through the full canonical of the sliced tree
    full = _gpu(arr, ctx).numpy()
    assert full[idx].tolist() == k["expect_taken"]


@pytest.mark.parametrize("case", [c["test"] for c in KATS["bitpacked_slices"]["cases"]])
def test_kat_bitpacked_slices_on_gpu(ctx, case):
    """bitpacking/compute/slice.rs:54-180: the sliced (and doubly sliced) BitPacked arrays
    canonicalize to the reference's scalar_at values, offset and length."""
    k = next(c for c in KATS["bitpacked_slices"]["cases"] if c["test"] == case)
    vals = _gen(k)
    arr = E.encode_bitpacked(vals, bit_width=k["bit_width"])
    for s in k["slices"]:
        arr = slice_any(arr, *s)
    assert arr.len == k["expect_len"]
    if "expect_offset" in k:
        assert arr.meta["offset"] == k["expect_offset"]
    if "expect_has_patches" in k:
        assert arr.meta["has_patches"] == k["expect_has_patches"]
    got = _gpu(arr, ctx).numpy()
    assert got.tobytes() == canon(arr)[0].tobytes()
    for i, v in k.get("expect_at", []):
        assert int(got[i]) == v
    lo = sum(s[0] for s in k["slices"])
    assert np.array_equal(got, vals[lo: lo + arr.len])


def test_kat_alp_nullable_patched_on_gpu(ctx):
    """alp/compress.rs:167-192: nullable f64 with a patch, e16/f13; the valid rows decode to the
    literal values and the null row stays null."""
    k = KATS["alp_f64_nullable_patched"]
    vals = np.array([struct.unpack("<d", bytes.fromhex(h))[0] for h in k["values_bits"]])
    valid = np.array(k["validity"])
    e, f, enc, idx, pv = E.alp_encode(vals)
    assert (e, f) == (k["expect_e"], k["expect_f"]) and idx.size > 0
    for child in (A.primitive(enc, validity=valid),):
        arr = A.alp(child, e, f, A.sparse(A.primitive(idx), A.primitive(pv, validity="ALL_VALID"), vals.size))
        res = _gpu(arr, ctx)
        got = res.numpy()
        assert res.validity_mask().tolist() == k["validity"]
        assert [struct.pack("<d", x).hex() for x in got[valid]] == k["expect_valid_decoded_bits"]
        ref, rvalid = canon(arr)
        assert got.tobytes() == ref.tobytes() and rvalid.tolist() == k["validity"]


def test_kat_dict_nullable_on_gpu(ctx):
    """dict/compress.rs:211-282: nullable primitive and VarBin dictionaries (slot 0 = the null
    entry, null rows coded 0) canonicalize to the original values with their nulls."""
    k = KATS["dict_encode_primitive_nulls"]
    for bitpack in (True, False):
        arr = E.encode_dict_nullable(np.array(k["values"], np.int32), k["validity"], bitpack_codes=bitpack)
        res = _gpu(arr, ctx)
        got = res.numpy()
        assert res.validity_mask().tolist() == k["validity"]
        assert [int(x) for x, ok in zip(got, k["validity"]) if ok] == \
            [v for v, ok in zip(k["values"], k["validity"]) if ok]
        ref, _ = canon(arr)
        assert got.tobytes() == ref.tobytes()
    k = KATS["dict_encode_varbin_nulls"]
    strs = [None if s is None else s.encode() for s in k["strings"]]
    arr = E.encode_dict_strings_nullable(strs)
    res = _gpu(arr, ctx)
    views, _ = res.numpy()
    heap = res.buffers()
    assert res.validity_mask().tolist() == [s is not None for s in strs]
    assert [view_bytes(views, heap, i) if s is not None else None for i, s in enumerate(strs)] == strs
    (rv, rh), _ = canon(arr)
    assert views.tobytes() == rv.tobytes()
