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
from vortex_amd._lib import VortexGpuError

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


# ---------------------------------------------------------------- round 5: slices, nulls, take
def _apply_slices(arr, slices):
    """First slice = SliceFn::slice as the KAT calls it (no bounds check), then compute::slice."""
    from oracle_tree import slice_checked
    for j, s in enumerate(slices):
        arr = (slice_any if j == 0 else slice_checked)(arr, *s)
    return arr


@pytest.mark.parametrize("bitpack", [False, True], ids=["primitive_deltas", "bitpacked_deltas"])
@pytest.mark.parametrize("case", [c["test"] for c in KATS["delta_slices"]["cases"]])
def test_kat_delta_slices_on_gpu(ctx, case, bitpack):
    """delta/compute.rs:162-405: jagged (remainder chunk with one scalar base) and non-jagged
    arrays, empty slices, slices inside / across 1024-value chunks and slices of slices,
    canonicalized by the engine from the sliced metadata (offset, partial bases/deltas).  The
    reference keeps the deltas plain; the BitPacked-deltas variant sends the same slices
    through the fused K1 -> K3 path."""
    k = next(c for c in KATS["delta_slices"]["cases"] if c["test"] == case)
    arr = _apply_slices(E.encode_delta(np.arange(k["n"], dtype=np.uint32), bitpack_deltas=bitpack), k["slices"])
    lo, hi = k["expect"]
    got = _gpu(arr, ctx).numpy()
    assert got.tolist() == list(range(lo, hi))
    assert got.tobytes() == canon(arr)[0].tobytes()


def _ree(b, ends_ptype="u64"):
    if "values" in b:
        ends, rv = E.runend_encode(np.array(b["values"], np.int32))
        ends = ends.astype(A.NP_OF_PTYPE[ends_ptype])
    else:
        ends = np.array(b["ends"], A.NP_OF_PTYPE[ends_ptype])
        rv = np.array(b["run_values"], np.int32)
    vv, validity = b.get("values_validity"), b.get("validity")
    if validity is not None and vv is None:
        vv = "ALL_VALID"
    return A.run_end(A.primitive(ends), A.primitive(rv, validity=vv), validity=validity)


def _masked(vals, valid):
    return [None if (valid is not None and not ok) else int(v)
            for v, ok in zip(vals, valid if valid is not None else [True] * len(vals))]


def test_kat_runend_nullable_on_gpu(ctx):
    """runend/compress.rs:180-210 decode_nullable: values and the validity bitmap."""
    k = KATS["runend_decode_nullable"]
    arr = _ree(dict(ends=k["ends"], run_values=k["run_values"], values_validity=k["values_validity"],
                    validity=k["validity"]), k["ends_ptype"])
    res = _gpu(arr, ctx)
    assert res.numpy().tolist() == k["expect_decoded"]
    assert res.validity_mask().tolist() == k["expect_validity"]


@pytest.mark.parametrize("case", [c["test"] for c in KATS["runend_compute"]["cases"]])
def test_kat_runend_compute_on_gpu(ctx, case):
    """runend/compute.rs:132-353: take (vxg_take_array), slices (SliceFn metadata: ends/values of
    the covering runs, offset, length) and slice-then-take, incl. nulls and the out-of-bounds
    take, all on the GPU."""
    k = next(c for c in KATS["runend_compute"]["cases"] if c["test"] == case)
    arr = _apply_slices(_ree(k["build"], k.get("ends_ptype", "u64")), k.get("slices", []))
    full = _gpu(arr, ctx)
    ref, rvalid = canon(arr)
    assert full.numpy().tobytes() == ref.tobytes()
    if "take" not in k:
        assert full.numpy().tolist() == k["expect"]
        if "expect_validity" in k:
            assert full.validity_mask().tolist() == k["expect_validity"]
        return
    idx = np.array(k["take"], np.int64)
    if "expect_error" in k:
        with pytest.raises(VortexGpuError, match="OutOfBounds|out of bounds"):
            A.take(arr.to(_dev()), idx, ctx)
        return
    res = A.take(arr.to(_dev()), idx, ctx)
    assert _masked(res.numpy(), res.validity_mask()) == k["expect"]


def _sparse_kat(k):
    idx = A.primitive(np.array(k["indices"], np.uint64))
    if "values_bits" in k:
        vals = np.array([struct.unpack("<d", bytes.fromhex(h))[0] for h in k["values_bits"]])
        return A.sparse(idx, A.primitive(vals, validity="ALL_VALID"), k["len"])
    return A.sparse(idx, A.primitive(np.array(k["values"], A.NP_OF_PTYPE[k["ptype"]])), k["len"], fill=k["fill"])


@pytest.mark.parametrize("case", [c["test"] for c in KATS["sparse_slices"]["cases"]])
def test_kat_sparse_slices_on_gpu(ctx, case):
    """sparse/compute/slice.rs:29-70: the sliced SparseArray (indices by search_sorted, new
    indices_offset) canonicalizes on the GPU to the fill with the one kept patch."""
    from oracle_tree import slice_checked
    k0 = KATS["sparse_slices"]
    k = next(c for c in k0["cases"] if c["test"] == case)
    arr = _sparse_kat(k0)
    for s in k["slices"]:
        arr = slice_checked(arr, *s)
    got = _gpu(arr, ctx).numpy()
    assert got.size == k["expect_len"]
    for i, v in k["expect_at"]:
        assert int(got[i]) == v
    assert int(np.count_nonzero(got)) == len(k["expect_values"])
    assert got.tobytes() == canon(arr)[0].tobytes()


@pytest.mark.parametrize("case", [c["test"] for c in KATS["sparse_take"]["cases"]])
def test_kat_sparse_take_on_gpu(ctx, case):
    """sparse/compute/take.rs:114-200: take on a null-filled f64 SparseArray.  The reference
    returns a SparseArray (positions, values); its canonical -- the taken values, null where no
    patch was hit -- is what vxg_take_array produces, and the restated SparseArray result
    canonicalizes to the same bytes on the GPU."""
    from oracle_tree import sparse_take
    k0 = KATS["sparse_take"]
    k = next(c for c in k0["cases"] if c["test"] == case)
    sp = _sparse_kat(k0)
    res = A.take(sp.to(_dev()), np.array(k["take"], np.int64), ctx)
    got, valid = res.numpy(), res.validity_mask()
    pos = k["expect_indices"]
    assert valid.tolist() == [i in pos for i in range(len(k["take"]))]
    assert [struct.pack("<d", got[i]).hex() for i in pos] == k["expect_values_bits"]
    taken = sparse_take(sp, k["take"])
    t = _gpu(taken, ctx)
    assert t.validity_mask().tolist() == valid.tolist()
    assert t.numpy()[valid].tobytes() == got[valid].tobytes()


def test_kat_sparse_bool_on_gpu(ctx):
    """sparse/flatten.rs:108-117: Sparse(Bool) with a true fill canonicalizes to Canonical::Bool;
    bits = fill with the patches, validity set exactly at the indices (:44-66)."""
    k = KATS["sparse_bool"]
    arr = A.sparse_bool(A.primitive(np.array(k["indices"], np.uint64)), A.bool_array(k["values"]), k["len"],
                        fill=k["fill"])
    res = _gpu(arr, ctx)
    assert res.kind == "bool"
    assert res.numpy().tolist() == k["expect"]
    assert res.validity_mask().tolist() == k["expect_validity"]


def test_kat_chunked_pack_sliced_varbin_on_gpu(ctx):
    """chunked/canonical.rs:254-273 pack_sliced_varbin: two sliced VarBinView chunks packed into
    one VarBinView (pack_views) read back as ["bar", "baz", "baz", "quak"]; a variant with
    out-of-line strings checks the rebased buffer_index of sliced chunks."""
    from oracle_tree import slice_checked
    k = KATS["chunked_pack_sliced_varbin"]
    for strs in ([s.encode() for s in k["strings"]],
                 [s.encode() * 5 for s in k["strings"]]):
        base = E.encode_varbinview(strs)
        arr = A.chunked([slice_checked(base, *s) for s in k["slices"]])
        res = _gpu(arr, ctx)
        views, _ = res.numpy()
        heap = res.buffers()
        expect = [s.encode() * (1 if strs[0] == b"foo" else 5) for s in k["expect"]]
        assert [view_bytes(views, heap, i) for i in range(views.shape[0])] == expect
        (rv, rb), _ = canon(arr)
        assert [view_bytes(rv, rb, i) for i in range(rv.shape[0])] == expect


# ---------------------------------------------------------------- round 6 (VERDICT r05 Missing 2)
def test_kat_dict_flatten_nullable_primitive_on_gpu(ctx):
    """dict/compute.rs:76-90: the canonical values buffer equals the reference's byte for byte,
    null rows included (the dictionary's null slot holds 0, as from_nullable_vec writes)."""
    import kat_trees as K
    k = KATS["dict_flatten_nullable_primitive"]
    for label, arr in K.dict_nullable_primitive(k):
        res = _gpu(arr, ctx)
        assert res.numpy().tobytes().hex() == k["expect_buffer_hex"], label
        assert res.validity_mask().tolist() == k["validity"], label


def test_kat_dict_flatten_nullable_varbin_on_gpu(ctx):
    """dict/compute.rs:92-114: VarBinView and VarBin dictionaries with a null slot canonicalize to
    the reference's iterator values ["a", "b", None, "a", None, "b"]."""
    import kat_trees as K
    k = KATS["dict_flatten_nullable_varbin"]
    want = [None if s is None else s.encode() for s in k["expect_strings"]]
    for label, arr in K.dict_nullable_varbin(k):
        res = _gpu(arr, ctx)
        views, _ = res.numpy()
        heap = res.buffers()
        assert K.masked([view_bytes(views, heap, i) for i in range(arr.len)], res.validity_mask()) == want, label
        (rv, rh), _ = canon(arr)
        assert views.tobytes() == rv.tobytes(), label


def test_kat_for_scalar_at_negative_on_gpu(ctx):
    """for/compute.rs:173-180: FoR over i32 with a negative reference (-100, shift 2)."""
    import kat_trees as K
    k = KATS["for_scalar_at_negative"]
    for label, arr in K.for_negative(k):
        got = _gpu(arr, ctx).numpy()
        assert got.tolist() == k["expect_decoded"], label
        assert got.tobytes() == canon(arr)[0].tobytes(), label


def test_kat_zigzag_nullable_scalar_at_on_gpu(ctx):
    """zigzag/compute.rs:96-106: ZigZag over an AllValid child; scalar_at(1) == -160."""
    import kat_trees as K
    k = KATS["zigzag_nullable_scalar_at"]
    for label, arr in K.zigzag_nullable(k):
        res = _gpu(arr, ctx)
        got = res.numpy()
        assert got.tolist() == k["expect_decoded"], label
        for i, v in k["expect_at"]:
            assert int(got[i]) == v
        valid = res.validity_mask()
        assert valid is None or valid.all()


def test_kat_alp_f32_compare_with_patches_on_gpu(ctx):
    """alp/compute.rs:187-201: f32 with patches; the last row (a patch) decodes to exactly
    1_000_000.9f32, so comparing with it is true there."""
    import kat_trees as K
    k = KATS["alp_f32_compare_with_patches"]
    vals = K.f32(k["values_bits"])
    for label, arr in K.alp_compare_with_patches(k):
        got = _gpu(arr, ctx).numpy()
        assert struct.pack("<f", got[-1]).hex() == k["expect_last_bits"], label
        assert bool(got[-1] == np.float32(1_000_000.9)) == k["expect_eq_last"]
        assert got.tobytes() == vals.tobytes(), label
        assert got.tobytes() == canon(arr)[0].tobytes(), label
