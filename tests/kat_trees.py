"""Array trees of the round-6 known-answer tests (tests/golden/kat.json), shared by the oracle
checks (test_oracle.py) and the GPU replays (test_gpu_kats.py) so both see the same trees.

Each builder returns [(label, array)]: the tree the reference test builds (its encoder's direct
output, e.g. FoR over a plain PrimitiveArray) and the compressor cascade over the same values
(BitPacked children), since the engine decodes the two through different kernels.
"""
import struct

import numpy as np

import vortex_amd.arrays as A
import vortex_amd.encode as E


def f32(bits_hex):
    return np.array([struct.unpack("<f", bytes.fromhex(h))[0] for h in bits_hex], np.float32)


def dict_nullable_primitive(k):
    """dict/compute.rs:76-90: dict_encode_typed_primitive::<i32> of a nullable array."""
    vals = np.array(k["values"], np.int32)
    return [("primitive_codes", E.encode_dict_nullable(vals, k["validity"], bitpack_codes=False)),
            ("bitpacked_codes", E.encode_dict_nullable(vals, k["validity"], bitpack_codes=True))]


def dict_nullable_varbin(k):
    """dict/compute.rs:92-114: dict_encode_varbinview (VarBinView dictionary, null slot 0), and
    the VarBin-dictionary form a file holds (dict_encode_varbin)."""
    strs = [None if s is None else s.encode() for s in k["strings"]]
    values = E.encode_varbinview([None] + [v.encode() for v in k["expect_values"][1:]])
    codes = A.primitive(np.array(k["expect_codes"], np.uint64))
    return [("varbinview_values", A.dict_array(values, codes)),
            ("varbin_values", E.encode_dict_strings_nullable(strs))]


def for_negative(k):
    """for/compute.rs:173-180: for_compress output (FoR over the plain u32 encoded values) and
    the FoR -> BitPacked cascade."""
    vals = np.array(k["values"], np.int32)
    enc = np.array(k["expect_encoded"], np.uint32)
    direct = A.frame_of_reference(A.primitive(enc), k["expect_reference"], k["expect_shift"], "i32")
    return [("for_primitive", direct), ("for_bitpacked", E.encode_for_bitpacked(vals))]


def zigzag_nullable(k):
    """zigzag/compute.rs:96-106: ZigZag of an AllValid i32 array (validity rides on the encoded
    child, zigzag/compress.rs:10-33)."""
    enc = np.array(k["expect_encoded"], np.uint32)
    return [("zigzag_primitive", A.zigzag(A.primitive(enc, validity="ALL_VALID")))]


def alp_compare_with_patches(k):
    """alp/compute.rs:187-201: alp_encode (plain encoded child + Sparse patches) and the cascade."""
    vals = f32(k["values_bits"])
    e, f, enc, idx, pv = E.alp_encode(vals)
    patches = A.sparse(A.primitive(idx), A.primitive(pv, validity="ALL_VALID"), vals.size) if idx.size else None
    return [("alp_primitive", A.alp(A.primitive(enc), e, f, patches)), ("alp_cascade", E.encode_alp(vals))]


def masked(vals, valid):
    return [None if (valid is not None and not ok) else v for v, ok in
            zip(vals, valid if valid is not None else [True] * len(vals))]

