"""ctypes loader for oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the parity checker / CPU baseline ("port").  See vx_oracle.h for citations.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "liboracle.so"
PT = {"u8": 0, "u16": 1, "u32": 2, "u64": 3, "i8": 4, "i16": 5, "i32": 6, "i64": 7,
      "f16": 8, "f32": 9, "f64": 10}
NP = {"u8": np.uint8, "u16": np.uint16, "u32": np.uint32, "u64": np.uint64, "i8": np.int8,
      "i16": np.int16, "i32": np.int32, "i64": np.int64, "f32": np.float32, "f64": np.float64}
VP, U64, UINT, INT, SZ = C.c_void_p, C.c_uint64, C.c_uint, C.c_int, C.c_size_t

_SIG = {
    "vxo_fl_index": (UINT, [UINT, UINT, UINT]),
    "vxo_fl_transpose": (UINT, [UINT]),
    "vxo_fl_pack_block": (None, [UINT, UINT, VP, VP]),
    "vxo_fl_unpack_block": (None, [UINT, UINT, VP, VP]),
    "vxo_fl_unpack_single": (U64, [UINT, UINT, VP, UINT]),
    "vxo_bitpack": (SZ, [INT, UINT, VP, SZ, VP]),
    "vxo_unpack": (INT, [INT, UINT, UINT, SZ, VP, SZ, VP]),
    "vxo_patch": (INT, [INT, VP, SZ, INT, VP, U64, VP, SZ]),
    "vxo_for_decode": (None, [INT, VP, SZ, U64, UINT, VP]),
    "vxo_delta_decode": (INT, [INT, VP, SZ, VP, SZ, SZ, SZ, VP]),
    "vxo_zigzag_decode": (None, [INT, VP, SZ, VP]),
    "vxo_alp_decode_f32": (None, [VP, SZ, UINT, UINT, VP]),
    "vxo_alp_decode_f64": (None, [VP, SZ, UINT, UINT, VP]),
    "vxo_alprd_decode_f32": (None, [VP, VP, UINT, VP, SZ, VP, VP, SZ, VP]),
    "vxo_alprd_decode_f64": (None, [VP, VP, UINT, VP, SZ, VP, VP, SZ, VP]),
    "vxo_take": (INT, [INT, VP, SZ, INT, VP, SZ, VP]),
    "vxo_runend_decode": (INT, [INT, VP, INT, VP, SZ, SZ, SZ, VP]),
    "vxo_runend_bool_decode": (INT, [INT, VP, SZ, SZ, INT, SZ, VP]),
    "vxo_runend_bool_encode": (SZ, [VP, SZ, VP, VP]),
    "vxo_bytebool_to_bits": (None, [VP, SZ, VP]),
    "vxo_roaring_bool_decode": (INT, [VP, SZ, SZ, VP]),
    "vxo_fill": (None, [INT, VP, SZ, VP]),
    "vxo_fsst_decompress": (SZ, [VP, VP, VP, SZ, VP]),
    "vxo_fsst_canonicalize": (INT, [VP, VP, VP, INT, VP, INT, VP, SZ, VP, VP, C.POINTER(SZ), VP]),
    "vxo_make_views": (None, [VP, VP, SZ, VP, C.c_uint32, VP]),
    "vxo_rebase_views": (None, [VP, SZ, C.c_uint32]),
}

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError("oracle/liboracle.so not built (make -C oracle)")
        _lib = C.CDLL(str(LIB_PATH))
        for k, (r, a) in _SIG.items():
            f = getattr(_lib, k)
            f.restype, f.argtypes = r, a
    return _lib


def p(a: np.ndarray):
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else C.c_void_p(0)
