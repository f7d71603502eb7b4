"""ctypes bindings for libvortex_gpu.so (include/vortex_gpu.h) and libvortex_enc.so.

The decode engine is native code only: if the HIP library is missing or does not load, every
entry point raises — there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
# VXG_GPU_LIB: load another build of the engine (A/B experiments); default the in-tree one
GPU_LIB_PATH = Path(os.environ["VXG_GPU_LIB"]) if os.environ.get("VXG_GPU_LIB") else _HERE / "libvortex_gpu.so"
ENC_LIB_PATH = _HERE / "libvortex_enc.so"

# ---- ids mirrored from include/vortex_gpu.h (reference encoding/mod.rs:106-147) ----------
ENC = dict(BOOL=2, PRIMITIVE=3, STRUCT=4, VARBIN=5, VARBINVIEW=6, SPARSE=8, CONSTANT=9,
           CHUNKED=10, ALP=17, BYTE_BOOL=18, DICT=20, FL_BITPACKED=21, FL_DELTA=22, FL_FOR=23,
           FSST=24, ROARING_BOOL=25, RUN_END=27, RUN_END_BOOL=28, ZIGZAG=29, ALP_RD=30)
PTYPES = ["u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64", "f16", "f32", "f64"]
PTYPE = {n: i for i, n in enumerate(PTYPES)}
DTYPE = dict(NULL=0, BOOL=1, PRIMITIVE=2, UTF8=3, BINARY=4)
VALIDITY = dict(NON_NULLABLE=0, ALL_VALID=1, ALL_INVALID=2, ARRAY=3)
ABI_VERSION = 8  # VXG_ABI_VERSION
STATUS = {0: "OK", 1: "OutOfBounds", 2: "ComputeError", 3: "InvalidArgument", 4: "InvalidSerde",
          5: "NotImplemented", 6: "MismatchedTypes", 7: "AssertionFailed", 8: "HipError",
          9: "OutOfMemory"}


class VortexGpuError(RuntimeError):
    """A non-OK vxg_status (VortexError variant name + vxg_last_error message)."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS.get(status, status)}: {msg}")
        self.status = status
        self.kind = STATUS.get(status, str(status))


class VxgBuffer(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("len", C.c_uint64)]


class _MBitPacked(C.Structure):
    _fields_ = [("bit_width", C.c_uint8), ("has_patches", C.c_uint8), ("offset", C.c_uint16)]


class _MFoR(C.Structure):
    _fields_ = [("reference", C.c_uint64), ("shift", C.c_uint8)]


class _MDelta(C.Structure):
    _fields_ = [("deltas_len", C.c_uint64), ("offset", C.c_uint16)]


class _MAlp(C.Structure):
    _fields_ = [("e", C.c_uint8), ("f", C.c_uint8), ("has_patches", C.c_uint8)]


class _MAlpRd(C.Structure):
    _fields_ = [("right_bit_width", C.c_uint8), ("dict_len", C.c_uint8),
                ("left_parts_ptype", C.c_uint8), ("has_exceptions", C.c_uint8),
                ("dict", C.c_uint16 * 8)]


class _MDict(C.Structure):
    _fields_ = [("codes_ptype", C.c_uint8), ("values_len", C.c_uint64)]


class _MFsst(C.Structure):
    _fields_ = [("symbols_len", C.c_uint64), ("codes_nullable", C.c_uint8),
                ("uncompressed_lengths_ptype", C.c_uint8)]


class _MRunEnd(C.Structure):
    _fields_ = [("ends_ptype", C.c_uint8), ("num_runs", C.c_uint64), ("offset", C.c_uint64)]


class _MSparse(C.Structure):
    _fields_ = [("indices_offset", C.c_uint64), ("indices_len", C.c_uint64),
                ("fill_is_null", C.c_uint8), ("fill", C.c_uint8 * 16)]


class _MConstant(C.Structure):
    _fields_ = [("is_null", C.c_uint8), ("scalar", C.c_uint8 * 16)]


class _MChunked(C.Structure):
    _fields_ = [("nchunks", C.c_uint64)]


class _MVarBin(C.Structure):
    _fields_ = [("offsets_ptype", C.c_uint8), ("bytes_len", C.c_uint64)]


class _MBool(C.Structure):
    _fields_ = [("first_byte_bit_offset", C.c_uint8)]


class _MRunEndBool(C.Structure):
    _fields_ = [("start", C.c_uint8), ("ends_ptype", C.c_uint8), ("num_runs", C.c_uint64),
                ("offset", C.c_uint64)]


class _MVarBinView(C.Structure):
    _fields_ = [("n_buffers", C.c_uint32)]


class VxgMeta(C.Union):
    _fields_ = [("bitpacked", _MBitPacked), ("for_", _MFoR), ("delta", _MDelta), ("alp", _MAlp),
                ("alprd", _MAlpRd), ("dict", _MDict), ("fsst", _MFsst), ("runend", _MRunEnd),
                ("sparse", _MSparse), ("constant", _MConstant), ("chunked", _MChunked),
                ("varbin", _MVarBin), ("boolean", _MBool), ("runendbool", _MRunEndBool),
                ("varbinview", _MVarBinView), ("raw", C.c_uint64 * 5)]


class VxgArray(C.Structure):
    pass


VxgArray._fields_ = [("encoding", C.c_uint16), ("dtype", C.c_uint8), ("ptype", C.c_uint8),
                     ("nullable", C.c_uint8), ("validity", C.c_uint8), ("reserved", C.c_uint16),
                     ("len", C.c_uint64), ("meta", VxgMeta), ("n_buffers", C.c_uint32),
                     ("n_children", C.c_uint32), ("buffers", C.POINTER(VxgBuffer)),
                     ("children", C.POINTER(VxgArray))]


class VxgDataBuffer(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("len", C.c_uint64)]


class VxgCanonical(C.Structure):
    _fields_ = [("kind", C.c_uint16), ("ptype", C.c_uint8), ("dtype", C.c_uint8),
                ("reserved", C.c_uint32), ("len", C.c_uint64), ("values", C.c_void_p),
                ("values_bytes", C.c_uint64), ("views", C.c_void_p), ("data", C.c_void_p),
                ("data_bytes", C.c_uint64), ("validity", C.c_void_p),
                ("n_data_buffers", C.c_uint32), ("data_buffers_cap", C.c_uint32),
                ("data_buffers", C.POINTER(VxgDataBuffer))]


PLAN_MEASURE = 1  # VXG_PLAN_MEASURE


class VxgPlanInfo(C.Structure):
    _fields_ = [("batched", C.c_uint32), ("branches", C.c_uint32), ("direct_nodes", C.c_uint32),
                ("n_candidates", C.c_uint32), ("candidate_batched", C.c_uint32 * 2),
                ("candidate_ms", C.c_float * 2), ("create_ms", C.c_float), ("selection", C.c_uint32),
                ("candidate_cost", C.c_uint32 * 2), ("reserved", C.c_uint32)]


PLAN_SELECTION = {0: "single", 1: "faster", 2: "tie_fewer_nodes", 3: "unmeasured"}


# vxg_option (ABI 8): per-context launch shapes
OPT_K1W_MIN_GROUPS, OPT_K1W_BPW, OPT_K1_WAVE = 1, 2, 3


class VxgLaunchStats(C.Structure):
    _fields_ = [("k1w_launches", C.c_uint64), ("k1w_last_groups", C.c_uint64), ("k1w_last_bpw", C.c_uint32),
                ("k1w_last_bpw_max", C.c_uint32), ("k1w_min_bpw", C.c_uint32), ("k1w_max_bpw", C.c_uint32)]


class VxgIntStats(C.Structure):
    _fields_ = [("n", C.c_uint64), ("min_bits", C.c_uint64), ("max_bits", C.c_uint64), ("trailing_zeros", C.c_uint32),
                ("reserved", C.c_uint32), ("bit_width_freq", C.c_uint64 * 65)]


class VxgDictChunk(C.Structure):
    _fields_ = [("packed", C.c_void_p), ("dict_values", C.c_void_p), ("out", C.c_void_p),
                ("n_blocks", C.c_uint64), ("len", C.c_uint64), ("dict_len", C.c_uint64)]


assert C.sizeof(VxgMeta) == 40, C.sizeof(VxgMeta)
assert C.sizeof(VxgArray) == 80, C.sizeof(VxgArray)

VP, U64, U32, INT, UINT = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int, C.c_uint
ST = C.c_int

# name -> (restype, argtypes); mirrors include/vortex_gpu.h exactly (tests check the set).
GPU_SIGNATURES = {
    "vxg_abi_version": (C.c_int, []),
    "vxg_open": (ST, [INT, C.POINTER(VP)]),
    "vxg_close": (ST, [VP]),
    "vxg_last_error": (C.c_char_p, []),
    "vxg_alloc": (ST, [VP, U64, C.POINTER(VP)]),
    "vxg_free": (ST, [VP, VP]),
    "vxg_host_alloc": (ST, [VP, U64, C.POINTER(VP)]),
    "vxg_host_free": (ST, [VP, VP]),
    "vxg_memcpy_h2d": (ST, [VP, VP, VP, U64, VP]),
    "vxg_memcpy_d2h": (ST, [VP, VP, VP, U64, VP]),
    "vxg_memcpy_d2d": (ST, [VP, VP, VP, U64, VP]),
    "vxg_stream_sync": (ST, [VP, VP]),
    "vxg_set_option": (ST, [VP, INT, C.c_int64]),
    "vxg_get_option": (ST, [VP, INT, C.POINTER(C.c_int64)]),
    "vxg_get_launch_stats": (ST, [VP, C.POINTER(VxgLaunchStats), INT]),
    "vxg_canonical_size": (ST, [VP, C.POINTER(VxgArray), C.POINTER(U64), C.POINTER(U64)]),
    "vxg_canonicalize": (ST, [VP, C.POINTER(VxgArray), C.POINTER(VxgCanonical), VP]),
    "vxg_plan_create": (ST, [VP, C.POINTER(VxgArray), C.POINTER(VxgCanonical), U32, C.POINTER(VP)]),
    "vxg_plan_create_ex": (ST, [VP, C.POINTER(VxgArray), C.POINTER(VxgCanonical), U32, U32, C.POINTER(VP)]),
    "vxg_plan_get_info": (ST, [VP, C.c_void_p]),
    "vxg_plan_select": (U32, [C.POINTER(C.c_float), C.POINTER(U32), U32, C.POINTER(U32)]),
    "vxg_plan_launch": (ST, [VP, VP]),
    "vxg_plan_destroy": (ST, [VP]),
    "vxg_canonical_layout": (ST, [VP, C.POINTER(VxgArray), C.POINTER(U64), C.POINTER(U64),
                                  C.POINTER(VxgDataBuffer), U32, C.POINTER(U32)]),
    "vxg_bitunpack": (ST, [VP, INT, UINT, UINT, U64, VP, U64, VP, VP]),
    "vxg_bitunpack_for": (ST, [VP, INT, UINT, UINT, U64, VP, U64, U64, UINT, INT, VP, VP]),
    "vxg_bitunpack_alp": (ST, [VP, INT, UINT, UINT, U64, VP, U64, U64, UINT, UINT, UINT, VP, VP]),
    "vxg_bitunpack_dict": (ST, [VP, INT, UINT, UINT, U64, VP, U64, VP, U64, UINT, VP, VP]),
    "vxg_bitunpack_dict_chunks": (ST, [VP, INT, UINT, UINT, C.POINTER(VxgDictChunk), U32, VP]),
    "vxg_patch": (ST, [VP, INT, VP, U64, INT, VP, U64, VP, U64, VP]),
    "vxg_for_decode": (ST, [VP, INT, VP, U64, U64, UINT, VP, VP]),
    "vxg_zigzag_decode": (ST, [VP, INT, VP, U64, VP, VP]),
    "vxg_alp_decode": (ST, [VP, INT, VP, U64, UINT, UINT, VP, VP]),
    "vxg_alprd_decode": (ST, [VP, INT, VP, VP, UINT, UINT, VP, U64, VP, VP, U64, VP, VP]),
    "vxg_take": (ST, [VP, UINT, VP, U64, INT, VP, U64, VP, VP]),
    "vxg_delta_decode": (ST, [VP, INT, VP, U64, VP, U64, U64, U64, VP, VP]),
    "vxg_runend_decode": (ST, [VP, UINT, VP, INT, VP, U64, U64, U64, VP, VP]),
    "vxg_runend_bool_decode": (ST, [VP, INT, VP, U64, U64, INT, U64, VP, U64, VP]),
    "vxg_bytebool_to_bits": (ST, [VP, VP, U64, VP, U64, VP]),
    "vxg_take_array": (ST, [VP, VP, INT, VP, U64, VP, VP]),
    "vxg_filter_array": (ST, [VP, VP, VP, VP, VP]),
    "vxg_fsst_scratch_bytes": (U64, [U64]),
    "vxg_fsst_decode": (ST, [VP, VP, VP, UINT, VP, INT, VP, INT, VP, U64, VP, VP, VP, VP, VP]),
    "vxg_fill": (ST, [VP, UINT, VP, U64, VP, VP]),
    "vxg_compute_int_stats": (ST, [VP, INT, VP, U64, C.POINTER(VxgIntStats), VP]),
    "vxg_bitpack": (ST, [VP, INT, UINT, VP, U64, VP, U64, VP]),
    "vxg_for_encode": (ST, [VP, INT, VP, U64, U64, UINT, VP, VP]),
    "vxg_for_bitpack": (ST, [VP, INT, U64, UINT, UINT, VP, U64, VP, U64, VP]),
    "vxg_gather_patches": (ST, [VP, INT, UINT, VP, U64, VP, VP, U64, C.POINTER(U64), VP]),
    "vxg_alp_encode": (ST, [VP, INT, VP, U64, C.POINTER(C.c_uint8), C.POINTER(C.c_uint8), VP, VP, VP, U64,
                            C.POINTER(U64), VP]),
    "vxg_fsst_compress": (ST, [VP, VP, VP, C.c_uint32, INT, VP, VP, U64, VP, U64, VP, U64, VP, VP, C.POINTER(U64), VP]),
}

class VxgFileColumn(C.Structure):
    _fields_ = [("name", C.c_char_p), ("dtype", C.c_uint8), ("ptype", C.c_uint8), ("nullable", C.c_uint8),
                ("is_extension", C.c_uint8), ("n_chunks", C.c_uint32), ("extension_id", C.c_char_p),
                ("extension_metadata", C.POINTER(C.c_uint8)), ("extension_metadata_len", C.c_uint64),
                ("rows", C.c_uint64)]


class VxgFileChunk(C.Structure):
    _fields_ = [("row_offset", C.c_uint64), ("rows", C.c_uint64), ("message_begin", C.c_uint64),
                ("message_end", C.c_uint64), ("buffers_begin", C.c_uint64)]


# include/vortex_file.h (the Vortex file reader, exported by libvortex_gpu.so)
FILE_SIGNATURES = {
    "vxg_file_open": (ST, [VP, U64, C.POINTER(VP)]),
    "vxg_file_close": (ST, [VP]),
    "vxg_file_info": (ST, [VP, C.POINTER(U64), C.POINTER(U32)]),
    "vxg_file_column_info": (ST, [VP, U32, C.POINTER(VxgFileColumn)]),
    "vxg_file_chunk_info": (ST, [VP, U32, U32, C.POINTER(VxgFileChunk)]),
    "vxg_file_chunk_offsets": (ST, [VP, U32, U32, U32, C.POINTER(U64)]),
    "vxg_file_column_array": (ST, [VP, U32, U32, U32, VP, U64, U64, VP, C.POINTER(C.POINTER(VxgArray))]),
}

ENC_SIGNATURES = {
    "vxe_bitpack": (U64, [INT, UINT, VP, U64, VP]),
    "vxe_roaring_bool_encode": (U64, [VP, U64, VP, U64]),
    "vxe_best_bit_width": (UINT, [INT, VP, U64]),
    "vxe_min_patchless_bit_width": (UINT, [INT, VP, U64]),
    "vxe_gather_patches": (U64, [INT, UINT, VP, U64, VP, VP, U64]),
    "vxe_for_compress": (INT, [INT, VP, U64, VP, C.POINTER(U64), C.POINTER(UINT)]),
    "vxe_delta_compress": (None, [INT, VP, U64, VP, VP]),
    "vxe_zigzag_encode": (None, [INT, VP, U64, VP]),
    "vxe_alp_encode_f64": (U64, [VP, U64, VP, VP, VP, VP, VP, U64]),
    "vxe_alp_encode_f32": (U64, [VP, U64, VP, VP, VP, VP, VP, U64]),
    "vxe_alprd_encode_f64": (U64, [VP, U64, VP, VP, VP, VP, VP, VP, VP, U64]),
    "vxe_alprd_encode_f32": (U64, [VP, U64, VP, VP, VP, VP, VP, VP, VP, U64]),
    "vxe_dict_encode": (U64, [INT, VP, U64, VP, VP, U64]),
    "vxe_runend_encode": (U64, [INT, VP, U64, VP, VP]),
    "vxe_fsst_train": (None, [VP, VP, U64, VP]),
    "vxe_fsst_compress": (U64, [VP, VP, VP, U64, VP, U64, VP]),
}


class VxeFsstTable(C.Structure):
    _fields_ = [("symbols", C.c_uint64 * 255), ("lens", C.c_uint8 * 255), ("n_symbols", C.c_uint32)]


def _load(path: Path, sigs: dict) -> C.CDLL:
    if not path.exists():
        raise ImportError(f"{path.name} is not built (run __graft_entry__.build() or make -C "
                          f"vortex_amd/csrc); the decode engine has no CPU fallback")
    lib = C.CDLL(str(path))
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)  # AttributeError = missing export: fail loudly
        fn.restype = res
        fn.argtypes = args
    return lib


_gpu = None
_enc = None


def gpu_lib() -> C.CDLL:
    global _gpu
    if _gpu is None:
        _gpu = _load(GPU_LIB_PATH, {**GPU_SIGNATURES, **FILE_SIGNATURES})
        if _gpu.vxg_abi_version() != ABI_VERSION:
            raise ImportError("libvortex_gpu.so ABI version mismatch")
    return _gpu


def enc_lib() -> C.CDLL:
    global _enc
    if _enc is None:
        _enc = _load(ENC_LIB_PATH, ENC_SIGNATURES)
    return _enc


def check(status: int) -> None:
    if status != 0:
        msg = gpu_lib().vxg_last_error().decode(errors="replace")
        raise VortexGpuError(status, msg)
