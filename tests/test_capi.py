"""CPU: the C-ABI libraries load and export exactly what include/*.h declares (no GPU calls)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

import vortex_amd._lib as L

ROOT = Path(__file__).resolve().parent.parent


def declared(header: str, prefix: str) -> set:
    text = (ROOT / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(rf"\b({prefix}_[a-z0-9_]+)\s*\(", text))


def exported(lib: Path, prefix: str) -> set:
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True,
                         check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.split() and ln.split()[-1].startswith(prefix + "_")}


def test_gpu_lib_exports_match_header():
    decl = declared("vortex_gpu.h", "vxg")
    assert decl == set(L.GPU_SIGNATURES), "ctypes signatures out of sync with vortex_gpu.h"
    fdecl = declared("vortex_file.h", "vxg")
    assert fdecl == set(L.FILE_SIGNATURES), "ctypes signatures out of sync with vortex_file.h"
    decl = decl | fdecl
    assert exported(L.GPU_LIB_PATH, "vxg") == decl
    lib = L.gpu_lib()  # loads (HIP runtime present in the image; no device needed)
    for name in decl:
        assert hasattr(lib, name)
    assert lib.vxg_abi_version() == L.ABI_VERSION


def test_enc_lib_exports_match_header():
    decl = declared("vortex_enc.h", "vxe")
    assert decl == set(L.ENC_SIGNATURES)
    assert exported(L.ENC_LIB_PATH, "vxe") == decl
    L.enc_lib()


def test_struct_layouts_match_c(tmp_path):
    """ctypes mirrors must have the C compiler's sizes AND field offsets for the header."""
    fields = {"vxg_array": (L.VxgArray, ["encoding", "len", "meta", "n_buffers", "n_children", "buffers",
                                         "children"]),
              "vxg_canonical": (L.VxgCanonical, ["kind", "len", "values", "views", "data", "data_bytes",
                                                 "validity", "n_data_buffers", "data_buffers_cap",
                                                 "data_buffers"]),
              "vxg_data_buffer": (L.VxgDataBuffer, ["offset", "len"]),
              "vxg_dict_chunk": (L.VxgDictChunk, ["packed", "out", "n_blocks", "dict_len"]),
              "vxg_file_column": (L.VxgFileColumn, ["name", "dtype", "is_extension", "n_chunks", "extension_id",
                                                    "extension_metadata_len", "rows"]),
              "vxg_file_chunk": (L.VxgFileChunk, ["row_offset", "rows", "message_end", "buffers_begin"])}
    src = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{ROOT}/include/vortex_gpu.h"', f'#include "{ROOT}/include/vortex_file.h"', "int main(){",
           'printf("vxg_meta %zu\\n", sizeof(vxg_meta));',
           'printf("runendbool.start %zu\\n", offsetof(vxg_meta, runendbool.start));',
           'printf("runendbool.ends_ptype %zu\\n", offsetof(vxg_meta, runendbool.ends_ptype));',
           'printf("runendbool.num_runs %zu\\n", offsetof(vxg_meta, runendbool.num_runs));',
           'printf("runendbool.offset %zu\\n", offsetof(vxg_meta, runendbool.offset));']
    for st, (_, fs) in fields.items():
        src.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f in fs:
            src.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    src.append("return 0;}")
    (tmp_path / "sz.c").write_text("\n".join(src))
    subprocess.run(["gcc", str(tmp_path / "sz.c"), "-o", str(tmp_path / "sz")], check=True)
    got = dict(ln.split() for ln in subprocess.run([str(tmp_path / "sz")], capture_output=True, text=True,
                                                    check=True).stdout.splitlines())
    assert int(got["vxg_meta"]) == C.sizeof(L.VxgMeta)
    for f in ("start", "ends_ptype", "num_runs", "offset"):
        assert int(got[f"runendbool.{f}"]) == getattr(L._MRunEndBool, f).offset, f
    for st, (cls, fs) in fields.items():
        assert int(got[st]) == C.sizeof(cls), st
        for f in fs:
            assert int(got[f"{st}.{f}"]) == getattr(cls, f).offset, (st, f)


def test_encoding_ids_match_reference():
    # vortex-array/src/encoding/mod.rs:106-147
    ref = dict(BOOL=2, PRIMITIVE=3, STRUCT=4, VARBIN=5, VARBINVIEW=6, SPARSE=8, CONSTANT=9, CHUNKED=10,
               ALP=17, BYTE_BOOL=18, DICT=20, FL_BITPACKED=21, FL_DELTA=22, FL_FOR=23, FSST=24, ROARING_BOOL=25, RUN_END=27,
               RUN_END_BOOL=28, ZIGZAG=29, ALP_RD=30)
    assert L.ENC == ref
    hdr = (ROOT / "include" / "vortex_gpu.h").read_text()
    for k, v in ref.items():
        assert re.search(rf"VXG_ENC_{k} = {v}\b", hdr), k


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    monkeypatch.setattr(L, "_gpu", None)
    monkeypatch.setattr(L, "GPU_LIB_PATH", tmp_path / "absent.so")
    with pytest.raises(ImportError, match="no CPU fallback"):
        L.gpu_lib()


def test_plan_select_tie_rule():
    """vxg_plan_select (host-only): the faster candidate unless another is within 3 % and its
    graph is smaller; unmeasured -> the smaller graph; deterministic on equal cost (VERDICT r04
    item 6: C3's candidates were 0.1871 vs 0.1907 ms, a coin flip before)."""
    import ctypes as C
    lib = L.gpu_lib()

    def sel(ms, cost):
        n = len(cost)
        s = C.c_uint32(99)
        msa = None if ms is None else (C.c_float * n)(*ms)
        best = lib.vxg_plan_select(msa, (C.c_uint32 * n)(*cost), n, C.byref(s))
        return best, L.PLAN_SELECTION[s.value]

    assert sel([0.2], [5]) == (0, "single")
    assert sel([0.1871, 0.1907], [3, 1]) == (1, "tie_fewer_nodes")   # within 3 %: smaller graph
    assert sel([0.1907, 0.1871], [1, 3]) == (0, "tie_fewer_nodes")
    assert sel([0.1871, 0.1907], [1, 3]) == (0, "tie_fewer_nodes")   # the faster is also smaller
    assert sel([0.2899, 0.3886], [40, 4]) == (0, "faster")            # C5 at 1 GPU: 34 % apart
    assert sel([0.120, 0.060], [40, 4]) == (1, "faster")
    assert sel([0.100, 0.1029], [7, 7]) == (0, "tie_fewer_nodes")     # equal cost: lowest index
    assert sel([0.1029, 0.100], [7, 7]) == (0, "tie_fewer_nodes")
    assert sel([0.100, 0.1031], [9, 1]) == (0, "faster")              # 3.1 % apart: not a tie
    assert sel(None, [9, 4]) == (1, "unmeasured")
    assert sel(None, [4, 4]) == (0, "unmeasured")
