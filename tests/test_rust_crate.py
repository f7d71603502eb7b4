"""The source-only Rust crate (rust/vortex-gpu): checks that need no Rust toolchain.

* ffi.rs is exactly what tools/gen_ffi_rs.py generates from the current headers (so the
  binding cannot drift from the C ABI), and declares every function the library exports;
* meta.rs reads every metadata field by the name the reference's serde structs use — the same
  names the reference-layout writer (tools/vxfile.py ref_metadata) emits and the C++ file reader
  parses — and handles every encoding id the engine decodes.
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CRATE = ROOT / "rust" / "vortex-gpu"


def test_ffi_rs_is_generated_from_headers():
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "gen_ffi_rs.py"), "--check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_ffi_rs_declares_every_header_function():
    ffi = (CRATE / "src" / "ffi.rs").read_text()
    for h in ("vortex_gpu.h", "vortex_file.h"):
        text = re.sub(r"/\*.*?\*/", "", (ROOT / "include" / h).read_text(), flags=re.S)
        for name in re.findall(r"\b(vxg_\w+)\s*\(", text):
            assert f"pub fn {name}(" in ffi, name


def test_meta_rs_field_names_match_the_reference_metadata():
    meta = (CRATE / "src" / "meta.rs").read_text()
    used = set(re.findall(r'\.(?:u64|bool|string|ptype|get)\("(\w+)"\)', meta))
    used |= set(re.findall(r'\.index\("(\w+)"\)', meta))
    writer = (ROOT / "tools" / "vxfile.py").read_text()
    i = writer.index("def ref_metadata")
    body = writer[i: writer.index("\ndef ", i + 10)]
    emitted = set(re.findall(r'"(\w+)":', body))
    missing = sorted(k for k in used if k not in emitted and k not in ("e", "f"))
    assert not missing, missing


def test_meta_rs_covers_every_decoded_encoding():
    meta = (CRATE / "src" / "meta.rs").read_text()
    header = (ROOT / "include" / "vortex_gpu.h").read_text()
    ids = re.findall(r"(VXG_ENC_\w+)\s*=", header)
    for name in ids:
        if name == "VXG_ENC_STRUCT":  # canonical: not decoded by the engine
            continue
        assert f"ffi::{name}" in meta, name


def test_scan_rs_uses_the_reader_and_plan_entry_points():
    """scan.rs (scan_file) drives the batched path: the file reader, one region copy per column,
    the layout query, and one plan for all columns -- every entry point exists in ffi.rs."""
    scan = (CRATE / "src" / "scan.rs").read_text()
    ffi = (CRATE / "src" / "ffi.rs").read_text()
    needed = ["vxg_file_open", "vxg_file_close", "vxg_file_info", "vxg_file_column_info", "vxg_file_chunk_info",
              "vxg_file_chunk_offsets", "vxg_file_column_array", "vxg_alloc", "vxg_memcpy_h2d",
              "vxg_canonical_layout", "vxg_plan_create", "vxg_plan_launch", "vxg_plan_destroy", "vxg_stream_sync"]
    for name in needed:
        assert f"ffi::{name}(" in scan, name
        assert f"pub fn {name}(" in ffi, name
    lib = (CRATE / "src" / "lib.rs").read_text()
    assert "mod scan;" in lib and "scan_file" in lib
    meta = (CRATE / "src" / "meta.rs").read_text()
    assert "fn ptype_of_code" in meta
