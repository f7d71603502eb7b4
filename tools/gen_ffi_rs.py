"""Generate rust/vortex-gpu/src/ffi.rs from include/vortex_gpu.h and include/vortex_file.h.

The headers are the drop-in boundary; this is the bindgen step a maintainer would otherwise run
(bindgen is not in this image).  It understands exactly the constructs the headers use:
  #define NAME <int>; typedef enum NAME {...} NAME; anonymous enum {...} constants;
  typedef struct/union NAME {...} NAME (anonymous struct members of a union become named
  structs NAME_member); opaque `typedef struct NAME NAME`; function prototypes.
  python tools/gen_ffi_rs.py            -> writes the file
  python tools/gen_ffi_rs.py --check    -> exit 1 if the committed file is stale
"""
from __future__ import annotations

import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
HEADERS = [ROOT / "include" / "vortex_gpu.h", ROOT / "include" / "vortex_file.h"]
OUT = ROOT / "rust" / "vortex-gpu" / "src" / "ffi.rs"

SCALARS = {"uint8_t": "u8", "uint16_t": "u16", "uint32_t": "u32", "uint64_t": "u64", "int8_t": "i8",
           "int16_t": "i16", "int32_t": "i32", "int64_t": "i64", "int": "c_int", "unsigned": "c_uint",
           "char": "c_char", "void": "c_void", "size_t": "usize", "double": "f64", "float": "f32",
           "unsigned long long": "u64"}


RUST_KEYWORDS = {"as", "async", "await", "box", "break", "const", "continue", "crate", "dyn", "else", "enum", "extern",
                 "false", "fn", "for", "if", "impl", "in", "let", "loop", "match", "mod", "move", "mut", "pub", "ref",
                 "return", "self", "static", "struct", "super", "trait", "true", "type", "unsafe", "use", "where",
                 "while"}


def ident(name: str) -> str:
    return "r#" + name if name in RUST_KEYWORDS else name


def strip_comments(s: str) -> str:
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def rust_type(ctype: str, known: set) -> str:
    """`const struct vxg_array*`, `vxg_ctx**`, `uint8_t` ... -> Rust."""
    t = ctype.strip()
    stars = t.count("*")
    base = t.replace("*", " ").split()
    is_const = "const" in base
    base = [b for b in base if b not in ("const", "struct", "union", "enum")]
    name = " ".join(base)
    r = SCALARS.get(name, name)
    if name not in SCALARS and name not in known:
        raise ValueError(f"unknown C type {ctype!r}")
    for i in range(stars):
        # only the pointee of the innermost pointer carries the header's const
        r = ("*const " if (i == 0 and is_const) else "*mut ") + r
    return r


def split_decl(decl: str):
    """'const uint8_t* name' / 'uint16_t dict[8]' -> (ctype, name, array_len)."""
    decl = " ".join(decl.split())
    m = re.match(r"(.*?)([A-Za-z_]\w*)\s*(\[(\d+)\])?$", decl)
    if not m:
        raise ValueError(decl)
    return m.group(1), m.group(2), m.group(4)


def fields(body: str, known: set, owner: str, extra: list) -> list[str]:
    out = []
    # anonymous struct members: struct { ... } name;
    for m in re.finditer(r"struct\s*\{(.*?)\}\s*(\w+)\s*;", body, flags=re.S):
        sname = f"{owner}_{m.group(2)}"
        extra.append(emit_struct("struct", sname, m.group(1), known, extra))
        known.add(sname)
    body2 = re.sub(r"struct\s*\{.*?\}\s*(\w+)\s*;", lambda m: f"{owner}_{m.group(1)} {m.group(1)};", body, flags=re.S)
    for d in body2.split(";"):
        d = d.strip()
        if not d:
            continue
        ctype, name, n = split_decl(d)
        rt = rust_type(ctype, known)
        out.append(f"    pub {ident(name)}: {'[' + rt + '; ' + n + ']' if n else rt},")
    return out


def emit_struct(kind: str, name: str, body: str, known: set, extra: list) -> str:
    fl = fields(body, known, name, extra)
    derive = "#[derive(Copy, Clone)]" if kind == "union" else "#[derive(Copy, Clone, Debug)]"
    return f"#[repr(C)]\n{derive}\npub {kind} {name} {{\n" + "\n".join(fl) + "\n}\n"


def generate() -> str:
    known: set = set()
    items: list[str] = []
    fns: list[str] = []
    for h in HEADERS:
        src = strip_comments(h.read_text())
        src = re.sub(r"^\s*#\s*(ifndef|ifdef|endif|include|else)[^\n]*", " ", src, flags=re.M)
        for m in re.finditer(r"^\s*#\s*define\s+(VXG_\w+)\s+(\d+)\s*$", src, flags=re.M):
            items.append(f"pub const {m.group(1)}: c_int = {m.group(2)};\n")
        src = re.sub(r"^\s*#[^\n]*", " ", src, flags=re.M)
        src = src.replace('extern "C" {', " ")
        toks = re.compile(r"typedef\s+enum\s+(\w+)\s*\{(.*?)\}\s*(\w+)\s*;|"
                          r"enum\s*\{(.*?)\}\s*;|"
                          r"typedef\s+(struct|union)\s+(\w+)\s*\{((?:[^{}]|\{[^{}]*\})*)\}\s*(\w+)\s*;|"
                          r"typedef\s+struct\s+(\w+)\s+(\w+)\s*;|"
                          r"([A-Za-z_][\w\s\*]*?\b)(vxg_\w+)\s*\(([^)]*)\)\s*;", re.S)
        for m in toks.finditer(src):
            if m.group(1):  # named enum type
                name = m.group(3)
                known.add(name)
                items.append(f"pub type {name} = c_int;\n")
                for k, v in re.findall(r"(\w+)\s*=\s*(-?\d+)", m.group(2)):
                    items.append(f"pub const {k}: {name} = {v};\n")
            elif m.group(4) is not None:  # anonymous constants
                for k, v in re.findall(r"(\w+)\s*=\s*(-?\d+)", m.group(4)):
                    items.append(f"pub const {k}: c_int = {v};\n")
            elif m.group(5):
                kind, name, body = m.group(5), m.group(8), m.group(7)
                known.add(name)
                extra: list = []
                s = emit_struct(kind, name, body, known, extra)
                items.extend(extra)
                items.append(s)
            elif m.group(9):  # opaque
                name = m.group(10)
                known.add(name)
                items.append(f"#[repr(C)]\npub struct {name} {{\n    _private: [u8; 0],\n}}\n")
            else:
                ret, name, args = m.group(11), m.group(12), m.group(13)
                rret = rust_type(ret, known)
                ra = []
                if args.strip() != "void":
                    for a in args.split(","):
                        ctype, an, n = split_decl(a)
                        ra.append(f"{ident(an)}: {rust_type(ctype, known)}")
                ret_s = "" if rret == "c_void" else f" -> {rret}"
                fns.append(f"    pub fn {name}({', '.join(ra)}){ret_s};\n")
    head = ("// @generated by tools/gen_ffi_rs.py from include/vortex_gpu.h and include/vortex_file.h.\n"
            "// Do not edit: regenerate with `python tools/gen_ffi_rs.py`.\n"
            "#![allow(non_camel_case_types, non_upper_case_globals, dead_code)]\n\n"
            "use std::os::raw::{c_char, c_int, c_uint, c_void};\n\n")
    body = ""
    for it in items:  # constants one per line, a blank line around type definitions
        body += it if it.startswith("pub const") or it.startswith("pub type") else "\n" + it
    return head + body + '\n#[link(name = "vortex_gpu")]\nextern "C" {\n' + "".join(fns) + "}\n"


def main():
    text = generate()
    if "--check" in sys.argv:
        if not OUT.exists() or OUT.read_text() != text:
            print(f"{OUT} is stale: run python tools/gen_ffi_rs.py")
            sys.exit(1)
        return
    OUT.parent.mkdir(parents=True, exist_ok=True)
    OUT.write_text(text)
    print(f"wrote {OUT} ({text.count('pub fn')} functions)")


if __name__ == "__main__":
    main()
