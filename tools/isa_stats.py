"""Static instruction mix of the kernels in a gfx950 assembly file (hipcc --cuda-device-only -S).

  python tools/isa_stats.py file.s [substring]      -> one line per kernel: VALU/SALU/LDS/VMEM
                                                       counts, VGPRs, SGPRs, LDS bytes, scratch
Static counts are not dynamic counts (loops), but they show where a kernel's code goes.
"""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\.Lfunc_end", text, re.S | re.M):
        yield m.group(1), m.group(2)


def meta(text, name, key):
    i = text.find(".amdhsa_kernel " + name)
    if i < 0:
        return None
    m = re.search(r"\." + key + r"\s+(\d+)", text[i: i + 4000])
    return int(m.group(1)) if m else None


def main():
    text = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, body in kernels(text):
        if sub not in name:
            continue
        ins = [ln.split()[0] for ln in body.splitlines()
               if ln.strip() and not ln.lstrip().startswith((".", ";")) and not ln.rstrip().endswith(":")
               and ":" not in ln.split()[0]]
        c = {k: sum(1 for x in ins if x.startswith(k)) for k in ("v_", "s_", "ds_", "global_", "buffer_", "flat_")}
        print(f"{name[:100]:100s} n={len(ins):5d} valu={c['v_']:5d} salu={c['s_']:5d} lds={c['ds_']:4d} "
              f"vmem={c['global_'] + c['buffer_'] + c['flat_']:4d} vgpr={meta(text, name, 'amdhsa_next_free_vgpr')} "
              f"sgpr={meta(text, name, 'amdhsa_next_free_sgpr')} lds_bytes={meta(text, name, 'amdhsa_group_segment_fixed_size')} "
              f"scratch={meta(text, name, 'amdhsa_private_segment_fixed_size')}")


if __name__ == "__main__":
    main()
