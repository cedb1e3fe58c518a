"""Static ISA statistics of the kernels in a hipcc --save-temps assembly file: instruction
counts (all, VALU, SALU, scalar loads, LDS, barriers, MFMA) and the spill traffic (v_writelane /
v_readlane of SGPR spills, scratch accesses of VGPR spills), plus the compiler's own resource
remarks (.sgpr_spill_count / .vgpr_spill_count in the metadata).

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -c --save-temps -o x.o csrc/pesq.hip
    python tools/isa_stats.py pesq-hip-amdgcn-amd-amdhsa-gfx950.s [name-filter]
"""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(\w+):\s*;\s*@\1\s*$", text, re.M):
        name = m.group(1)
        end = text.find(".Lfunc_end", m.end())
        yield name, text[m.end():end]


def stats(body):
    ins = [ln.strip() for ln in body.split("\n")]
    ins = [ln for ln in ins if ln and not ln.startswith((".", ";")) and not ln.endswith(":")]

    def cnt(p):
        r = re.compile(p)
        return sum(1 for ln in ins if r.match(ln))

    return {
        "instr": len(ins),
        "valu": cnt(r"v_(?!mfma|readlane|writelane|readfirstlane)"),
        "mfma": cnt(r"v_mfma"),
        "salu": cnt(r"s_(?!load|buffer_load|waitcnt|barrier|nop|cbranch|branch|endpgm|setprio)"),
        "s_load": cnt(r"s_(load|buffer_load)"),
        "lds": cnt(r"ds_"),
        "barrier": cnt(r"s_barrier"),
        "writelane": cnt(r"v_writelane"),
        "readlane": cnt(r"v_readlane"),
        "scratch": cnt(r"scratch_|buffer_(store|load)_dword\w* v\d+, off"),
    }


def resources(text):
    """name -> the compiler's resource metadata (amdhsa.kernels: registers, spills, LDS, scratch)."""
    out = {}
    i = text.find("amdhsa.kernels:")
    if i < 0:
        return out
    for entry in re.split(r"\n  - ", text[i:]):
        m = re.search(r"^\s+\.name:\s+(\S+)", entry, re.M)
        if not m:
            continue
        r = {}
        for key in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                    "group_segment_fixed_size", "private_segment_fixed_size"):
            k = re.search(r"\." + key + r":\s+(\d+)", entry)
            if k:
                r[key] = int(k.group(1))
        out[m.group(1)] = r
    return out


def main():
    text = open(sys.argv[1]).read()
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    res = resources(text)
    short = {"vgpr_count": "vgpr", "agpr_count": "agpr", "sgpr_count": "sgpr", "vgpr_spill_count": "vgpr_spill",
             "sgpr_spill_count": "sgpr_spill", "group_segment_fixed_size": "lds_bytes",
             "private_segment_fixed_size": "scratch_bytes"}
    for name, body in kernels(text):
        if filt not in name:
            continue
        s = stats(body)
        print(name[:90])
        print("   " + "  ".join(f"{k} {v}" for k, v in s.items()))
        if name in res:
            print("   " + "  ".join(f"{short[k]} {v}" for k, v in res[name].items()))


if __name__ == "__main__":
    main()
