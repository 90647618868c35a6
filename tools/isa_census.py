"""Instruction census of the gfx950 NTT kernels ("Carry chains").

Compiles csrc/kernels.hip to gfx950 assembly (device only, the library's flags) and counts, per kernel, the
instruction lines by class: VALU, hazard s_nop (and the wait states they request), LDS, barriers, waitcnt, SALU,
scalar / vector memory.  The carry-chain hazards show up as s_nop: a VALU carry write read by the next VALU needs
wait states the compiler fills with s_nop when nothing independent is scheduled between them.
    python3 tools/isa_census.py [--defs "-DX=1 ..."] [--asm /tmp/k.s] [kernel-regex ...]
Prints one JSON object {kernel: {class: count}}.
"""
import json
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "encrypt-zkvm_amd" / "csrc" / "kernels.hip"
DEFAULT = [r"ntt_pass1ILi10ELi4096ELb1E", r"ntt_pass1ILi10ELi4096ELb0E", r"ntt_pass2ILi10ELi4096E"]


def compile_asm(defs, out):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           *defs.split(), str(SRC), "-o", out]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)


def census(lines):
    c = {"lines": 0, "valu": 0, "s_nop": 0, "nop_wait_states": 0, "lds": 0, "barrier": 0, "waitcnt": 0, "salu": 0,
         "smem": 0, "vmem": 0, "v_mad_u64_u32": 0, "carry_ops": 0, "cndmask": 0}
    for ln in lines:
        t = ln.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c["lines"] += 1
        if op == "s_nop":
            c["s_nop"] += 1
            c["nop_wait_states"] += int(t.split()[1], 0) + 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op == "s_barrier":
            c["barrier"] += 1
        elif op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif op.startswith(("s_load", "s_buffer_load")):
            c["smem"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
            if op.startswith("v_mad_u64_u32"):
                c["v_mad_u64_u32"] += 1
            if re.match(r"v_(add|addc|sub|subb|subrev|subbrev)_co_u32", op):
                c["carry_ops"] += 1
            if op.startswith("v_cndmask"):
                c["cndmask"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c


def main():
    args = sys.argv[1:]
    defs, asm = "", None
    if "--defs" in args:
        i = args.index("--defs")
        defs = args[i + 1]
        del args[i:i + 2]
    if "--asm" in args:
        i = args.index("--asm")
        asm = args[i + 1]
        del args[i:i + 2]
    pats = args or DEFAULT
    if asm is None or not Path(asm).exists():
        asm = asm or "/tmp/zk_kernels_census.s"
        compile_asm(defs, asm)
    text = Path(asm).read_text().splitlines()
    out = {}
    for pat in pats:
        for i, ln in enumerate(text):
            m = re.match(r"^(_Z\w+):", ln)
            if not m or not re.search(pat, m.group(1)):
                continue
            end = next(j for j in range(i + 1, len(text)) if text[j].startswith(".Lfunc_end"))
            out[m.group(1)] = census(text[i + 1:end])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
