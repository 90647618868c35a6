"""Generate encrypt-zkvm_amd/csrc/addsub_asm.hpp: two radix-2 butterflies' sums and differences mod p,
(a + b, a - b, c + d, c - d), as one inline-asm block whose four carry chains are interleaved by a list scheduler.

Why ("Carry chains"): the compiler emits each fe_add / fe_sub as its own carry chain through
VCC, one chain at a time, and pads every carry hand-off with s_nop (gfx950: a VALU carry write must be 2 wait states
ahead of the VALU that reads it) -- 523 of ntt_pass2's 3,095 lines.  Four independent chains with their own SGPR
pairs fill each other's wait states instead.  The subtraction also drops one lane-mask select: on a borrow the
result is d + p (mod 2^128), whose low limb is d0 + borrow (the borrow itself as carry-in) and whose other limbs
add the mask-selected words of p, so one v_cndmask builds the mask instead of two.

The scheduler checks every hazard it relies on (asserted again on the emitted sequence):
  VALU writes an SGPR -> a VALU reads it:   >= 2 wait states between them
  SALU writes an SGPR -> a VALU reads it:   >= 1
  VALU writes an SGPR -> a SALU reads it:   0   (as hipcc's own carry code does)
and fills a gap with s_nop only when no independent instruction is ready.
    python3 tools/gen_addsub_asm.py            (rewrites the header; prints the instruction census)
"""
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "encrypt-zkvm_amd" / "csrc" / "addsub_asm.hpp"

P_LIMB1 = 0xFFFFD300  # p = 2^128 - 45 2^40 + 1: limbs (1, 0xffffd300, 0xffffffff, 0xffffffff)


class Ins:
    def __init__(self, text, vdst=(), vsrc=(), sdst=(), ssrc=(), salu=False):
        self.text, self.vdst, self.vsrc, self.sdst, self.ssrc, self.salu = text, vdst, vsrc, sdst, ssrc, salu


def build(lazy_ab, lazy_cd):
    """Instruction DAG for apb = a + b, amb = a - b, cpd = c + d, cmd = c - d (in place: the sums land in a / c,
    the differences in fresh registers S / D, b and d are clobbered)."""
    ins = []

    def add_chain(x, y, carry, tag, lazy, tmp):
        # s = x + y into x (x_k is read by the subtraction first: the caller orders that)
        for k in range(4):
            op = "v_add_co_u32 {%s%d}, {%s}, {%s%d}, {%s%d}" % (x, k, carry, x, k, y, k) if k == 0 else \
                 "v_addc_co_u32 {%s%d}, {%s}, {%s%d}, {%s%d}, {%s}" % (x, k, carry, x, k, y, k, carry)
            ins.append(Ins(op, vdst=(f"{x}{k}",), vsrc=(f"{x}{k}", f"{y}{k}"), sdst=(carry,),
                           ssrc=((carry,) if k else ()), salu=False))
            ins[-1].tag = (tag, "s", k)
        if lazy:
            # one fold on carry: s + C = s - p (mod 2^128), C = 0x2cff_ffffffff, into x
            m, pm = tmp
            ins.append(Ins("v_cndmask_b32_e64 {%s}, 0, -1, {%s}" % (m, carry), vdst=(m,), ssrc=(carry,)))
            ins.append(Ins("v_and_b32 {%s}, 0x2cff, {%s}" % (pm, m), vdst=(pm,), vsrc=(m,)))
            for k in range(4):
                src = {0: m, 1: pm}.get(k)
                if k == 0:
                    op = "v_add_co_u32 {%s0}, {%s}, {%s0}, {%s}" % (x, carry, x, m)
                    ins.append(Ins(op, vdst=(f"{x}0",), vsrc=(f"{x}0", m), sdst=(carry,)))
                elif src:
                    op = "v_addc_co_u32 {%s%d}, {%s}, {%s%d}, {%s}, {%s}" % (x, k, carry, x, k, src, carry)
                    ins.append(Ins(op, vdst=(f"{x}{k}",), vsrc=(f"{x}{k}", src), sdst=(carry,), ssrc=(carry,)))
                else:
                    op = "v_addc_co_u32 {%s%d}, {%s}, {%s%d}, 0, {%s}" % (x, k, carry, x, k, carry)
                    ins.append(Ins(op, vdst=(f"{x}{k}",), vsrc=(f"{x}{k}",), sdst=(carry,), ssrc=(carry,)))
        else:
            # t = s + C into y (y is dead once both chains read it); s >= p <=> carry(s) or carry(t); select into x
            c2 = carry + "t"
            for k in range(4):
                if k == 0:
                    op = "v_add_co_u32 {%s0}, {%s}, {%s0}, -1" % (y, c2, x)
                    ins.append(Ins(op, vdst=(f"{y}0",), vsrc=(f"{x}0",), sdst=(c2,)))
                elif k == 1:
                    op = "v_addc_co_u32 {%s1}, {%s}, {%s1}, {C1}, {%s}" % (y, c2, x, c2)
                    ins.append(Ins(op, vdst=(f"{y}1",), vsrc=(f"{x}1", "C1"), sdst=(c2,), ssrc=(c2,)))
                else:
                    op = "v_addc_co_u32 {%s%d}, {%s}, {%s%d}, 0, {%s}" % (y, k, c2, x, k, c2)
                    ins.append(Ins(op, vdst=(f"{y}{k}",), vsrc=(f"{x}{k}",), sdst=(c2,), ssrc=(c2,)))
            ins.append(Ins("s_or_b64 {%s}, {%s}, {%s}" % (carry, carry, c2), sdst=(carry,), ssrc=(carry, c2), salu=True))
            for k in range(4):
                op = "v_cndmask_b32_e64 {%s%d}, {%s%d}, {%s%d}, {%s}" % (x, k, x, k, y, k, carry)
                ins.append(Ins(op, vdst=(f"{x}{k}",), vsrc=(f"{x}{k}", f"{y}{k}"), ssrc=(carry,)))

    def sub_chain(x, y, out, bw, tmp):
        # d = x - y into out; on borrow out += p (mod 2^128): limb 0 takes the borrow as carry-in
        for k in range(4):
            op = "v_sub_co_u32 {%s0}, {%s}, {%s0}, {%s0}" % (out, bw, x, y) if k == 0 else \
                 "v_subb_co_u32 {%s%d}, {%s}, {%s%d}, {%s%d}, {%s}" % (out, k, bw, x, k, y, k, bw)
            ins.append(Ins(op, vdst=(f"{out}{k}",), vsrc=(f"{x}{k}", f"{y}{k}"), sdst=(bw,), ssrc=((bw,) if k else ())))
        m, pm = tmp
        ins.append(Ins("v_cndmask_b32_e64 {%s}, 0, -1, {%s}" % (m, bw), vdst=(m,), ssrc=(bw,)))
        ins.append(Ins("v_and_b32 {%s}, 0x%x, {%s}" % (pm, P_LIMB1, m), vdst=(pm,), vsrc=(m,)))
        ins.append(Ins("v_addc_co_u32 {%s0}, {%s}, {%s0}, 0, {%s}" % (out, bw, out, bw), vdst=(f"{out}0",),
                       vsrc=(f"{out}0",), sdst=(bw,), ssrc=(bw,)))
        for k in (1, 2, 3):
            src = pm if k == 1 else m
            ins.append(Ins("v_addc_co_u32 {%s%d}, {%s}, {%s%d}, {%s}, {%s}" % (out, k, bw, out, k, src, bw),
                           vdst=(f"{out}{k}",), vsrc=(f"{out}{k}", src), sdst=(bw,), ssrc=(bw,)))

    # the subtraction reads a, b first (its output goes to fresh registers); the addition then overwrites a
    sub_chain("a", "b", "S", "bS", ("mS", "pS"))
    add_chain("a", "b", "cA", "A", lazy_ab, ("b0", "b1"))
    sub_chain("c", "d", "D", "bD", ("mD", "pD"))
    add_chain("c", "d", "cC", "C", lazy_cd, ("d0", "d1"))
    return ins


def deps(ins):
    """Edges (i -> j, min_ws): j after i, with at least min_ws wait states between them."""
    edges = []
    for j, b in enumerate(ins):
        for i in range(j):
            a = ins[i]
            ws = None
            if set(a.vdst) & set(b.vsrc) or set(a.vsrc) & set(b.vdst) or set(a.vdst) & set(b.vdst):
                ws = 0
            if set(a.sdst) & set(b.ssrc):
                ws = max(ws or 0, 0 if b.salu else (1 if a.salu else 2))
            if set(a.ssrc) & set(b.sdst) or set(a.sdst) & set(b.sdst):
                ws = max(ws or 0, 0)
            if ws is not None:
                edges.append((i, j, ws))
    return edges


def schedule(ins):
    n = len(ins)
    edges = deps(ins)
    succ = [[] for _ in range(n)]
    preds = [[] for _ in range(n)]
    for i, j, ws in edges:
        succ[i].append((j, ws))
        preds[j].append((i, ws))
    # priority: longest path (in instructions + required wait states) to the end
    height = [0] * n
    for i in reversed(range(n)):
        height[i] = 1 + max([height[j] + ws for j, ws in succ[i]], default=0)
    done_at = {}  # instruction -> issue slot
    out = []
    slot = 0
    left = set(range(n))
    while left:
        ready = [i for i in left if all(p in done_at and slot - done_at[p] - 1 >= ws for p, ws in preds[i])]
        if not ready:
            out.append(None)  # one wait state
            slot += 1
            continue
        i = max(ready, key=lambda k: (height[k], -k))
        out.append(i)
        done_at[i] = slot
        slot += 1
        left.remove(i)
    # re-verify on the emitted sequence
    pos = {i: s for s, i in enumerate(out) if i is not None}
    for i, j, ws in edges:
        assert pos[j] - pos[i] - 1 >= ws, (ins[i].text, ins[j].text, ws)
    return out


def emit(name, lazy_ab, lazy_cd):
    ins = build(lazy_ab, lazy_cd)
    seq = schedule(ins)
    lines = []
    nop = 0
    for i in seq + ["end"]:
        if i is None:
            nop += 1
            continue
        if nop:
            lines.append(f"s_nop {nop - 1}")
            nop = 0
        if i != "end":
            lines.append(ins[i].text)
    # operands
    outs = [f"a{k}" for k in range(4)] + [f"b{k}" for k in range(4)] + [f"c{k}" for k in range(4)] + \
           [f"d{k}" for k in range(4)] + [f"S{k}" for k in range(4)] + [f"D{k}" for k in range(4)] + \
           ["mS", "pS", "mD", "pD", "cA", "cAt", "bS", "cC", "cCt", "bD"]
    ins_ops = ["C1"]
    num = {o: i for i, o in enumerate(outs + ins_ops)}
    used = set()
    for ln in lines:
        for o in num:
            if "{%s}" % o in ln:
                used.add(o)
    body = []
    for ln in lines:
        for o, i in sorted(num.items(), key=lambda kv: -len(kv[0])):
            ln = ln.replace("{%s}" % o, f"%{i}")
        body.append(ln)
    cons = []
    for o in outs:
        if o[0] in "abcd" and o[1:].isdigit():
            cons.append(f'"+v"({o[0]}[{o[1]}])')
        elif o[0] in "SD" and o[1:].isdigit():
            cons.append(f'"=&v"({o[0]}[{o[1]}])')
        elif o in ("mS", "pS", "mD", "pD"):
            cons.append(f'"=&v"({o})')
        else:
            cons.append(f'"=&s"({o})')
    census = {"instructions": sum(1 for x in seq if x is not None), "wait_states": sum(1 for x in seq if x is None),
              "s_nop": sum(1 for ln in lines if ln.startswith("s_nop")),
              "sgpr_touching": sum(1 for x in ins if (x.sdst or x.ssrc) and not x.salu)}
    asm = "\n".join(f'        "{ln}\\n\\t"' for ln in body[:-1]) + f'\n        "{body[-1]}"'
    fn = f"""// {name}: lazy a + b: {str(lazy_ab).lower()}, lazy c + d: {str(lazy_cd).lower()}.  {census['instructions']} instructions,
// {census['s_nop']} s_nop ({census['wait_states']} wait states), {census['sgpr_touching']} SGPR-touching VALU.
__device__ __forceinline__ void {name}(uint32_t a[4], uint32_t b[4], uint32_t c[4], uint32_t d[4], uint32_t S[4],
                                     uint32_t D[4]) {{
    uint32_t mS, pS, mD, pD;
    uint64_t cA, cAt, bS, cC, cCt, bD;
    const uint32_t C1 = 0x2cffu;
    asm({asm}
        : {', '.join(cons)}
        : "v"(C1)
        : "scc");
    (void)cAt;
    (void)cCt;
}}
"""
    return fn, census


def build_fold2():
    """Two independent ws_fold reductions (f128.hpp): (r0..r3) + (s4 + s5 2^32) 2^128 mod p, in place in r."""
    ins = []
    for X in "AB":
        R = lambda k: f"{X}{k}"  # noqa: E731
        sB, sC, sD = f"{X}sB", f"{X}sC", f"{X}sD"
        ins.append(Ins(f"v_subb_co_u32 {{{R(0)}}}, {{{sB}}}, {{{R(0)}}}, {{{X}s4}}, {{ones}}", vdst=(R(0),),
                       vsrc=(R(0), f"{X}s4"), sdst=(sB,), ssrc=("ones",)))
        ins.append(Ins(f"v_subb_co_u32 {{{R(1)}}}, {{{sB}}}, {{{R(1)}}}, {{{X}s5}}, {{{sB}}}", vdst=(R(1),),
                       vsrc=(R(1), f"{X}s5"), sdst=(sB,), ssrc=(sB,)))
        for k in (2, 3):
            ins.append(Ins(f"v_subb_co_u32 {{{R(k)}}}, {{{sB}}}, {{{R(k)}}}, 0, {{{sB}}}", vdst=(R(k),), vsrc=(R(k),),
                           sdst=(sB,), ssrc=(sB,)))
        ins.append(Ins(f"v_subb_co_u32 {{{R(4)}}}, {{{sB}}}, 0, 0, {{{sB}}}", vdst=(R(4),), sdst=(sB,), ssrc=(sB,)))
        ins.append(Ins(f"v_add_co_u32 {{{R(1)}}}, {{{sC}}}, {{{R(1)}}}, {{{X}m0}}", vdst=(R(1),), vsrc=(R(1), f"{X}m0"),
                       sdst=(sC,)))
        ins.append(Ins(f"v_addc_co_u32 {{{R(2)}}}, {{{sC}}}, {{{R(2)}}}, {{{X}m1}}, {{{sC}}}", vdst=(R(2),),
                       vsrc=(R(2), f"{X}m1"), sdst=(sC,), ssrc=(sC,)))
        for k in (3, 4):
            ins.append(Ins(f"v_addc_co_u32 {{{R(k)}}}, {{{sC}}}, {{{R(k)}}}, 0, {{{sC}}}", vdst=(R(k),), vsrc=(R(k),),
                           sdst=(sC,), ssrc=(sC,)))
        ins.append(Ins(f"v_add_u32 {{{X}n}}, -1, {{{R(4)}}}", vdst=(f"{X}n",), vsrc=(R(4),)))
        ins.append(Ins(f"v_and_b32 {{{X}c}}, 0x2cff, {{{X}n}}", vdst=(f"{X}c",), vsrc=(f"{X}n",)))
        ins.append(Ins(f"v_sub_co_u32 {{{R(0)}}}, {{{sD}}}, {{{R(0)}}}, {{{X}n}}", vdst=(R(0),), vsrc=(R(0), f"{X}n"),
                       sdst=(sD,)))
        ins.append(Ins(f"v_subb_co_u32 {{{R(1)}}}, {{{sD}}}, {{{R(1)}}}, {{{X}c}}, {{{sD}}}", vdst=(R(1),),
                       vsrc=(R(1), f"{X}c"), sdst=(sD,), ssrc=(sD,)))
        for k in (2, 3):
            ins.append(Ins(f"v_subb_co_u32 {{{R(k)}}}, {{{sD}}}, {{{R(k)}}}, 0, {{{sD}}}", vdst=(R(k),), vsrc=(R(k),),
                           sdst=(sD,), ssrc=(sD,)))
    return ins


def lines_of(ins, seq):
    lines, nop = [], 0
    for i in seq + ["end"]:
        if i is None:
            nop += 1
            continue
        if nop:
            lines.append(f"s_nop {nop - 1}")
            nop = 0
        if i != "end":
            lines.append(ins[i].text)
    return lines


def emit_fold2():
    ins = build_fold2()
    seq = schedule(ins)
    lines = lines_of(ins, seq)
    ops = []  # (name, constraint, c expression)
    for X, x in (("A", "a"), ("B", "b")):
        ops += [(f"{X}{k}", "+v", f"{x}[{k}]") for k in range(4)]
        ops += [(f"{X}4", "=&v", f"{x}4"), (f"{X}n", "=&v", f"{x}n"), (f"{X}c", "=&v", f"{x}c")]
        ops += [(f"{X}s{t}", "=&s", f"{x}s{t}") for t in "BCD"]
    ins_ops = []
    for X, x in (("A", "a"), ("B", "b")):
        ins_ops += [(f"{X}s4", "v", f"{x}s4"), (f"{X}s5", "v", f"{x}s5"), (f"{X}m0", "v", f"{x}m0"),
                    (f"{X}m1", "v", f"{x}m1")]
    ins_ops.append(("ones", "s", "ones"))
    num = {o[0]: i for i, o in enumerate(ops + ins_ops)}
    body = []
    for ln in lines:
        for o, i in sorted(num.items(), key=lambda kv: -len(kv[0])):
            ln = ln.replace("{%s}" % o, f"%{i}")
        body.append(ln)
    census = {"instructions": sum(1 for x in seq if x is not None), "wait_states": sum(1 for x in seq if x is None),
              "s_nop": sum(1 for ln in lines if ln.startswith("s_nop")),
              "sgpr_touching": sum(1 for x in ins if (x.sdst or x.ssrc) and not x.salu)}
    asm = "\n".join(f'        "{ln}\\n\\t"' for ln in body[:-1]) + f'\n        "{body[-1]}"'
    outc = ", ".join(f'"{c}"({e})' for _, c, e in ops)
    inc = ", ".join(f'"{c}"({e})' for _, c, e in ins_ops)
    fn = f"""// ws_fold2_asm: two independent ws_fold reductions (f128.hpp) interleaved.  {census['instructions']} instructions,
// {census['s_nop']} s_nop ({census['wait_states']} wait states), {census['sgpr_touching']} SGPR-touching VALU.  a, b: the low 128 bits
// in, the reduced values out; (as4, as5), (bs4, bs5): the words above 2^128 (s5 < 2^3); am0 / am1, bm0 / bm1: the
// low / high word of (s4 + 1) K + s5 K 2^32 (ws_fold's m0, m1).
__device__ __forceinline__ void ws_fold2_asm(uint32_t a[4], uint32_t as4, uint32_t as5, uint32_t am0, uint32_t am1,
                                             uint32_t b[4], uint32_t bs4, uint32_t bs5, uint32_t bm0, uint32_t bm1) {{
    uint32_t a4, an, ac, b4, bn, bc;
    uint64_t asB, asC, asD, bsB, bsC, bsD;
    const uint64_t ones = ~0ull;
#ifdef __HIP_DEVICE_COMPILE__  // (the host pass never emits this device function, but would parse "s"(ones) as x86's)
    asm({asm}
        : {outc}
        : {inc});
#endif
}}
"""
    return fn, census


def main():
    parts, cen = [], {}
    fn, c = emit_fold2()
    parts.append(fn)
    cen["ws_fold2_asm"] = c
    for name, la, lc in (("addsub2_asm_cc", False, False), ("addsub2_asm_ll", True, True),
                         ("addsub2_asm_lc", True, False)):
        fn, c = emit(name, la, lc)
        parts.append(fn)
        cen[name] = c
    hdr = f"""// addsub_asm.hpp -- GENERATED by tools/gen_addsub_asm.py; do not edit.
//
// ws_fold2_asm: two multiplies' final reductions interleaved (their carry chains fill each other's wait states).
// addsub2_asm_*: two butterflies' sums and differences mod p in one asm block: on entry a, b, c, d (32-bit limbs, little
// endian); on exit a = a + b, S = a - b, c = c + d, D = c - d (b and d clobbered).  The four carry chains run
// interleaved on their own SGPR pairs (list-scheduled; every gfx950 carry hazard checked by the generator), so
// the wait states a carry hand-off needs are filled by the other chains instead of s_nop.  Sums are canonical
// (s >= p <=> carry(a + b) or carry(a + b + C)), or lazy (< 2^128, one fold of C on carry: fe_add_lazy's
// contract, the first operand any value < 2^128, the second canonical).  Differences: d = a - b, plus p on a
// borrow (the same values as fe_sub).
#pragma once
#include <stdint.h>

"""
    OUT.write_text(hdr + "\n".join(parts))
    import json
    print(json.dumps(cen, indent=1))


if __name__ == "__main__":
    main()
