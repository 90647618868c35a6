# Generates instr5_ubench.hip: do the two instruction classes the prove path is bound by share one issue
# resource?  The NTT / evaluator stream is carry writers and 64-bit MADs (~1.7 slots each back to back), the
# BLAKE3 stream is 3-source ops (v_add3_u32, v_alignbit_b32, ~2 slots).  Each class alone, then alternated 1:1
# in one wave's stream (mix_*), or split over the waves of a SIMD (xw_*: waves in even slots of a SIMD one class, odd slots the other): a mixed cost near the mean of the two says they compete for the same slots (fusing the
# row hash into the evaluator would gain nothing); a cost near 1 says they overlap.  Run from tools/ubench.
tests = {
 "add_u32":          ["v_add_u32_e32 %{i}, %{i}, %8"]*8,
 "add3_u32":         ["v_add3_u32 %{i}, %{i}, %8, %{i}"]*8,
 "alignbit_rot":     ["v_alignbit_b32 %{i}, %{i}, %{i}, 16"]*8,
 "xor_b32":          ["v_xor_b32 %{i}, %{i}, %8"]*8,
 "add_co":           ["v_add_co_u32 %{i}, s[{s}:{s1}], %{i}, %8"]*8,
 "addc_co":          ["v_addc_co_u32 %{i}, s[{s}:{s1}], %{i}, 0, s[{s}:{s1}]"]*8,
 "mad_u64_u32":      ["v_mad_u64_u32 {A}, s[{s}:{s1}], %8, %8, {A}"]*8,
 "mix_addco_xor":    ["v_add_co_u32 %{i}, s[{s}:{s1}], %{i}, %8", "v_xor_b32 %{i}, %{i}, %8"]*4,
 "mix_addco_add3":   ["v_add_co_u32 %{i}, s[{s}:{s1}], %{i}, %8", "v_add3_u32 %{i}, %{i}, %8, %{i}"]*4,
 "mix_addco_align":  ["v_add_co_u32 %{i}, s[{s}:{s1}], %{i}, %8", "v_alignbit_b32 %{i}, %{i}, %{i}, 16"]*4,
 "mix_addc_add3":    ["v_addc_co_u32 %{i}, s[{s}:{s1}], %{i}, 0, s[{s}:{s1}]", "v_add3_u32 %{i}, %{i}, %8, %{i}"]*4,
 "mix_mad_add3":     ["v_mad_u64_u32 {A}, s[{s}:{s1}], %8, %8, {A}", "v_add3_u32 %{j}, %{j}, %8, %{j}"]*4,
 "mix_mad_align":    ["v_mad_u64_u32 {A}, s[{s}:{s1}], %8, %8, {A}", "v_alignbit_b32 %{j}, %{j}, %{j}, 16"]*4,
 "mix_mad_xor":      ["v_mad_u64_u32 {A}, s[{s}:{s1}], %8, %8, {A}", "v_xor_b32 %{j}, %{j}, %8"]*4,
 "mix_add3_xor":     ["v_add3_u32 %{i}, %{i}, %8, %{i}", "v_xor_b32 %{i}, %{i}, %8"]*4,
}
src = ['#include <hip/hip_runtime.h>', '#include <stdio.h>', '#include <stdint.h>', '#define ITERS 4096']
for name, ins in tests.items():
    body = []
    wide = any("{A}" in t for t in ins)
    for k, t in enumerate(ins):
        s = 40 + 2 * (k % 6)
        body.append(t.format(A=f"%{(k//2)%4}", s=s, s1=s+1, j=4 + (k//2)%4, i=k % 8))
    asm = "\\n\\t".join(body)
    if wide:
        decl = ("uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; "
                "uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;")
    else:
        decl = "uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;"
    src.append(f'''__global__ void k_{name}(uint64_t *out, uint32_t seed) {{
    {decl}
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {{
        asm volatile("{asm}" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }}
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}}''')
xw = {
 "xw_addco_xor":   ("v_add_co_u32 %{i}, s[{s}:{s1}], %{i}, %8", "v_xor_b32 %{i}, %{i}, %8", False),
 "xw_addco_add3":  ("v_add_co_u32 %{i}, s[{s}:{s1}], %{i}, %8", "v_add3_u32 %{i}, %{i}, %8, %{i}", False),
 "xw_addco_align": ("v_add_co_u32 %{i}, s[{s}:{s1}], %{i}, %8", "v_alignbit_b32 %{i}, %{i}, %{i}, 16", False),
 "xw_mad_add3":    ("v_mad_u64_u32 {A}, s[{s}:{s1}], %8, %8, {A}", "v_add3_u32 %{j}, %{j}, %8, %{j}", True),
 "xw_mad_xor":     ("v_mad_u64_u32 {A}, s[{s}:{s1}], %8, %8, {A}", "v_xor_b32 %{j}, %{j}, %8", True),
}
for name, (ta, tb, wide) in xw.items():
    def body(t):
        return "\\n\\t".join(t.format(A=f"%{(k//2)%4}", s=40 + 2 * (k % 6), s1=41 + 2 * (k % 6), j=4 + (k//2)%4, i=k % 8) for k in range(8))
    if wide:
        decl = ("uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; "
                "uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;")
    else:
        decl = "uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;"
    ops = '"+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51"'
    src.append(f"""__global__ void k_{name}(uint64_t *out, uint32_t seed) {{
    {decl}
    uint32_t x = seed | 1;
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 0, 4)" : "=s"(hw));  // wave slot within its SIMD
    if (hw & 1) {{
        for (int it = 0; it < ITERS; it++) asm volatile("{body(ta)}" : {ops});
    }} else {{
        for (int it = 0; it < ITERS; it++) asm volatile("{body(tb)}" : {ops});
    }}
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}}""")
tests.update({k: None for k in xw})
src.append('typedef void (*kfn)(uint64_t *, uint32_t);')
src.append('''static float tk(kfn k, uint64_t *out, int blocks) {
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 4; r++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); if (r && ms < best) best = ms;
    }
    return best;
}''')
src.append('int main() { uint64_t *out; (void)hipMalloc(&out, sizeof(uint64_t) * 256 * 8 * 256); const int blocks = 256 * 8;')
src.append('  float base = tk(k_add_u32, out, blocks);')
src.append('  printf("slots per instruction (v_add_u32 = 1), 8 waves per SIMD\\n");')
for name in tests:
    src.append(f'  printf("%-16s %.2f\\n", "{name}", tk(k_{name}, out, blocks) / base);')
src.append('  return 0; }')
open("instr5_ubench.hip", "w").write("\n".join(src) + "\n")
