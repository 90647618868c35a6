# Generates instr2_ubench.hip: issue cost of VALU instruction classes (encoding, SGPR writes, 3-source ops)
# and of two-instruction mixes, each relative to v_add_u32.  Run from tools/ubench.
tests = {
 "add_u32_e32":    ["v_add_u32_e32 %{i}, %{i}, %8"]*8,
 "add_u32_e64":    ["v_add_u32_e64 %{i}, %{i}, %8"]*8,
 "xor_b32":        ["v_xor_b32 %{i}, %{i}, %8"]*8,
 "alignbit":       ["v_alignbit_b32 %{i}, %{i}, %{i}, 7"]*8,
 "add3":           ["v_add3_u32 %{i}, %{i}, %8, %8"]*8,
 "addco_e64_nodep":["v_add_co_u32_e64 %{i}, s[{s}:{s1}], %{i}, %8"]*8,
 "cndmask_e32":    ["v_cndmask_b32_e32 %{i}, %{i}, %8, vcc"]*8,
 "cmp_e64":        ["v_cmp_lt_u32_e64 s[{s}:{s1}], %{i}, %8"]*8,
 "mix_e64_vop2":   ["v_add_u32_e64 %{i}, %{i}, %8", "v_xor_b32 %{i}, %{i}, %8"]*4,
 "mix_align_add3": ["v_alignbit_b32 %{i}, %{i}, %{i}, 7", "v_add3_u32 %{i}, %{i}, %8, %8"]*4,
 "mix_addco_align":["v_add_co_u32_e64 %{i}, s[{s}:{s1}], %{i}, %8", "v_alignbit_b32 %{i}, %{i}, %{i}, 7"]*4,
 "mix_addco_xor":  ["v_add_co_u32_e64 %{i}, s[{s}:{s1}], %{i}, %8", "v_xor_b32 %{i}, %{i}, %8"]*4,
 "mix_align_xor":  ["v_alignbit_b32 %{i}, %{i}, %{i}, 7", "v_xor_b32 %{i}, %{i}, %8"]*4,
 "mix_mad_xor":    ["v_mad_u64_u32 {A}, s[{s}:{s1}], %8, %8, {A}", "v_xor_b32 %{j}, %{j}, %8"]*4,
 "mad_u64_sgpr":   ["v_mad_u64_u32 {A}, s[{s}:{s1}], %8, %8, {A}"]*8,
}
src = ['#include <hip/hip_runtime.h>', '#include <stdio.h>', '#include <stdint.h>', '#define ITERS 4096']
for name, ins in tests.items():
    body = []
    mad = any("{A}" in t for t in ins)
    for k, t in enumerate(ins):
        s = 40 + 2 * (k % 6)
        body.append(t.format(A=f"%{(k//2)%4}", s=s, s1=s+1, j=4 + (k//2)%4, i=k % 8))
    asm = "\\n\\t".join(body)
    if mad:
        decl = "uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4, a5 = 5, a6 = 6, a7 = 7;"
    else:
        decl = "uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;"
    src.append(f'''__global__ void k_{name}(uint64_t *out, uint32_t seed) {{
    {decl}
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 vcc, -1" ::: "vcc");
    for (int it = 0; it < ITERS; it++) {{
        asm volatile("{asm}" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }}
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}}''')
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
src.append('  float base = tk(k_add_u32_e32, out, blocks);')
for name in tests:
    src.append(f'  printf("%-16s %.2f\\n", "{name}", tk(k_{name}, out, blocks) / base);')
src.append('  return 0; }')
open("instr2_ubench.hip", "w").write("\n".join(src) + "\n")
