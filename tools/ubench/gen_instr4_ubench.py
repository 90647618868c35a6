# Generates instr4_ubench.hip: issue cost (relative to v_add_u32) of the instructions an unsaturated-limb or an
# FP64 f128 multiply would be made of -- 24-bit multiplies, 64-bit shifts and adds, FP64 FMA, packed FP32, dot
# products -- alone and interleaved 1:1 with plain VGPR instructions.  Run from tools/ubench.
tests = {
 "add_u32":        ["v_add_u32_e32 %{i}, %{i}, %8"]*8,
 "mul_u32_u24":    ["v_mul_u32_u24 %{i}, %{i}, %8"]*8,
 "mul_hi_u32_u24": ["v_mul_hi_u32_u24 %{i}, %{i}, %8"]*8,
 "mad_u32_u24":    ["v_mad_u32_u24 %{i}, %{i}, %8, %{i}"]*8,
 "mul_lo_u32":     ["v_mul_lo_u32 %{i}, %{i}, %8"]*8,
 "and_b32":        ["v_and_b32 %{i}, %{i}, %8"]*8,
 "lshr_b32":       ["v_lshrrev_b32 %{i}, 7, %{i}"]*8,
 "bfe_u32":        ["v_bfe_u32 %{i}, %{i}, 3, 22"]*8,
 "lshl_or":        ["v_lshl_or_b32 %{i}, %{i}, 3, %8"]*8,
 "lshrrev_b64":    ["v_lshrrev_b64 {A}, 26, {A}"]*8,
 "lshl_add_u64":   ["v_lshl_add_u64 {A}, {A}, 0, {A}"]*8,
 "fma_f64":        ["v_fma_f64 {A}, {A}, {A}, {A}"]*8,
 "add_f64":        ["v_add_f64 {A}, {A}, {A}"]*8,
 "mul_f64":        ["v_mul_f64 {A}, {A}, {A}"]*8,
 "pk_fma_f32":     ["v_pk_fma_f32 {A}, {A}, {A}, {A}"]*8,
 "fma_f32":        ["v_fma_f32 %{i}, %{i}, %8, %{i}"]*8,
 "cvt_f64_u32":    ["v_cvt_f64_u32 {A}, %{j}"]*8,
 "dot2_u32_u16":   ["v_dot2_u32_u16 %{i}, %{i}, %8, %{i}"]*8,
 "mad_u64_u32":    ["v_mad_u64_u32 {A}, s[{s}:{s1}], %8, %8, {A}"]*8,
 "mix_mul24_xor":  ["v_mul_u32_u24 %{i}, %{i}, %8", "v_xor_b32 %{i}, %{i}, %8"]*4,
 "mix_mulhi24_lo": ["v_mul_hi_u32_u24 %{i}, %{i}, %8", "v_mul_u32_u24 %{i}, %{i}, %8"]*4,
 "mix_fma64_xor":  ["v_fma_f64 {A}, {A}, {A}, {A}", "v_xor_b32 %{j}, %{j}, %8"]*4,
 "mix_add64_xor":  ["v_lshl_add_u64 {A}, {A}, 0, {A}", "v_xor_b32 %{j}, %{j}, %8"]*4,
 "mix_mad_mul24":  ["v_mad_u64_u32 {A}, s[{s}:{s1}], %8, %8, {A}", "v_mul_u32_u24 %{j}, %{j}, %8"]*4,
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
for name in tests:
    src.append(f'  printf("%-16s %.2f\\n", "{name}", tk(k_{name}, out, blocks) / base);')
src.append('  return 0; }')
open("instr4_ubench.hip", "w").write("\n".join(src) + "\n")
