# Generates instr3_ubench.hip: issue cost of carry-writing (W) instructions back to back vs interleaved
# with plain VGPR instructions (N), per 8-instruction iteration, relative to v_add_u32.  Run from tools/ubench.
W = "v_add_co_u32_e64 %{i}, s[{s}:{s1}], %{i}, %8"
N = "v_add_u32_e32 %{i}, %{i}, %8"
Cn = "v_cndmask_b32_e64 %{i}, %{i}, %8, s[50:51]"
M = "v_mad_u64_u32 %{A}, s[{s}:{s1}], %8, %8, %{A}"
tests = {
 "ref_add":  [N]*8,
 "W8":       [W]*8,
 "W1N1":     [W, N]*4,
 "W2N1":     [W, W, N, W, W, N, W, W],
 "W1N2":     [W, N, N, W, N, N, W, N],
 "W1Cnd1":   [W, Cn]*4,
 "Cnd8":     [Cn]*8,
 "N_only4":  [N]*4,
}
src = ['#include <hip/hip_runtime.h>', '#include <stdio.h>', '#include <stdint.h>', '#define ITERS 4096']
for name, ins in tests.items():
    body = []
    for k, t in enumerate(ins):
        s = 40 + 2 * (k % 5)
        body.append(t.format(s=s, s1=s+1, i=k % 8, A=k % 4))
    asm = "\\n\\t".join(body)
    src.append(f'''__global__ void k_{name}(uint64_t *out, uint32_t seed) {{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[50:51], -1" ::: "s50", "s51");
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
    for (int r = 0; r < 5; r++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); if (r && ms < best) best = ms;
    }
    return best;
}''')
src.append('int main() { uint64_t *out; (void)hipMalloc(&out, sizeof(uint64_t) * 256 * 8 * 256); const int blocks = 256 * 8;')
src.append('  float base = tk(k_ref_add, out, blocks) / 8;  // per instruction')
for name, ins in tests.items():
    src.append(f'  printf("%-10s %d instr: %.2f add-equivalents per iteration\\n", "{name}", {len(ins)}, tk(k_{name}, out, blocks) / base);')
src.append('  return 0; }')
open("instr3_ubench.hip", "w").write("\n".join(src) + "\n")
