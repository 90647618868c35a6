#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 4096
__global__ void k_ref_add(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[50:51], -1" ::: "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_u32_e32 %0, %0, %8\n\tv_add_u32_e32 %1, %1, %8\n\tv_add_u32_e32 %2, %2, %8\n\tv_add_u32_e32 %3, %3, %8\n\tv_add_u32_e32 %4, %4, %8\n\tv_add_u32_e32 %5, %5, %8\n\tv_add_u32_e32 %6, %6, %8\n\tv_add_u32_e32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_W8(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[50:51], -1" ::: "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %8\n\tv_add_co_u32_e64 %1, s[42:43], %1, %8\n\tv_add_co_u32_e64 %2, s[44:45], %2, %8\n\tv_add_co_u32_e64 %3, s[46:47], %3, %8\n\tv_add_co_u32_e64 %4, s[48:49], %4, %8\n\tv_add_co_u32_e64 %5, s[40:41], %5, %8\n\tv_add_co_u32_e64 %6, s[42:43], %6, %8\n\tv_add_co_u32_e64 %7, s[44:45], %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_W1N1(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[50:51], -1" ::: "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %8\n\tv_add_u32_e32 %1, %1, %8\n\tv_add_co_u32_e64 %2, s[44:45], %2, %8\n\tv_add_u32_e32 %3, %3, %8\n\tv_add_co_u32_e64 %4, s[48:49], %4, %8\n\tv_add_u32_e32 %5, %5, %8\n\tv_add_co_u32_e64 %6, s[42:43], %6, %8\n\tv_add_u32_e32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_W2N1(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[50:51], -1" ::: "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %8\n\tv_add_co_u32_e64 %1, s[42:43], %1, %8\n\tv_add_u32_e32 %2, %2, %8\n\tv_add_co_u32_e64 %3, s[46:47], %3, %8\n\tv_add_co_u32_e64 %4, s[48:49], %4, %8\n\tv_add_u32_e32 %5, %5, %8\n\tv_add_co_u32_e64 %6, s[42:43], %6, %8\n\tv_add_co_u32_e64 %7, s[44:45], %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_W1N2(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[50:51], -1" ::: "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %8\n\tv_add_u32_e32 %1, %1, %8\n\tv_add_u32_e32 %2, %2, %8\n\tv_add_co_u32_e64 %3, s[46:47], %3, %8\n\tv_add_u32_e32 %4, %4, %8\n\tv_add_u32_e32 %5, %5, %8\n\tv_add_co_u32_e64 %6, s[42:43], %6, %8\n\tv_add_u32_e32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_W1Cnd1(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[50:51], -1" ::: "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %8\n\tv_cndmask_b32_e64 %1, %1, %8, s[50:51]\n\tv_add_co_u32_e64 %2, s[44:45], %2, %8\n\tv_cndmask_b32_e64 %3, %3, %8, s[50:51]\n\tv_add_co_u32_e64 %4, s[48:49], %4, %8\n\tv_cndmask_b32_e64 %5, %5, %8, s[50:51]\n\tv_add_co_u32_e64 %6, s[42:43], %6, %8\n\tv_cndmask_b32_e64 %7, %7, %8, s[50:51]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_Cnd8(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[50:51], -1" ::: "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_cndmask_b32_e64 %0, %0, %8, s[50:51]\n\tv_cndmask_b32_e64 %1, %1, %8, s[50:51]\n\tv_cndmask_b32_e64 %2, %2, %8, s[50:51]\n\tv_cndmask_b32_e64 %3, %3, %8, s[50:51]\n\tv_cndmask_b32_e64 %4, %4, %8, s[50:51]\n\tv_cndmask_b32_e64 %5, %5, %8, s[50:51]\n\tv_cndmask_b32_e64 %6, %6, %8, s[50:51]\n\tv_cndmask_b32_e64 %7, %7, %8, s[50:51]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_N_only4(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[50:51], -1" ::: "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_u32_e32 %0, %0, %8\n\tv_add_u32_e32 %1, %1, %8\n\tv_add_u32_e32 %2, %2, %8\n\tv_add_u32_e32 %3, %3, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
typedef void (*kfn)(uint64_t *, uint32_t);
static float tk(kfn k, uint64_t *out, int blocks) {
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); if (r && ms < best) best = ms;
    }
    return best;
}
int main() { uint64_t *out; (void)hipMalloc(&out, sizeof(uint64_t) * 256 * 8 * 256); const int blocks = 256 * 8;
  float base = tk(k_ref_add, out, blocks) / 8;  // per instruction
  printf("%-10s %d instr: %.2f add-equivalents per iteration\n", "ref_add", 8, tk(k_ref_add, out, blocks) / base);
  printf("%-10s %d instr: %.2f add-equivalents per iteration\n", "W8", 8, tk(k_W8, out, blocks) / base);
  printf("%-10s %d instr: %.2f add-equivalents per iteration\n", "W1N1", 8, tk(k_W1N1, out, blocks) / base);
  printf("%-10s %d instr: %.2f add-equivalents per iteration\n", "W2N1", 8, tk(k_W2N1, out, blocks) / base);
  printf("%-10s %d instr: %.2f add-equivalents per iteration\n", "W1N2", 8, tk(k_W1N2, out, blocks) / base);
  printf("%-10s %d instr: %.2f add-equivalents per iteration\n", "W1Cnd1", 8, tk(k_W1Cnd1, out, blocks) / base);
  printf("%-10s %d instr: %.2f add-equivalents per iteration\n", "Cnd8", 8, tk(k_Cnd8, out, blocks) / base);
  printf("%-10s %d instr: %.2f add-equivalents per iteration\n", "N_only4", 4, tk(k_N_only4, out, blocks) / base);
  return 0; }
