#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 4096
__global__ void k_v_add_u32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\tv_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_mov_b32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mov_b32 %0, %1\n\tv_mov_b32 %1, %2\n\tv_mov_b32 %2, %3\n\tv_mov_b32 %3, %4\n\tv_mov_b32 %4, %5\n\tv_mov_b32 %5, %6\n\tv_mov_b32 %6, %7\n\tv_mov_b32 %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_add_co_e32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32 %0, vcc, %0, %8\n\tv_add_co_u32 %1, vcc, %1, %8\n\tv_add_co_u32 %2, vcc, %2, %8\n\tv_add_co_u32 %3, vcc, %3, %8\n\tv_add_co_u32 %4, vcc, %4, %8\n\tv_add_co_u32 %5, vcc, %5, %8\n\tv_add_co_u32 %6, vcc, %6, %8\n\tv_add_co_u32 %7, vcc, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_add_co_e64s(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32 %0, s[40:41], %0, %8\n\tv_add_co_u32 %1, s[42:43], %1, %8\n\tv_add_co_u32 %2, s[44:45], %2, %8\n\tv_add_co_u32 %3, s[46:47], %3, %8\n\tv_add_co_u32 %4, s[40:41], %4, %8\n\tv_add_co_u32 %5, s[42:43], %5, %8\n\tv_add_co_u32 %6, s[44:45], %6, %8\n\tv_add_co_u32 %7, s[46:47], %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_addc_e32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_addc_co_u32 %0, vcc, %0, %8, vcc\n\tv_addc_co_u32 %1, vcc, %1, %8, vcc\n\tv_addc_co_u32 %2, vcc, %2, %8, vcc\n\tv_addc_co_u32 %3, vcc, %3, %8, vcc\n\tv_addc_co_u32 %4, vcc, %4, %8, vcc\n\tv_addc_co_u32 %5, vcc, %5, %8, vcc\n\tv_addc_co_u32 %6, vcc, %6, %8, vcc\n\tv_addc_co_u32 %7, vcc, %7, %8, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_addc_e64s(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_addc_co_u32 %0, s[40:41], %0, %8, s[40:41]\n\tv_addc_co_u32 %1, s[42:43], %1, %8, s[42:43]\n\tv_addc_co_u32 %2, s[44:45], %2, %8, s[44:45]\n\tv_addc_co_u32 %3, s[46:47], %3, %8, s[46:47]\n\tv_addc_co_u32 %4, s[40:41], %4, %8, s[40:41]\n\tv_addc_co_u32 %5, s[42:43], %5, %8, s[42:43]\n\tv_addc_co_u32 %6, s[44:45], %6, %8, s[44:45]\n\tv_addc_co_u32 %7, s[46:47], %7, %8, s[46:47]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_addc_e64_in(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_addc_co_u32 %0, s[40:41], %0, 0, s[48:49]\n\tv_addc_co_u32 %1, s[42:43], %1, 0, s[48:49]\n\tv_addc_co_u32 %2, s[44:45], %2, 0, s[48:49]\n\tv_addc_co_u32 %3, s[46:47], %3, 0, s[48:49]\n\tv_addc_co_u32 %4, s[40:41], %4, 0, s[48:49]\n\tv_addc_co_u32 %5, s[42:43], %5, 0, s[48:49]\n\tv_addc_co_u32 %6, s[44:45], %6, 0, s[48:49]\n\tv_addc_co_u32 %7, s[46:47], %7, 0, s[48:49]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_cndmask_e64(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_cndmask_b32 %0, %0, %8, s[48:49]\n\tv_cndmask_b32 %1, %1, %8, s[48:49]\n\tv_cndmask_b32 %2, %2, %8, s[48:49]\n\tv_cndmask_b32 %3, %3, %8, s[48:49]\n\tv_cndmask_b32 %4, %4, %8, s[48:49]\n\tv_cndmask_b32 %5, %5, %8, s[48:49]\n\tv_cndmask_b32 %6, %6, %8, s[48:49]\n\tv_cndmask_b32 %7, %7, %8, s[48:49]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_mad_u64(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_mad_u64_u32 %1, s[42:43], %8, %8, %1\n\tv_mad_u64_u32 %2, s[44:45], %8, %8, %2\n\tv_mad_u64_u32 %3, s[46:47], %8, %8, %3\n\tv_mad_u64_u32 %4, s[40:41], %8, %8, %4\n\tv_mad_u64_u32 %5, s[42:43], %8, %8, %5\n\tv_mad_u64_u32 %6, s[44:45], %8, %8, %6\n\tv_mad_u64_u32 %7, s[46:47], %8, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_mad_u64_nc(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mad_u64_u32 %0, s[50:51], %8, %8, %0\n\tv_mad_u64_u32 %1, s[50:51], %8, %8, %1\n\tv_mad_u64_u32 %2, s[50:51], %8, %8, %2\n\tv_mad_u64_u32 %3, s[50:51], %8, %8, %3\n\tv_mad_u64_u32 %4, s[50:51], %8, %8, %4\n\tv_mad_u64_u32 %5, s[50:51], %8, %8, %5\n\tv_mad_u64_u32 %6, s[50:51], %8, %8, %6\n\tv_mad_u64_u32 %7, s[50:51], %8, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_mul_lo_u32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mul_lo_u32 %0, %0, %8\n\tv_mul_lo_u32 %1, %1, %8\n\tv_mul_lo_u32 %2, %2, %8\n\tv_mul_lo_u32 %3, %3, %8\n\tv_mul_lo_u32 %4, %4, %8\n\tv_mul_lo_u32 %5, %5, %8\n\tv_mul_lo_u32 %6, %6, %8\n\tv_mul_lo_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_mul_hi_u32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mul_hi_u32 %0, %0, %8\n\tv_mul_hi_u32 %1, %1, %8\n\tv_mul_hi_u32 %2, %2, %8\n\tv_mul_hi_u32 %3, %3, %8\n\tv_mul_hi_u32 %4, %4, %8\n\tv_mul_hi_u32 %5, %5, %8\n\tv_mul_hi_u32 %6, %6, %8\n\tv_mul_hi_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_add3_u32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add3_u32 %0, %0, %8, %1\n\tv_add3_u32 %1, %1, %8, %2\n\tv_add3_u32 %2, %2, %8, %3\n\tv_add3_u32 %3, %3, %8, %4\n\tv_add3_u32 %4, %4, %8, %5\n\tv_add3_u32 %5, %5, %8, %6\n\tv_add3_u32 %6, %6, %8, %7\n\tv_add3_u32 %7, %7, %8, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_mov_b64(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mov_b64 %0, %1\n\tv_mov_b64 %1, %2\n\tv_mov_b64 %2, %3\n\tv_mov_b64 %3, %4\n\tv_mov_b64 %4, %5\n\tv_mov_b64 %5, %6\n\tv_mov_b64 %6, %7\n\tv_mov_b64 %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_v_lshl_add_u64(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49", "s50", "s51");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1\n\tv_lshl_add_u64 %1, %1, 0, %2\n\tv_lshl_add_u64 %2, %2, 0, %3\n\tv_lshl_add_u64 %3, %3, 0, %4\n\tv_lshl_add_u64 %4, %4, 0, %5\n\tv_lshl_add_u64 %5, %5, 0, %6\n\tv_lshl_add_u64 %6, %6, 0, %7\n\tv_lshl_add_u64 %7, %7, 0, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_mad_add(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t x = seed | 1, y = threadIdx.x, z = seed ^ 5, w = 7;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mad_u64_u32 %0, s[40:41], %7, %4, %0\n\tv_add_u32 %5, %5, %7\n\tv_mad_u64_u32 %1, s[42:43], %7, %4, %1\n\tv_add_u32 %6, %6, %7\n\tv_mad_u64_u32 %2, s[44:45], %7, %4, %2\n\tv_add_u32 %5, %5, %7\n\tv_mad_u64_u32 %3, s[46:47], %7, %4, %3\n\tv_add_u32 %6, %6, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(y), "+v"(z), "+v"(w), "+v"(x) :
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ x ^ y ^ z ^ w);
}
__global__ void k_mix_addc_add(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t x = seed | 1, y = threadIdx.x, z = seed ^ 5, w = 7;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_addc_co_u32 %0, s[40:41], %0, %7, s[40:41]\n\tv_add_u32 %5, %5, %7\n\tv_addc_co_u32 %1, s[42:43], %1, %7, s[42:43]\n\tv_add_u32 %6, %6, %7\n\tv_addc_co_u32 %2, s[44:45], %2, %7, s[44:45]\n\tv_add_u32 %5, %5, %7\n\tv_addc_co_u32 %3, s[46:47], %3, %7, s[46:47]\n\tv_add_u32 %6, %6, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(y), "+v"(z), "+v"(w), "+v"(x) :
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ x ^ y ^ z ^ w);
}
__global__ void k_mix_mad_addc(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t x = seed | 1, y = threadIdx.x, z = seed ^ 5, w = 7;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mad_u64_u32 %0, s[40:41], %7, %4, %0\n\tv_addc_co_u32 %5, s[50:51], %5, %7, s[50:51]\n\tv_mad_u64_u32 %1, s[42:43], %7, %4, %1\n\tv_addc_co_u32 %6, s[52:53], %6, %7, s[52:53]\n\tv_mad_u64_u32 %2, s[44:45], %7, %4, %2\n\tv_addc_co_u32 %5, s[50:51], %5, %7, s[50:51]\n\tv_mad_u64_u32 %3, s[46:47], %7, %4, %3\n\tv_addc_co_u32 %6, s[52:53], %6, %7, s[52:53]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(y), "+v"(z), "+v"(w), "+v"(x) :
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ x ^ y ^ z ^ w);
}
__global__ void k_mix_cnd_add(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t x = seed | 1, y = threadIdx.x, z = seed ^ 5, w = 7;
    asm volatile("s_mov_b64 s[48:49], -1" ::: "s48", "s49");
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_cndmask_b32 %0, %0, %7, s[48:49]\n\tv_xor_b32 %5, %5, %0\n\tv_cndmask_b32 %1, %1, %7, s[48:49]\n\tv_xor_b32 %6, %6, %1\n\tv_cndmask_b32 %2, %2, %7, s[48:49]\n\tv_xor_b32 %5, %5, %2\n\tv_cndmask_b32 %3, %3, %7, s[48:49]\n\tv_xor_b32 %6, %6, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(y), "+v"(z), "+v"(w), "+v"(x) :
                     : "vcc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ x ^ y ^ z ^ w);
}
#include "../../encrypt-zkvm_amd/csrc/f128.hpp"
__global__ void k_fe_mul(uint64_t *out, uint32_t seed) {
    fe a[4], b = fe_make(threadIdx.x + seed, 12345);
    for (int i = 0; i < 4; i++) a[i] = fe_make(i + 1, blockIdx.x);
    for (int it = 0; it < ITERS / 4; it++) {
#pragma unroll
        for (int i = 0; i < 4; i++) a[i] = fe_mul(a[i], b);
    }
    uint64_t s = 0;
    for (int i = 0; i < 4; i++) s ^= a[i].lo ^ a[i].hi;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
typedef void (*kfn)(uint64_t *, uint32_t);
static float tk(kfn k, uint64_t *out, int blocks) {
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 4; r++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); if (r && ms < best) best = ms;
    }
    return best;
}
int main() { uint64_t *out; (void)hipMalloc(&out, sizeof(uint64_t) * 256 * 8 * 256 * 2); const int blocks = 256 * 8;
  double n = (double)blocks * 4 * ITERS * 8; float base = tk(k_v_add_u32, out, blocks);
  { float t = tk(k_v_add_u32, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_add_u32", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_mov_b32, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_mov_b32", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_add_co_e32, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_add_co_e32", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_add_co_e64s, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_add_co_e64s", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_addc_e32, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_addc_e32", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_addc_e64s, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_addc_e64s", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_addc_e64_in, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_addc_e64_in", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_cndmask_e64, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_cndmask_e64", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_mad_u64, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_mad_u64", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_mad_u64_nc, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_mad_u64_nc", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_mul_lo_u32, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_mul_lo_u32", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_mul_hi_u32, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_mul_hi_u32", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_add3_u32, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_add3_u32", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_mov_b64, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_mov_b64", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_v_lshl_add_u64, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32  %.1f G wave-instr/s per SIMD\n", "v_lshl_add_u64", t, t / base, n / 1024 / (t * 1e6)); }
  { float t = tk(k_mix_mad_add, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32 (8 instr)\n", "mix_mad_add", t, t / base); }
  { float t = tk(k_mix_addc_add, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32 (8 instr)\n", "mix_addc_add", t, t / base); }
  { float t = tk(k_mix_mad_addc, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32 (8 instr)\n", "mix_mad_addc", t, t / base); }
  { float t = tk(k_mix_cnd_add, out, blocks); printf("%-16s %8.4f ms  %.2f x v_add_u32 (8 instr)\n", "mix_cnd_add", t, t / base); }
  { float t = tk(k_fe_mul, out, blocks); printf("%-16s %8.4f ms  %.2f v_add_u32 per fe_mul\n", "fe_mul", t, t / base * 8.0); }
  return 0; }
