#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 4096
__global__ void k_add_u32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_u32_e32 %0, %0, %8\n\tv_add_u32_e32 %1, %1, %8\n\tv_add_u32_e32 %2, %2, %8\n\tv_add_u32_e32 %3, %3, %8\n\tv_add_u32_e32 %4, %4, %8\n\tv_add_u32_e32 %5, %5, %8\n\tv_add_u32_e32 %6, %6, %8\n\tv_add_u32_e32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mul_u32_u24(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mul_u32_u24 %0, %0, %8\n\tv_mul_u32_u24 %1, %1, %8\n\tv_mul_u32_u24 %2, %2, %8\n\tv_mul_u32_u24 %3, %3, %8\n\tv_mul_u32_u24 %4, %4, %8\n\tv_mul_u32_u24 %5, %5, %8\n\tv_mul_u32_u24 %6, %6, %8\n\tv_mul_u32_u24 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mul_hi_u32_u24(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mul_hi_u32_u24 %0, %0, %8\n\tv_mul_hi_u32_u24 %1, %1, %8\n\tv_mul_hi_u32_u24 %2, %2, %8\n\tv_mul_hi_u32_u24 %3, %3, %8\n\tv_mul_hi_u32_u24 %4, %4, %8\n\tv_mul_hi_u32_u24 %5, %5, %8\n\tv_mul_hi_u32_u24 %6, %6, %8\n\tv_mul_hi_u32_u24 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mad_u32_u24(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mad_u32_u24 %0, %0, %8, %0\n\tv_mad_u32_u24 %1, %1, %8, %1\n\tv_mad_u32_u24 %2, %2, %8, %2\n\tv_mad_u32_u24 %3, %3, %8, %3\n\tv_mad_u32_u24 %4, %4, %8, %4\n\tv_mad_u32_u24 %5, %5, %8, %5\n\tv_mad_u32_u24 %6, %6, %8, %6\n\tv_mad_u32_u24 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mul_lo_u32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mul_lo_u32 %0, %0, %8\n\tv_mul_lo_u32 %1, %1, %8\n\tv_mul_lo_u32 %2, %2, %8\n\tv_mul_lo_u32 %3, %3, %8\n\tv_mul_lo_u32 %4, %4, %8\n\tv_mul_lo_u32 %5, %5, %8\n\tv_mul_lo_u32 %6, %6, %8\n\tv_mul_lo_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_and_b32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_and_b32 %0, %0, %8\n\tv_and_b32 %1, %1, %8\n\tv_and_b32 %2, %2, %8\n\tv_and_b32 %3, %3, %8\n\tv_and_b32 %4, %4, %8\n\tv_and_b32 %5, %5, %8\n\tv_and_b32 %6, %6, %8\n\tv_and_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_lshr_b32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_lshrrev_b32 %0, 7, %0\n\tv_lshrrev_b32 %1, 7, %1\n\tv_lshrrev_b32 %2, 7, %2\n\tv_lshrrev_b32 %3, 7, %3\n\tv_lshrrev_b32 %4, 7, %4\n\tv_lshrrev_b32 %5, 7, %5\n\tv_lshrrev_b32 %6, 7, %6\n\tv_lshrrev_b32 %7, 7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_bfe_u32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_bfe_u32 %0, %0, 3, 22\n\tv_bfe_u32 %1, %1, 3, 22\n\tv_bfe_u32 %2, %2, 3, 22\n\tv_bfe_u32 %3, %3, 3, 22\n\tv_bfe_u32 %4, %4, 3, 22\n\tv_bfe_u32 %5, %5, 3, 22\n\tv_bfe_u32 %6, %6, 3, 22\n\tv_bfe_u32 %7, %7, 3, 22" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_lshl_or(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_lshl_or_b32 %0, %0, 3, %8\n\tv_lshl_or_b32 %1, %1, 3, %8\n\tv_lshl_or_b32 %2, %2, 3, %8\n\tv_lshl_or_b32 %3, %3, 3, %8\n\tv_lshl_or_b32 %4, %4, 3, %8\n\tv_lshl_or_b32 %5, %5, 3, %8\n\tv_lshl_or_b32 %6, %6, 3, %8\n\tv_lshl_or_b32 %7, %7, 3, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_lshrrev_b64(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_lshrrev_b64 %0, 26, %0\n\tv_lshrrev_b64 %0, 26, %0\n\tv_lshrrev_b64 %1, 26, %1\n\tv_lshrrev_b64 %1, 26, %1\n\tv_lshrrev_b64 %2, 26, %2\n\tv_lshrrev_b64 %2, 26, %2\n\tv_lshrrev_b64 %3, 26, %3\n\tv_lshrrev_b64 %3, 26, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_lshl_add_u64(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %0\n\tv_lshl_add_u64 %0, %0, 0, %0\n\tv_lshl_add_u64 %1, %1, 0, %1\n\tv_lshl_add_u64 %1, %1, 0, %1\n\tv_lshl_add_u64 %2, %2, 0, %2\n\tv_lshl_add_u64 %2, %2, 0, %2\n\tv_lshl_add_u64 %3, %3, 0, %3\n\tv_lshl_add_u64 %3, %3, 0, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_fma_f64(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_fma_f64 %0, %0, %0, %0\n\tv_fma_f64 %0, %0, %0, %0\n\tv_fma_f64 %1, %1, %1, %1\n\tv_fma_f64 %1, %1, %1, %1\n\tv_fma_f64 %2, %2, %2, %2\n\tv_fma_f64 %2, %2, %2, %2\n\tv_fma_f64 %3, %3, %3, %3\n\tv_fma_f64 %3, %3, %3, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_add_f64(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_f64 %0, %0, %0\n\tv_add_f64 %0, %0, %0\n\tv_add_f64 %1, %1, %1\n\tv_add_f64 %1, %1, %1\n\tv_add_f64 %2, %2, %2\n\tv_add_f64 %2, %2, %2\n\tv_add_f64 %3, %3, %3\n\tv_add_f64 %3, %3, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mul_f64(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mul_f64 %0, %0, %0\n\tv_mul_f64 %0, %0, %0\n\tv_mul_f64 %1, %1, %1\n\tv_mul_f64 %1, %1, %1\n\tv_mul_f64 %2, %2, %2\n\tv_mul_f64 %2, %2, %2\n\tv_mul_f64 %3, %3, %3\n\tv_mul_f64 %3, %3, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_pk_fma_f32(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_pk_fma_f32 %0, %0, %0, %0\n\tv_pk_fma_f32 %0, %0, %0, %0\n\tv_pk_fma_f32 %1, %1, %1, %1\n\tv_pk_fma_f32 %1, %1, %1, %1\n\tv_pk_fma_f32 %2, %2, %2, %2\n\tv_pk_fma_f32 %2, %2, %2, %2\n\tv_pk_fma_f32 %3, %3, %3, %3\n\tv_pk_fma_f32 %3, %3, %3, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_fma_f32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_fma_f32 %0, %0, %8, %0\n\tv_fma_f32 %1, %1, %8, %1\n\tv_fma_f32 %2, %2, %8, %2\n\tv_fma_f32 %3, %3, %8, %3\n\tv_fma_f32 %4, %4, %8, %4\n\tv_fma_f32 %5, %5, %8, %5\n\tv_fma_f32 %6, %6, %8, %6\n\tv_fma_f32 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_cvt_f64_u32(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_cvt_f64_u32 %0, %4\n\tv_cvt_f64_u32 %0, %4\n\tv_cvt_f64_u32 %1, %5\n\tv_cvt_f64_u32 %1, %5\n\tv_cvt_f64_u32 %2, %6\n\tv_cvt_f64_u32 %2, %6\n\tv_cvt_f64_u32 %3, %7\n\tv_cvt_f64_u32 %3, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_dot2_u32_u16(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_dot2_u32_u16 %0, %0, %8, %0\n\tv_dot2_u32_u16 %1, %1, %8, %1\n\tv_dot2_u32_u16 %2, %2, %8, %2\n\tv_dot2_u32_u16 %3, %3, %8, %3\n\tv_dot2_u32_u16 %4, %4, %8, %4\n\tv_dot2_u32_u16 %5, %5, %8, %5\n\tv_dot2_u32_u16 %6, %6, %8, %6\n\tv_dot2_u32_u16 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mad_u64_u32(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_mad_u64_u32 %0, s[42:43], %8, %8, %0\n\tv_mad_u64_u32 %1, s[44:45], %8, %8, %1\n\tv_mad_u64_u32 %1, s[46:47], %8, %8, %1\n\tv_mad_u64_u32 %2, s[48:49], %8, %8, %2\n\tv_mad_u64_u32 %2, s[50:51], %8, %8, %2\n\tv_mad_u64_u32 %3, s[40:41], %8, %8, %3\n\tv_mad_u64_u32 %3, s[42:43], %8, %8, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_mul24_xor(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mul_u32_u24 %0, %0, %8\n\tv_xor_b32 %1, %1, %8\n\tv_mul_u32_u24 %2, %2, %8\n\tv_xor_b32 %3, %3, %8\n\tv_mul_u32_u24 %4, %4, %8\n\tv_xor_b32 %5, %5, %8\n\tv_mul_u32_u24 %6, %6, %8\n\tv_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_mulhi24_lo(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mul_hi_u32_u24 %0, %0, %8\n\tv_mul_u32_u24 %1, %1, %8\n\tv_mul_hi_u32_u24 %2, %2, %8\n\tv_mul_u32_u24 %3, %3, %8\n\tv_mul_hi_u32_u24 %4, %4, %8\n\tv_mul_u32_u24 %5, %5, %8\n\tv_mul_hi_u32_u24 %6, %6, %8\n\tv_mul_u32_u24 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_fma64_xor(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_fma_f64 %0, %0, %0, %0\n\tv_xor_b32 %4, %4, %8\n\tv_fma_f64 %1, %1, %1, %1\n\tv_xor_b32 %5, %5, %8\n\tv_fma_f64 %2, %2, %2, %2\n\tv_xor_b32 %6, %6, %8\n\tv_fma_f64 %3, %3, %3, %3\n\tv_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_add64_xor(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %0\n\tv_xor_b32 %4, %4, %8\n\tv_lshl_add_u64 %1, %1, 0, %1\n\tv_xor_b32 %5, %5, %8\n\tv_lshl_add_u64 %2, %2, 0, %2\n\tv_xor_b32 %6, %6, %8\n\tv_lshl_add_u64 %3, %3, 0, %3\n\tv_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_mad_mul24(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_mul_u32_u24 %4, %4, %8\n\tv_mad_u64_u32 %1, s[44:45], %8, %8, %1\n\tv_mul_u32_u24 %5, %5, %8\n\tv_mad_u64_u32 %2, s[48:49], %8, %8, %2\n\tv_mul_u32_u24 %6, %6, %8\n\tv_mad_u64_u32 %3, s[40:41], %8, %8, %3\n\tv_mul_u32_u24 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
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
int main() { uint64_t *out; (void)hipMalloc(&out, sizeof(uint64_t) * 256 * 8 * 256); const int blocks = 256 * 8;
  float base = tk(k_add_u32, out, blocks);
  printf("%-16s %.2f\n", "add_u32", tk(k_add_u32, out, blocks) / base);
  printf("%-16s %.2f\n", "mul_u32_u24", tk(k_mul_u32_u24, out, blocks) / base);
  printf("%-16s %.2f\n", "mul_hi_u32_u24", tk(k_mul_hi_u32_u24, out, blocks) / base);
  printf("%-16s %.2f\n", "mad_u32_u24", tk(k_mad_u32_u24, out, blocks) / base);
  printf("%-16s %.2f\n", "mul_lo_u32", tk(k_mul_lo_u32, out, blocks) / base);
  printf("%-16s %.2f\n", "and_b32", tk(k_and_b32, out, blocks) / base);
  printf("%-16s %.2f\n", "lshr_b32", tk(k_lshr_b32, out, blocks) / base);
  printf("%-16s %.2f\n", "bfe_u32", tk(k_bfe_u32, out, blocks) / base);
  printf("%-16s %.2f\n", "lshl_or", tk(k_lshl_or, out, blocks) / base);
  printf("%-16s %.2f\n", "lshrrev_b64", tk(k_lshrrev_b64, out, blocks) / base);
  printf("%-16s %.2f\n", "lshl_add_u64", tk(k_lshl_add_u64, out, blocks) / base);
  printf("%-16s %.2f\n", "fma_f64", tk(k_fma_f64, out, blocks) / base);
  printf("%-16s %.2f\n", "add_f64", tk(k_add_f64, out, blocks) / base);
  printf("%-16s %.2f\n", "mul_f64", tk(k_mul_f64, out, blocks) / base);
  printf("%-16s %.2f\n", "pk_fma_f32", tk(k_pk_fma_f32, out, blocks) / base);
  printf("%-16s %.2f\n", "fma_f32", tk(k_fma_f32, out, blocks) / base);
  printf("%-16s %.2f\n", "cvt_f64_u32", tk(k_cvt_f64_u32, out, blocks) / base);
  printf("%-16s %.2f\n", "dot2_u32_u16", tk(k_dot2_u32_u16, out, blocks) / base);
  printf("%-16s %.2f\n", "mad_u64_u32", tk(k_mad_u64_u32, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_mul24_xor", tk(k_mix_mul24_xor, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_mulhi24_lo", tk(k_mix_mulhi24_lo, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_fma64_xor", tk(k_mix_fma64_xor, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_add64_xor", tk(k_mix_add64_xor, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_mad_mul24", tk(k_mix_mad_mul24, out, blocks) / base);
  return 0; }
