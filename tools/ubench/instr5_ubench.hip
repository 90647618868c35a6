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
__global__ void k_add3_u32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add3_u32 %0, %0, %8, %0\n\tv_add3_u32 %1, %1, %8, %1\n\tv_add3_u32 %2, %2, %8, %2\n\tv_add3_u32 %3, %3, %8, %3\n\tv_add3_u32 %4, %4, %8, %4\n\tv_add3_u32 %5, %5, %8, %5\n\tv_add3_u32 %6, %6, %8, %6\n\tv_add3_u32 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_alignbit_rot(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_alignbit_b32 %0, %0, %0, 16\n\tv_alignbit_b32 %1, %1, %1, 16\n\tv_alignbit_b32 %2, %2, %2, 16\n\tv_alignbit_b32 %3, %3, %3, 16\n\tv_alignbit_b32 %4, %4, %4, 16\n\tv_alignbit_b32 %5, %5, %5, 16\n\tv_alignbit_b32 %6, %6, %6, 16\n\tv_alignbit_b32 %7, %7, %7, 16" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_xor_b32(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_xor_b32 %0, %0, %8\n\tv_xor_b32 %1, %1, %8\n\tv_xor_b32 %2, %2, %8\n\tv_xor_b32 %3, %3, %8\n\tv_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %8\n\tv_xor_b32 %6, %6, %8\n\tv_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_add_co(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32 %0, s[40:41], %0, %8\n\tv_add_co_u32 %1, s[42:43], %1, %8\n\tv_add_co_u32 %2, s[44:45], %2, %8\n\tv_add_co_u32 %3, s[46:47], %3, %8\n\tv_add_co_u32 %4, s[48:49], %4, %8\n\tv_add_co_u32 %5, s[50:51], %5, %8\n\tv_add_co_u32 %6, s[40:41], %6, %8\n\tv_add_co_u32 %7, s[42:43], %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_addc_co(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_addc_co_u32 %0, s[40:41], %0, 0, s[40:41]\n\tv_addc_co_u32 %1, s[42:43], %1, 0, s[42:43]\n\tv_addc_co_u32 %2, s[44:45], %2, 0, s[44:45]\n\tv_addc_co_u32 %3, s[46:47], %3, 0, s[46:47]\n\tv_addc_co_u32 %4, s[48:49], %4, 0, s[48:49]\n\tv_addc_co_u32 %5, s[50:51], %5, 0, s[50:51]\n\tv_addc_co_u32 %6, s[40:41], %6, 0, s[40:41]\n\tv_addc_co_u32 %7, s[42:43], %7, 0, s[42:43]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
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
__global__ void k_mix_addco_xor(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32 %0, s[40:41], %0, %8\n\tv_xor_b32 %1, %1, %8\n\tv_add_co_u32 %2, s[44:45], %2, %8\n\tv_xor_b32 %3, %3, %8\n\tv_add_co_u32 %4, s[48:49], %4, %8\n\tv_xor_b32 %5, %5, %8\n\tv_add_co_u32 %6, s[40:41], %6, %8\n\tv_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_addco_add3(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32 %0, s[40:41], %0, %8\n\tv_add3_u32 %1, %1, %8, %1\n\tv_add_co_u32 %2, s[44:45], %2, %8\n\tv_add3_u32 %3, %3, %8, %3\n\tv_add_co_u32 %4, s[48:49], %4, %8\n\tv_add3_u32 %5, %5, %8, %5\n\tv_add_co_u32 %6, s[40:41], %6, %8\n\tv_add3_u32 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_addco_align(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add_co_u32 %0, s[40:41], %0, %8\n\tv_alignbit_b32 %1, %1, %1, 16\n\tv_add_co_u32 %2, s[44:45], %2, %8\n\tv_alignbit_b32 %3, %3, %3, 16\n\tv_add_co_u32 %4, s[48:49], %4, %8\n\tv_alignbit_b32 %5, %5, %5, 16\n\tv_add_co_u32 %6, s[40:41], %6, %8\n\tv_alignbit_b32 %7, %7, %7, 16" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_addc_add3(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_addc_co_u32 %0, s[40:41], %0, 0, s[40:41]\n\tv_add3_u32 %1, %1, %8, %1\n\tv_addc_co_u32 %2, s[44:45], %2, 0, s[44:45]\n\tv_add3_u32 %3, %3, %8, %3\n\tv_addc_co_u32 %4, s[48:49], %4, 0, s[48:49]\n\tv_add3_u32 %5, %5, %8, %5\n\tv_addc_co_u32 %6, s[40:41], %6, 0, s[40:41]\n\tv_add3_u32 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_mad_add3(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_add3_u32 %4, %4, %8, %4\n\tv_mad_u64_u32 %1, s[44:45], %8, %8, %1\n\tv_add3_u32 %5, %5, %8, %5\n\tv_mad_u64_u32 %2, s[48:49], %8, %8, %2\n\tv_add3_u32 %6, %6, %8, %6\n\tv_mad_u64_u32 %3, s[40:41], %8, %8, %3\n\tv_add3_u32 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_mad_align(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_alignbit_b32 %4, %4, %4, 16\n\tv_mad_u64_u32 %1, s[44:45], %8, %8, %1\n\tv_alignbit_b32 %5, %5, %5, 16\n\tv_mad_u64_u32 %2, s[48:49], %8, %8, %2\n\tv_alignbit_b32 %6, %6, %6, 16\n\tv_mad_u64_u32 %3, s[40:41], %8, %8, %3\n\tv_alignbit_b32 %7, %7, %7, 16" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_mad_xor(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_xor_b32 %4, %4, %8\n\tv_mad_u64_u32 %1, s[44:45], %8, %8, %1\n\tv_xor_b32 %5, %5, %8\n\tv_mad_u64_u32 %2, s[48:49], %8, %8, %2\n\tv_xor_b32 %6, %6, %8\n\tv_mad_u64_u32 %3, s[40:41], %8, %8, %3\n\tv_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_mix_add3_xor(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        asm volatile("v_add3_u32 %0, %0, %8, %0\n\tv_xor_b32 %1, %1, %8\n\tv_add3_u32 %2, %2, %8, %2\n\tv_xor_b32 %3, %3, %8\n\tv_add3_u32 %4, %4, %8, %4\n\tv_xor_b32 %5, %5, %8\n\tv_add3_u32 %6, %6, %8, %6\n\tv_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_xw_addco_xor(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 0, 4)" : "=s"(hw));  // wave slot within its SIMD
    if (hw & 1) {
        for (int it = 0; it < ITERS; it++) asm volatile("v_add_co_u32 %0, s[40:41], %0, %8\n\tv_add_co_u32 %1, s[42:43], %1, %8\n\tv_add_co_u32 %2, s[44:45], %2, %8\n\tv_add_co_u32 %3, s[46:47], %3, %8\n\tv_add_co_u32 %4, s[48:49], %4, %8\n\tv_add_co_u32 %5, s[50:51], %5, %8\n\tv_add_co_u32 %6, s[40:41], %6, %8\n\tv_add_co_u32 %7, s[42:43], %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    } else {
        for (int it = 0; it < ITERS; it++) asm volatile("v_xor_b32 %0, %0, %8\n\tv_xor_b32 %1, %1, %8\n\tv_xor_b32 %2, %2, %8\n\tv_xor_b32 %3, %3, %8\n\tv_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %8\n\tv_xor_b32 %6, %6, %8\n\tv_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_xw_addco_add3(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 0, 4)" : "=s"(hw));  // wave slot within its SIMD
    if (hw & 1) {
        for (int it = 0; it < ITERS; it++) asm volatile("v_add_co_u32 %0, s[40:41], %0, %8\n\tv_add_co_u32 %1, s[42:43], %1, %8\n\tv_add_co_u32 %2, s[44:45], %2, %8\n\tv_add_co_u32 %3, s[46:47], %3, %8\n\tv_add_co_u32 %4, s[48:49], %4, %8\n\tv_add_co_u32 %5, s[50:51], %5, %8\n\tv_add_co_u32 %6, s[40:41], %6, %8\n\tv_add_co_u32 %7, s[42:43], %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    } else {
        for (int it = 0; it < ITERS; it++) asm volatile("v_add3_u32 %0, %0, %8, %0\n\tv_add3_u32 %1, %1, %8, %1\n\tv_add3_u32 %2, %2, %8, %2\n\tv_add3_u32 %3, %3, %8, %3\n\tv_add3_u32 %4, %4, %8, %4\n\tv_add3_u32 %5, %5, %8, %5\n\tv_add3_u32 %6, %6, %8, %6\n\tv_add3_u32 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_xw_addco_align(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t x = seed | 1;
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 0, 4)" : "=s"(hw));  // wave slot within its SIMD
    if (hw & 1) {
        for (int it = 0; it < ITERS; it++) asm volatile("v_add_co_u32 %0, s[40:41], %0, %8\n\tv_add_co_u32 %1, s[42:43], %1, %8\n\tv_add_co_u32 %2, s[44:45], %2, %8\n\tv_add_co_u32 %3, s[46:47], %3, %8\n\tv_add_co_u32 %4, s[48:49], %4, %8\n\tv_add_co_u32 %5, s[50:51], %5, %8\n\tv_add_co_u32 %6, s[40:41], %6, %8\n\tv_add_co_u32 %7, s[42:43], %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    } else {
        for (int it = 0; it < ITERS; it++) asm volatile("v_alignbit_b32 %0, %0, %0, 16\n\tv_alignbit_b32 %1, %1, %1, 16\n\tv_alignbit_b32 %2, %2, %2, 16\n\tv_alignbit_b32 %3, %3, %3, 16\n\tv_alignbit_b32 %4, %4, %4, 16\n\tv_alignbit_b32 %5, %5, %5, 16\n\tv_alignbit_b32 %6, %6, %6, 16\n\tv_alignbit_b32 %7, %7, %7, 16" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_xw_mad_add3(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 0, 4)" : "=s"(hw));  // wave slot within its SIMD
    if (hw & 1) {
        for (int it = 0; it < ITERS; it++) asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_mad_u64_u32 %0, s[42:43], %8, %8, %0\n\tv_mad_u64_u32 %1, s[44:45], %8, %8, %1\n\tv_mad_u64_u32 %1, s[46:47], %8, %8, %1\n\tv_mad_u64_u32 %2, s[48:49], %8, %8, %2\n\tv_mad_u64_u32 %2, s[50:51], %8, %8, %2\n\tv_mad_u64_u32 %3, s[40:41], %8, %8, %3\n\tv_mad_u64_u32 %3, s[42:43], %8, %8, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    } else {
        for (int it = 0; it < ITERS; it++) asm volatile("v_add3_u32 %4, %4, %8, %4\n\tv_add3_u32 %4, %4, %8, %4\n\tv_add3_u32 %5, %5, %8, %5\n\tv_add3_u32 %5, %5, %8, %5\n\tv_add3_u32 %6, %6, %8, %6\n\tv_add3_u32 %6, %6, %8, %6\n\tv_add3_u32 %7, %7, %8, %7\n\tv_add3_u32 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
__global__ void k_xw_mad_xor(uint64_t *out, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a4 = 4 + threadIdx.x, a5 = 5, a6 = 6, a7 = 7;
    uint32_t x = seed | 1;
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 0, 4)" : "=s"(hw));  // wave slot within its SIMD
    if (hw & 1) {
        for (int it = 0; it < ITERS; it++) asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_mad_u64_u32 %0, s[42:43], %8, %8, %0\n\tv_mad_u64_u32 %1, s[44:45], %8, %8, %1\n\tv_mad_u64_u32 %1, s[46:47], %8, %8, %1\n\tv_mad_u64_u32 %2, s[48:49], %8, %8, %2\n\tv_mad_u64_u32 %2, s[50:51], %8, %8, %2\n\tv_mad_u64_u32 %3, s[40:41], %8, %8, %3\n\tv_mad_u64_u32 %3, s[42:43], %8, %8, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
    } else {
        for (int it = 0; it < ITERS; it++) asm volatile("v_xor_b32 %4, %4, %8\n\tv_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %8\n\tv_xor_b32 %5, %5, %8\n\tv_xor_b32 %6, %6, %8\n\tv_xor_b32 %6, %6, %8\n\tv_xor_b32 %7, %7, %8\n\tv_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51");
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
  printf("slots per instruction (v_add_u32 = 1), 8 waves per SIMD\n");
  printf("%-16s %.2f\n", "add_u32", tk(k_add_u32, out, blocks) / base);
  printf("%-16s %.2f\n", "add3_u32", tk(k_add3_u32, out, blocks) / base);
  printf("%-16s %.2f\n", "alignbit_rot", tk(k_alignbit_rot, out, blocks) / base);
  printf("%-16s %.2f\n", "xor_b32", tk(k_xor_b32, out, blocks) / base);
  printf("%-16s %.2f\n", "add_co", tk(k_add_co, out, blocks) / base);
  printf("%-16s %.2f\n", "addc_co", tk(k_addc_co, out, blocks) / base);
  printf("%-16s %.2f\n", "mad_u64_u32", tk(k_mad_u64_u32, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_addco_xor", tk(k_mix_addco_xor, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_addco_add3", tk(k_mix_addco_add3, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_addco_align", tk(k_mix_addco_align, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_addc_add3", tk(k_mix_addc_add3, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_mad_add3", tk(k_mix_mad_add3, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_mad_align", tk(k_mix_mad_align, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_mad_xor", tk(k_mix_mad_xor, out, blocks) / base);
  printf("%-16s %.2f\n", "mix_add3_xor", tk(k_mix_add3_xor, out, blocks) / base);
  printf("%-16s %.2f\n", "xw_addco_xor", tk(k_xw_addco_xor, out, blocks) / base);
  printf("%-16s %.2f\n", "xw_addco_add3", tk(k_xw_addco_add3, out, blocks) / base);
  printf("%-16s %.2f\n", "xw_addco_align", tk(k_xw_addco_align, out, blocks) / base);
  printf("%-16s %.2f\n", "xw_mad_add3", tk(k_xw_mad_add3, out, blocks) / base);
  printf("%-16s %.2f\n", "xw_mad_xor", tk(k_xw_mad_xor, out, blocks) / base);
  return 0; }
