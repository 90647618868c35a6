// Microbenchmark: VALU issue cost (cycles per wave64 instruction per SIMD) of the instruction
// classes the f128 multiply is made of, measured with s_memtime (shader clock) inside the loop.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 issue_ubench.hip -o issue_ubench
// Every kernel runs W waves per SIMD (blocks of 256 threads, B blocks per CU) and reports
//   cyc/instr = (loop cycles of a wave) * (waves per SIMD) / (instructions of a wave)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../../encrypt-zkvm_amd/csrc/f128.hpp"

#define ITERS 2048

__global__ void k_add(uint64_t *out, uint64_t *cyc, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const uint32_t x = seed;
    uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; it++) {
        asm volatile(
            "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
            "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x));
    }
    uint64_t t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_mad(uint64_t *out, uint64_t *cyc, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    const uint32_t x = seed, y = threadIdx.x * 7;
    uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; it++) {
        asm volatile(
            "v_mad_u64_u32 %0, s[40:41], %4, %5, %0\n\tv_mad_u64_u32 %1, s[42:43], %4, %5, %1\n\t"
            "v_mad_u64_u32 %2, s[44:45], %4, %5, %2\n\tv_mad_u64_u32 %3, s[46:47], %4, %5, %3\n\t"
            "v_mad_u64_u32 %0, s[40:41], %4, %5, %0\n\tv_mad_u64_u32 %1, s[42:43], %4, %5, %1\n\t"
            "v_mad_u64_u32 %2, s[44:45], %4, %5, %2\n\tv_mad_u64_u32 %3, s[46:47], %4, %5, %3\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(y) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    }
    uint64_t t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// 64-bit add with carry chain through VCC: add_co then addc (two independent 64-bit accumulators x4)
__global__ void k_addc(uint64_t *out, uint64_t *cyc, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const uint32_t x = seed;
    uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; it++) {
        asm volatile(
            "v_add_co_u32 %0, s[40:41], %0, %8\n\tv_add_co_u32 %2, s[42:43], %2, %8\n\t"
            "v_add_co_u32 %4, s[44:45], %4, %8\n\tv_add_co_u32 %6, s[46:47], %6, %8\n\t"
            "v_addc_co_u32 %1, s[40:41], %1, 0, s[40:41]\n\tv_addc_co_u32 %3, s[42:43], %3, 0, s[42:43]\n\t"
            "v_addc_co_u32 %5, s[44:45], %5, 0, s[44:45]\n\tv_addc_co_u32 %7, s[46:47], %7, 0, s[46:47]\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(x) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    }
    uint64_t t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// v_lshl_add_u64 (64-bit add in one instruction)
__global__ void k_add64(uint64_t *out, uint64_t *cyc, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const uint64_t x = seed;
    uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; it++) {
        asm volatile(
            "v_lshl_add_u64 %0, %0, 0, %8\n\tv_lshl_add_u64 %1, %1, 0, %8\n\tv_lshl_add_u64 %2, %2, 0, %8\n\t"
            "v_lshl_add_u64 %3, %3, 0, %8\n\tv_lshl_add_u64 %4, %4, 0, %8\n\tv_lshl_add_u64 %5, %5, 0, %8\n\t"
            "v_lshl_add_u64 %6, %6, 0, %8\n\tv_lshl_add_u64 %7, %7, 0, %8\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x));
    }
    uint64_t t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// v_mov_b64 (one 64-bit move)
__global__ void k_mov64(uint64_t *out, uint64_t *cyc, uint32_t seed) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint64_t t0 = clock64();
    for (int it = 0; it < ITERS; it++) {
        asm volatile(
            "v_mov_b64 %0, %1\n\tv_mov_b64 %1, %2\n\tv_mov_b64 %2, %3\n\tv_mov_b64 %3, %0\n\t"
            "v_mov_b64 %0, %1\n\tv_mov_b64 %1, %2\n\tv_mov_b64 %2, %3\n\tv_mov_b64 %3, %0\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    }
    uint64_t t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ seed;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_fmul(uint64_t *out, uint64_t *cyc, uint32_t seed) {
    fe a[4], b = fe_make(threadIdx.x + seed, 12345);
    for (int i = 0; i < 4; i++) a[i] = fe_make(i + 1, blockIdx.x);
    uint64_t t0 = clock64();
    for (int it = 0; it < ITERS / 16; it++) {
#pragma unroll
        for (int i = 0; i < 4; i++) a[i] = fe_mul(a[i], b);
    }
    uint64_t t1 = clock64();
    uint64_t s = 0;
    for (int i = 0; i < 4; i++) s ^= a[i].lo ^ a[i].hi;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

typedef void (*kfn)(uint64_t *, uint64_t *, uint32_t);
static void run(const char *name, kfn k, double instr_per_wave, int blocks_per_cu, uint64_t *out, uint64_t *cyc) {
    const int blocks = 256 * blocks_per_cu;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, cyc, 1u);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, cyc, 3u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    static uint64_t h[256 * 64];
    hipMemcpy(h, cyc, sizeof(uint64_t) * blocks, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks; i++) mean += (double)h[i];
    mean /= blocks;
    const double waves_per_simd = blocks_per_cu * 4.0 / 4.0;  // 4 waves per block, 4 SIMDs per CU
    printf("%-10s W=%2.0f  %7.3f ms  loop %9.0f cyc/wave  %.2f cyc per wave-instr per SIMD  (clock %.2f GHz)\n", name,
           waves_per_simd, ms, mean, mean / instr_per_wave * 1.0 / waves_per_simd * 1.0, mean / (ms * 1e6));
}

int main() {
    uint64_t *out, *cyc;
    hipMalloc(&out, sizeof(uint64_t) * 256 * 64 * 256);
    hipMalloc(&cyc, sizeof(uint64_t) * 256 * 64);
    for (int bpc : {2, 4, 8}) {
        run("add_u32", k_add, ITERS * 8.0, bpc, out, cyc);
        run("mad_u64", k_mad, ITERS * 8.0, bpc, out, cyc);
        run("addc", k_addc, ITERS * 8.0, bpc, out, cyc);
        run("lshl_add64", k_add64, ITERS * 8.0, bpc, out, cyc);
        run("mov_b64", k_mov64, ITERS * 8.0, bpc, out, cyc);
        run("fe_mul", k_fmul, ITERS / 16 * 4.0, bpc, out, cyc);  // cyc per fe_mul
    }
    return 0;
}
