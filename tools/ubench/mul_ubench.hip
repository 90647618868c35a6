// Microbenchmark: throughput of v_mad_u64_u32 vs v_add_u32, and of f128 multiply variants.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 mul_ubench.hip -o mul_ubench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../encrypt-zkvm_amd/csrc/f128.hpp"

#define ITERS 4096
__global__ void k_mad(uint64_t *out, uint32_t seed) {
    uint64_t a[8];
    uint32_t x = threadIdx.x + seed, y = blockIdx.x * 7 + 3;
    for (int i = 0; i < 8; i++) a[i] = i;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) a[i] = (uint64_t)(x + i) * (y + it) + a[i];
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; i++) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_add(uint64_t *out, uint32_t seed) {
    uint32_t a[8];
    uint32_t x = threadIdx.x + seed;
    for (int i = 0; i < 8; i++) a[i] = i;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) a[i] = (a[i] ^ x) + it;
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; i++) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fmul(uint64_t *out, uint32_t seed) {
    fe a[4], b = fe_make(threadIdx.x + seed, 12345);
    for (int i = 0; i < 4; i++) a[i] = fe_make(i + 1, blockIdx.x);
    for (int it = 0; it < ITERS / 16; it++) {
#pragma unroll
        for (int i = 0; i < 4; i++) a[i] = fe_mul(a[i], b);
    }
    uint64_t s = 0;
    for (int i = 0; i < 4; i++) s ^= a[i].lo ^ a[i].hi;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fadd(uint64_t *out, uint32_t seed) {
    fe a[4], b = fe_make(threadIdx.x + seed, 12345);
    for (int i = 0; i < 4; i++) a[i] = fe_make(i + 1, blockIdx.x);
    for (int it = 0; it < ITERS / 4; it++) {
#pragma unroll
        for (int i = 0; i < 4; i++) a[i] = fe_add(a[i], b);
    }
    uint64_t s = 0;
    for (int i = 0; i < 4; i++) s ^= a[i].lo ^ a[i].hi;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fsub(uint64_t *out, uint32_t seed) {
    fe a[4], b = fe_make(threadIdx.x + seed, 12345);
    for (int i = 0; i < 4; i++) a[i] = fe_make(i + 1, blockIdx.x);
    for (int it = 0; it < ITERS / 4; it++) {
#pragma unroll
        for (int i = 0; i < 4; i++) a[i] = fe_sub(a[i], b);
    }
    uint64_t s = 0;
    for (int i = 0; i < 4; i++) s ^= a[i].lo ^ a[i].hi;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
float timeit(K k, uint64_t *out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const int blocks = 256 * 8;  // 8 blocks of 256 threads per CU
    uint64_t *out;
    hipMalloc(&out, sizeof(uint64_t) * blocks * 256);
    double lanes = (double)blocks * 256;
    float t;
    t = timeit(k_mad, out, blocks);
    printf("v_mad_u64_u32: %.3f ms, %.1f G lane-ops/s\n", t, lanes * ITERS * 8 / (t * 1e6));
    t = timeit(k_add, out, blocks);
    printf("u32 xor+add  : %.3f ms, %.1f G lane-ops/s (2 ops each)\n", t, lanes * ITERS * 8 * 2 / (t * 1e6));
    t = timeit(k_fmul, out, blocks);
    printf("fe_mul       : %.3f ms, %.2f G muls/s\n", t, lanes * (ITERS / 16) * 4 / (t * 1e6));
    t = timeit(k_fadd, out, blocks);
    printf("fe_add       : %.3f ms, %.2f G adds/s\n", t, lanes * (ITERS / 4) * 4 / (t * 1e6));
    t = timeit(k_fsub, out, blocks);
    printf("fe_sub       : %.3f ms, %.2f G subs/s\n", t, lanes * (ITERS / 4) * 4 / (t * 1e6));
    return 0;
}
