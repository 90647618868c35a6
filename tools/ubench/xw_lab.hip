// Cross-wave overlap of the two bounding instruction mixes (follow-up to instr5_ubench: carry writers issued by one
// wave overlap 3-source ops issued by another wave of the same SIMD, but not within one wave's stream).
//   k_fm  : every wave runs f128 multiplies (the library fe_mul, 4 independent chains)   -- NTT / evaluator mix
//   k_b3  : every wave runs BLAKE3 compressions (the library b3::compress, 2 chains)       -- row hashing / Merkle mix
//   k_mix : waves in odd slots of their SIMD run the k_fm loop, even slots the k_b3 loop (hardware HW_ID)
//   k_blk : the same split by wave index within the block (waves of one block land on different SIMDs)
// The iteration counts make k_fm and k_b3 take about the same time; if the mixes competed for one issue resource
// k_mix would take (T_fm + T_b3) / 2, if they overlapped fully max(T_fm, T_b3) / 2.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../../encrypt-zkvm_amd/csrc/blake3.hpp"

#ifndef FM_IT
#define FM_IT 1024
#endif
#ifndef B3_IT
#define B3_IT 212
#endif

__device__ __forceinline__ uint64_t fm_loop(uint32_t seed) {
    fe a[4], b = fe_make(threadIdx.x + seed, 12345);
    for (int i = 0; i < 4; i++) a[i] = fe_make(i + 1, blockIdx.x);
    for (int it = 0; it < FM_IT; it++) {
#pragma unroll
        for (int i = 0; i < 4; i++) a[i] = fe_mul(a[i], b);
    }
    uint64_t s = 0;
    for (int i = 0; i < 4; i++) s ^= a[i].lo ^ a[i].hi;
    return s;
}
__device__ __forceinline__ uint64_t b3_loop(uint32_t seed) {
    uint32_t a[8], b[8], m[16];
    for (int i = 0; i < 8; i++) { a[i] = seed + threadIdx.x * 8 + i; b[i] = a[i] ^ 0x9e3779b9u * (i + 1); }
    for (int i = 0; i < 16; i++) m[i] = blockIdx.x + i * 0x01000193u;
    for (int it = 0; it < B3_IT; it++) {
        b3::compress(a, m, 0, 0, 64, 11);
        b3::compress(b, m, 0, 0, 64, 11);
        m[it & 15] ^= a[0];
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; i++) s ^= a[i] ^ ((uint64_t)b[i] << 32);
    return s;
}
__global__ void __launch_bounds__(256) k_fm(uint64_t *out, uint32_t seed) {
    out[blockIdx.x * blockDim.x + threadIdx.x] = fm_loop(seed);
}
__global__ void __launch_bounds__(256) k_b3(uint64_t *out, uint32_t seed) {
    out[blockIdx.x * blockDim.x + threadIdx.x] = b3_loop(seed);
}
__global__ void __launch_bounds__(256) k_mix(uint64_t *out, uint32_t seed) {
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 0, 4)" : "=s"(hw));  // wave slot within its SIMD
    out[blockIdx.x * blockDim.x + threadIdx.x] = (hw & 1) ? fm_loop(seed) : b3_loop(seed);
}
__global__ void __launch_bounds__(256) k_blk(uint64_t *out, uint32_t seed) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    out[blockIdx.x * blockDim.x + threadIdx.x] = (w & 1) ? fm_loop(seed) : b3_loop(seed);
}
// how the waves of the k_mix grid split: count of waves per (slot parity)
__global__ void k_census(unsigned *cnt) {
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 0, 4)" : "=s"(hw));
    if ((threadIdx.x & 63) == 0) atomicAdd(&cnt[hw & 1], 1u);
}
typedef void (*kfn)(uint64_t *, uint32_t);
static float tk(kfn k, uint64_t *out, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r && ms < best) best = ms;
    }
    return best;
}
int main() {
    const int blocks = 256 * 8;  // 8 waves per SIMD
    uint64_t *out;
    unsigned *cnt;
    if (hipMalloc(&out, sizeof(uint64_t) * blocks * 256) != hipSuccess || hipMalloc(&cnt, 8) != hipSuccess) return 1;
    (void)hipMemset(cnt, 0, 8);
    hipLaunchKernelGGL(k_census, dim3(blocks), dim3(256), 0, 0, cnt);
    unsigned c[2];
    (void)hipMemcpy(c, cnt, 8, hipMemcpyDeviceToHost);
    const float fm = tk(k_fm, out, blocks), b3 = tk(k_b3, out, blocks), mix = tk(k_mix, out, blocks), blk = tk(k_blk, out, blocks);
    printf("waves in odd / even SIMD slots: %u / %u\n", c[1], c[0]);
    printf("fe_mul only   %.3f ms\nblake3 only   %.3f ms\n", fm, b3);
    printf("mixed by SIMD slot   %.3f ms  (competing: %.3f, overlapped: %.3f)\n", mix, (fm + b3) / 2, (fm > b3 ? fm : b3) / 2);
    printf("mixed by block wave  %.3f ms\n", blk);
    return 0;
}
