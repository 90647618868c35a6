// fe_mul throughput vs independent chains per thread (ILP) and waves per SIMD (W)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../encrypt-zkvm_amd/csrc/f128.hpp"
#define ITERS 1024
// cost probes (not field multiplies): the product alone, and the product plus the first fold
__device__ __forceinline__ fe probe_prod(fe a, fe b) {
    uint32_t r[8];
    mul_wide(a, b, r);
    return fe{join32(r[0] ^ r[4], r[1] ^ r[5]), join32(r[2] ^ r[6], r[3] ^ r[7])};
}
__device__ __forceinline__ fe probe_reduce(fe a, fe b) {
    return reduce_fold(lo32(a.lo), hi32(a.lo), lo32(a.hi), hi32(a.hi), lo32(b.lo), hi32(b.lo), lo32(b.hi), hi32(b.hi));
}
__device__ __forceinline__ fe probe_add(fe a, fe b) { return fe_add(a, b); }
__device__ __forceinline__ fe probe_sub(fe a, fe b) { return fe_sub(a, b); }
template <int V>
__device__ __forceinline__ fe op(fe a, fe b) {
    if constexpr (V == 0) return fe_mul(a, b);
    if constexpr (V == 1) return probe_prod(a, b);
    if constexpr (V == 2) return probe_reduce(a, b);
    if constexpr (V == 3) return probe_add(a, b);
    if constexpr (V == 4) return probe_sub(a, b);
}
template <int C, int V = 0>
__global__ void __launch_bounds__(256) k_fmul(uint64_t *out, uint32_t seed) {
    fe a[C], b = fe_make(threadIdx.x + seed, 12345);
    for (int i = 0; i < C; i++) a[i] = fe_make(i + 1, blockIdx.x);
    for (int it = 0; it < ITERS * 4 / C; it++) {
#pragma unroll
        for (int i = 0; i < C; i++) a[i] = op<V>(a[i], b);
    }
    uint64_t s = 0;
    for (int i = 0; i < C; i++) s ^= a[i].lo ^ a[i].hi;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_add(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const uint32_t x = seed;
    for (int it = 0; it < ITERS * 8; it++) {
        asm volatile(
            "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
            "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
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
int main() {
    uint64_t *out; (void)hipMalloc(&out, sizeof(uint64_t) * 256 * 8 * 256);
    for (int W : {2, 4, 8}) {
        const int blocks = 256 * W;  // W blocks of 4 waves per CU -> W waves per SIMD
        const float ta = tk(k_add, out, blocks);  // 64 Ki adds per thread
        const float t1 = tk(k_fmul<1>, out, blocks), t2 = tk(k_fmul<2>, out, blocks), t4 = tk(k_fmul<4>, out, blocks), t8 = tk(k_fmul<8>, out, blocks);
        // 4096 fe_mul per thread; express as v_add_u32-equivalents per fe_mul (peak-normalised)
        auto u = [&](float t) { return t / ta * 65536.0 / 4096.0; };
        printf("W=%d  add %.3f ms | fe_mul add-equiv per mul: ILP1 %.1f  ILP2 %.1f  ILP4 %.1f  ILP8 %.1f\n", W, ta, u(t1), u(t2), u(t4), u(t8));
        if (W == 8) {
            printf("   ILP4: product %.1f  reduce_fold %.1f  fe_add %.1f  fe_sub %.1f\n", u(tk(k_fmul<4, 1>, out, blocks)),
                   u(tk(k_fmul<4, 2>, out, blocks)), u(tk(k_fmul<4, 3>, out, blocks)), u(tk(k_fmul<4, 4>, out, blocks)));
        }
    }
    return 0;
}
