// f128 multiply variants: bit-exact check against the host multiply (random and edge operands) and
// throughput (4 independent chains per thread, 8 waves per SIMD) in v_add_u32-equivalents per multiply.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 fmul_lab.hip -o fmul_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include "../../encrypt-zkvm_amd/csrc/f128.hpp"
#include "fmul_variants.hpp"

#define NV FMUL_NVARIANTS
__device__ __forceinline__ fe vmul(int v, fe a, fe b);
template <int V>
__global__ void k_check(const fe *a, const fe *b, const WSet *w, fe *o, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) {
        uint32_t W[16];
        for (int k = 0; k < 16; k++) W[k] = w[i].w[k];
        o[i] = fmul_variant<V>(a[i], b[i], W);
    }
}
template <int V>
__global__ void __launch_bounds__(256) k_tput(uint64_t *out, uint32_t seed, const WSet *wtab) {
    fe a[4], b = fe_make(threadIdx.x + seed, 12345);
    uint32_t W[16];
    for (int k = 0; k < 16; k++) W[k] = wtab[threadIdx.x & 7].w[k] + seed;
    for (int i = 0; i < 4; i++) a[i] = fe_make(i + 1, blockIdx.x);
    for (int it = 0; it < 1024; it++) {
#pragma unroll
        for (int i = 0; i < 4; i++) a[i] = fmul_variant<V>(a[i], b, W);
    }
    uint64_t s = 0;
    for (int i = 0; i < 4; i++) s ^= a[i].lo ^ a[i].hi;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// Lower bound of an unsaturated representation: 5 limbs of 26 bits (130 bits), the 25 partial
// products accumulated per column in 64 bits (each column < 5 * 2^52, so no carry ever leaves a column: no SGPR
// carry chains), then the 9 columns normalised back to 26-bit limbs.  This is NOT a field multiply -- the reduction
// mod p (2^130 = 4C, C = 45 * 2^40 - 1, a second limb product and normalisation) and the conversion to and from the
// 4 x 32-bit storage form are left out -- so its slot count bounds the form from below.
__device__ __forceinline__ void unsat_mul_norm(uint32_t a[5], const uint32_t b[5]) {
    uint64_t col[9];
#pragma unroll
    for (int k = 0; k < 9; k++) col[k] = 0;
#pragma unroll
    for (int i = 0; i < 5; i++)
#pragma unroll
        for (int j = 0; j < 5; j++) col[i + j] += (uint64_t)a[i] * b[j];
    uint64_t carry = 0;
    uint32_t t[10];
#pragma unroll
    for (int k = 0; k < 9; k++) {
        const uint64_t c = col[k] + carry;
        t[k] = (uint32_t)c & 0x3ffffffu;
        carry = c >> 26;
    }
    t[9] = (uint32_t)carry;
    // feed the product back (a dependency chain); the high limbs are folded in with plain xors to keep them live
#pragma unroll
    for (int i = 0; i < 5; i++) a[i] = (t[i] ^ t[i + 5]) & 0x3ffffffu;
}
__global__ void __launch_bounds__(256) k_tput_unsat(uint64_t *out, uint32_t seed) {
    uint32_t a[4][5], b[5];
    for (int i = 0; i < 5; i++) b[i] = (threadIdx.x * 2654435761u + seed + i) & 0x3ffffffu;
    for (int c = 0; c < 4; c++)
        for (int i = 0; i < 5; i++) a[c][i] = (blockIdx.x + c * 7 + i) & 0x3ffffffu;
    for (int it = 0; it < 1024; it++) {
#pragma unroll
        for (int c = 0; c < 4; c++) unsat_mul_norm(a[c], b);
    }
    uint64_t s = 0;
    for (int c = 0; c < 4; c++)
        for (int i = 0; i < 5; i++) s ^= a[c][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add(uint64_t *out, uint32_t seed) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const uint32_t x = seed;
    for (int it = 0; it < 8192; it++) {
        asm volatile(
            "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
            "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8\n\t"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
static WSet *g_wtab;
typedef void (*kfn0)(uint64_t *, uint32_t);
typedef void (*kfn)(uint64_t *, uint32_t, const WSet *);
static float tk(kfn0 k, uint64_t *out, int blocks) {
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0u);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); if (r && ms < best) best = ms;
    }
    return best;
}
static float tk(kfn k, uint64_t *out, int blocks) {
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0u, (const WSet *)g_wtab);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); if (r && ms < best) best = ms;
    }
    return best;
}
template <int V>
static int run_variant(uint64_t *out, const fe *da, const fe *db, fe *dout, const std::vector<fe> &ha, const std::vector<fe> &hb, float tadd) {
    const size_t n = ha.size();
    static WSet *dw = nullptr;
    if (!dw) {
        std::vector<WSet> hw(n);
        for (size_t i = 0; i < n; i++) hw[i] = make_wset(hb[i]);
        (void)hipMalloc(&dw, n * sizeof(WSet));
        (void)hipMemcpy(dw, hw.data(), n * sizeof(WSet), hipMemcpyHostToDevice);
        g_wtab = dw;
    }
    hipLaunchKernelGGL(k_check<V>, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, (const WSet *)dw, dout, n);
    std::vector<fe> ho(n);
    (void)hipMemcpy(ho.data(), dout, n * sizeof(fe), hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) {
        const fe want = fe_mul(ha[i], hb[i]);
        if (!fe_eq(want, ho[i])) {
            if (bad < 3) printf("  v%d mismatch %zu: a=%016lx%016lx b=%016lx%016lx got %016lx%016lx want %016lx%016lx\n", V, i,
                                ha[i].hi, ha[i].lo, hb[i].hi, hb[i].lo, ho[i].hi, ho[i].lo, want.hi, want.lo);
            bad++;
        }
    }
    const float t = tk(k_tput<V>, out, 256 * 8);
    // k_add: 65536 adds per thread; k_tput: 4096 multiplies per thread
    printf("variant %d (%s): %s, %.1f add-equivalents per multiply\n", V, fmul_variant_name(V), bad ? "WRONG" : "bit-exact",
           t / tadd * 65536.0 / 4096.0);
    return bad != 0;
}
template <int V>
static int run_all(uint64_t *out, const fe *da, const fe *db, fe *dout, const std::vector<fe> &ha, const std::vector<fe> &hb, float tadd) {
    int r = run_variant<V>(out, da, db, dout, ha, hb, tadd);
    if constexpr (V + 1 < NV) r |= run_all<V + 1>(out, da, db, dout, ha, hb, tadd);
    return r;
}
int main() {
    const fe P = fe{ZK_P_LO, ZK_P_HI};
    std::vector<fe> edge = {fe_zero(), fe_one(), fe{ZK_P_LO - 1, ZK_P_HI}, fe{ZK_P_LO - 2, ZK_P_HI}, fe{0, 1}, fe{~0ull, 0},
                            fe{0xffffffffull, 0}, fe{0, 0xffffffff00000000ull}, fe{ZK_P_LO - 1 - ZK_C, ZK_P_HI},
                            fe{1ull << 63, 1ull << 63}, fe{0x2cffffffffffull, 0}, fe{0, 0x8000000000000000ull}};
    (void)P;
    std::vector<fe> ha, hb;
    for (auto x : edge)
        for (auto y : edge) { ha.push_back(x); hb.push_back(y); }
    uint64_t st = 0x9e3779b97f4a7c15ull;
    auto rnd = [&] { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
    for (int i = 0; i < (1 << 20); i++) {
        fe x{rnd(), rnd()}, y{rnd(), rnd()};
        // canonical operands; bias some toward p - small and small values
        if (x.hi == ~0ull && x.lo >= ZK_P_LO) x.lo -= ZK_C + 1;
        if (y.hi == ~0ull && y.lo >= ZK_P_LO) y.lo -= ZK_C + 1;
        if ((i & 7) == 1) x.hi = ~0ull, x.lo = ZK_P_LO - 1 - (rnd() & 0xffffff);
        if ((i & 7) == 2) y.hi = 0, y.lo &= 0xffffffff;
        if ((i & 15) == 3) x.hi = ~0ull, y.hi = ~0ull, x.lo = ZK_P_LO - 1 - (rnd() >> 20), y.lo = ZK_P_LO - 1 - (rnd() >> 20);
        ha.push_back(x);
        hb.push_back(y);
    }
    const size_t n = ha.size();
    fe *da, *db, *dout;
    uint64_t *out;
    (void)hipMalloc(&da, n * sizeof(fe));
    (void)hipMalloc(&db, n * sizeof(fe));
    (void)hipMalloc(&dout, n * sizeof(fe));
    (void)hipMalloc(&out, sizeof(uint64_t) * 256 * 8 * 256);
    (void)hipMemcpy(da, ha.data(), n * sizeof(fe), hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb.data(), n * sizeof(fe), hipMemcpyHostToDevice);
    const float tadd = tk(k_add, out, 256 * 8);
    const int rc = run_all<0>(out, da, db, dout, ha, hb, tadd);
    const float tu = tk(k_tput_unsat, out, 256 * 8);
    printf("unsaturated 5 x 26-bit limbs, product + normalisation only (no reduction, no conversion; a lower bound): "
           "%.1f add-equivalents per multiply\n", tu / tadd * (8192.0 * 8) / (1024.0 * 4));
    return rc;
}
