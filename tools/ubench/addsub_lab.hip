// addsub2 variants: the compiler's four chains through VCC (ZK_ADDSUB_ASM=0's form) against the generated
// interleaved asm blocks (csrc/addsub_asm.hpp): bit-exact check against the host field ops on random, edge and
// lazy (non-canonical first operand) inputs, then throughput in v_add_u32-equivalent issue slots per addsub2 (two
// adds + two subs), 8 waves per SIMD, 4 independent chains per thread.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o addsub_lab addsub_lab.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <vector>

#include "../../encrypt-zkvm_amd/csrc/f128.hpp"

// the compiler's form (what ZK_ADDSUB_ASM=0 builds)
template <int V>
__device__ __forceinline__ void ref_addsub2(fe a, fe b, fe c, fe d, fe &apb, fe &amb, fe &cpd, fe &cmd) {
    apb = V != 0 ? fe_add_lazy(a, b) : fe_add(a, b);
    amb = fe_sub(a, b);
    cpd = V == 1 ? fe_add_lazy(c, d) : fe_add(c, d);
    cmd = fe_sub(c, d);
}

template <int V, bool ASM>
__global__ void k_check(const fe *in, fe *out, size_t n) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe r[4];
    if (ASM) addsub2_v<V>(in[4 * i], in[4 * i + 1], in[4 * i + 2], in[4 * i + 3], r[0], r[1], r[2], r[3]);
    else ref_addsub2<V>(in[4 * i], in[4 * i + 1], in[4 * i + 2], in[4 * i + 3], r[0], r[1], r[2], r[3]);
    for (int k = 0; k < 4; k++) out[4 * i + k] = r[k];
}

template <bool ASM>
__global__ void __launch_bounds__(256) k_tput(uint64_t *out, uint32_t seed) {
    fe x[8];
    for (int i = 0; i < 8; i++) x[i] = fe_make(threadIdx.x + seed + i, blockIdx.x + i);
    for (int it = 0; it < 512; it++) {
        fe y[8];
        if (ASM) {
            addsub2_v<0>(x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]);
            addsub2_v<0>(x[4], x[5], x[6], x[7], y[4], y[5], y[6], y[7]);
        } else {
            ref_addsub2<0>(x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]);
            ref_addsub2<0>(x[4], x[5], x[6], x[7], y[4], y[5], y[6], y[7]);
        }
        for (int i = 0; i < 8; i++) x[i] = y[i];
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; i++) s ^= x[i].lo ^ x[i].hi;
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
typedef void (*kfn)(uint64_t *, uint32_t);
static float tk(kfn k, uint64_t *out, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e9;
    for (int r = 0; r < 6; r++) {
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

static fe h_add_lazy(fe a, fe b) {
    unsigned __int128 x = fe_to_u128(a), y = fe_to_u128(b), s = x + y;
    if (s < x) s += (unsigned __int128)ZK_C;  // s - 2^128 + C
    return fe_from_u128(s);
}

int main() {
    uint64_t st = 0x9e3779b97f4a7c15ull;
    auto rnd = [&] { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
    const fe p1{ZK_P_LO - 1, ZK_P_HI};
    const fe edge[] = {fe_zero(), fe_one(), p1, fe{ZK_P_LO - 2, ZK_P_HI}, fe{0, 1}, fe{~0ull, 0}, fe{0xffffffffull, 0},
                       fe{ZK_P_LO - 1 - ZK_C, ZK_P_HI}, fe{1ull << 63, 1ull << 63}, fe{ZK_C, 0}, fe{ZK_C + 1, 0},
                       fe{0, ~0ull}, fe{ZK_P_LO, ZK_P_HI - 1}};
    auto canon = [&] {
        fe x{rnd(), rnd()};
        const int sel = (int)(rnd() & 7);
        if (sel == 1) x.hi = ~0ull, x.lo = ZK_P_LO - 1 - (rnd() >> (rnd() & 63));
        if (sel == 2) x = edge[rnd() % 13];
        if (x.hi == ~0ull && x.lo >= ZK_P_LO) x.lo -= ZK_C + 1;
        return x;
    };
    auto any128 = [&] {  // lazy first operands: any value < 2^128, biased to >= p
        fe x{rnd(), rnd()};
        const int sel = (int)(rnd() & 3);
        if (sel == 1) x.hi = ~0ull, x.lo = ZK_P_LO + (rnd() >> (rnd() & 63));
        if (sel == 2) x = fe{~0ull, ~0ull};
        return x;
    };
    const size_t n = 1 << 21;
    int bad_total = 0;
    fe *din, *dout;
    (void)hipMalloc(&din, 4 * n * sizeof(fe));
    (void)hipMalloc(&dout, 4 * n * sizeof(fe));
    for (int V = 0; V < 3; V++) {
        std::vector<fe> in(4 * n), got(4 * n), ref(4 * n);
        for (size_t i = 0; i < n; i++) {
            const bool la = V != 0, lc = V == 1;
            in[4 * i] = la ? any128() : canon();
            in[4 * i + 1] = canon();
            in[4 * i + 2] = lc ? any128() : canon();
            in[4 * i + 3] = canon();
            if (i < 169) {  // every pair of edge values
                in[4 * i] = edge[i % 13], in[4 * i + 1] = edge[i / 13];
                in[4 * i + 2] = edge[i / 13], in[4 * i + 3] = edge[i % 13];
            }
        }
        (void)hipMemcpy(din, in.data(), 4 * n * sizeof(fe), hipMemcpyHostToDevice);
        for (int asmv = 0; asmv < 2; asmv++) {
            if (V == 0) hipLaunchKernelGGL((asmv ? k_check<0, true> : k_check<0, false>), dim3(n / 256), dim3(256), 0, 0, din, dout, n);
            if (V == 1) hipLaunchKernelGGL((asmv ? k_check<1, true> : k_check<1, false>), dim3(n / 256), dim3(256), 0, 0, din, dout, n);
            if (V == 2) hipLaunchKernelGGL((asmv ? k_check<2, true> : k_check<2, false>), dim3(n / 256), dim3(256), 0, 0, din, dout, n);
            (void)hipMemcpy(got.data(), dout, 4 * n * sizeof(fe), hipMemcpyDeviceToHost);
            size_t bad = 0;
            for (size_t i = 0; i < n; i++) {
                const fe a = in[4 * i], b = in[4 * i + 1], c = in[4 * i + 2], d = in[4 * i + 3];
                const fe e0 = V != 0 ? h_add_lazy(a, b) : fe_add(a, b);
                const fe e2 = V == 1 ? h_add_lazy(c, d) : fe_add(c, d);
                const fe e1 = fe_sub(a, b), e3 = fe_sub(c, d);
                bad += !fe_eq(e0, got[4 * i]) || !fe_eq(e1, got[4 * i + 1]) || !fe_eq(e2, got[4 * i + 2]) ||
                       !fe_eq(e3, got[4 * i + 3]);
            }
            printf("variant %d (%s): %s (%zu of %zu wrong)\n", V, asmv ? "asm" : "compiler", bad ? "WRONG" : "bit-exact",
                   bad, n);
            bad_total += bad != 0;
        }
    }
    uint64_t *out;
    (void)hipMalloc(&out, sizeof(uint64_t) * 256 * 8 * 256);
    const float tadd = tk(k_add, out, 256 * 8);
    const float tc = tk(k_tput<false>, out, 256 * 8), ta = tk(k_tput<true>, out, 256 * 8);
    // k_add: 8192 x 8 adds per thread; k_tput: 512 x 2 addsub2 per thread
    const double per = 8192.0 * 8.0 / (512.0 * 2.0);
    printf("addsub2 issue slots: compiler %.1f, asm %.1f (v_add_u32 = 1)\n", tc / tadd * per, ta / tadd * per);
    return bad_total;
}
