// fe_add variants: the library's (compiler carry chains through VCC) vs hand-interleaved asm chains
// with distinct SGPR carry pairs.  Bit-exact check + throughput in v_add_u32-equivalents per add.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include "../../encrypt-zkvm_amd/csrc/f128.hpp"

// Hazard rules used (gfx950, as hipcc's own code for these instructions respects them):
//   VALU writes an SGPR carry -> VALU reads it: >= 2 wait states;  VALU write -> SALU read: 0;
//   SALU write -> VALU read: >= 1.
__device__ __forceinline__ fe add_asm1(fe a, fe b) {
    uint32_t s0, s1, s2, s3, u0, u1, u2, u3;
    uint64_t cA, cB, m;
    const uint32_t C1 = 0x2cffu;
    asm("v_add_co_u32 %0, %8, %11, %15\n\t"
        "v_add_co_u32 %4, %9, %0, -1\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32 %1, %8, %12, %16, %8\n\t"
        "v_addc_co_u32 %5, %9, %1, %19, %9\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32 %2, %8, %13, %17, %8\n\t"
        "v_addc_co_u32 %6, %9, %2, 0, %9\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32 %3, %8, %14, %18, %8\n\t"
        "v_addc_co_u32 %7, %9, %3, 0, %9\n\t"
        "s_or_b64 %10, %8, %9\n\t"
        "s_nop 0\n\t"
        "v_cndmask_b32 %0, %0, %4, %10\n\t"
        "v_cndmask_b32 %1, %1, %5, %10\n\t"
        "v_cndmask_b32 %2, %2, %6, %10\n\t"
        "v_cndmask_b32 %3, %3, %7, %10"
        : "=&v"(s0), "=&v"(s1), "=&v"(s2), "=&v"(s3), "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3), "=&s"(cA), "=&s"(cB), "=&s"(m)
        : "v"(lo32(a.lo)), "v"(hi32(a.lo)), "v"(lo32(a.hi)), "v"(hi32(a.hi)), "v"(lo32(b.lo)), "v"(hi32(b.lo)), "v"(lo32(b.hi)),
          "v"(hi32(b.hi)), "v"(C1)
        : "scc");
    return fe{join32(s0, s1), join32(s2, s3)};
}

// two independent adds, four interleaved chains, no nops
__device__ __forceinline__ void add_asm2(fe a, fe b, fe c, fe d, fe &r1, fe &r2) {
    uint32_t s[4], u[4], t[4], v[4];
    uint64_t cA, cB, cC, cD, m1, m2;
    const uint32_t C1 = 0x2cffu;
    asm("v_add_co_u32 %0, %16, %22, %26\n\t"        // s0      (cA)
        "v_add_co_u32 %8, %18, %30, %34\n\t"        // t0      (cC)
        "v_add_co_u32 %4, %17, %0, -1\n\t"          // u0      (cB)
        "v_addc_co_u32 %1, %16, %23, %27, %16\n\t"  // s1
        "v_add_co_u32 %12, %19, %8, -1\n\t"         // v0      (cD)
        "v_addc_co_u32 %9, %18, %31, %35, %18\n\t"  // t1
        "v_addc_co_u32 %5, %17, %1, %38, %17\n\t"   // u1
        "v_addc_co_u32 %2, %16, %24, %28, %16\n\t"  // s2
        "v_addc_co_u32 %13, %19, %9, %38, %19\n\t"  // v1
        "v_addc_co_u32 %10, %18, %32, %36, %18\n\t" // t2
        "v_addc_co_u32 %6, %17, %2, 0, %17\n\t"     // u2
        "v_addc_co_u32 %3, %16, %25, %29, %16\n\t"  // s3
        "v_addc_co_u32 %14, %19, %10, 0, %19\n\t"   // v2
        "v_addc_co_u32 %11, %18, %33, %37, %18\n\t" // t3
        "v_addc_co_u32 %7, %17, %3, 0, %17\n\t"     // u3
        "s_nop 0\n\t"
        "v_addc_co_u32 %15, %19, %11, 0, %19\n\t"   // v3
        "s_or_b64 %20, %16, %17\n\t"
        "s_or_b64 %21, %18, %19\n\t"
        "v_cndmask_b32 %0, %0, %4, %20\n\t"
        "v_cndmask_b32 %1, %1, %5, %20\n\t"
        "v_cndmask_b32 %2, %2, %6, %20\n\t"
        "v_cndmask_b32 %3, %3, %7, %20\n\t"
        "v_cndmask_b32 %8, %8, %12, %21\n\t"
        "v_cndmask_b32 %9, %9, %13, %21\n\t"
        "v_cndmask_b32 %10, %10, %14, %21\n\t"
        "v_cndmask_b32 %11, %11, %15, %21"
        : "=&v"(s[0]), "=&v"(s[1]), "=&v"(s[2]), "=&v"(s[3]), "=&v"(u[0]), "=&v"(u[1]), "=&v"(u[2]), "=&v"(u[3]),
          "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]),
          "=&s"(cA), "=&s"(cB), "=&s"(cC), "=&s"(cD), "=&s"(m1), "=&s"(m2)
        : "v"(lo32(a.lo)), "v"(hi32(a.lo)), "v"(lo32(a.hi)), "v"(hi32(a.hi)), "v"(lo32(b.lo)), "v"(hi32(b.lo)), "v"(lo32(b.hi)),
          "v"(hi32(b.hi)), "v"(lo32(c.lo)), "v"(hi32(c.lo)), "v"(lo32(c.hi)), "v"(hi32(c.hi)), "v"(lo32(d.lo)), "v"(hi32(d.lo)),
          "v"(lo32(d.hi)), "v"(hi32(d.hi)), "v"(C1)
        : "scc");
    r1 = fe{join32(s[0], s[1]), join32(s[2], s[3])};
    r2 = fe{join32(t[0], t[1]), join32(t[2], t[3])};
}

template <int V>
__device__ __forceinline__ void op2(fe &x, fe &y, fe b) {
    if constexpr (V == 0) { x = fe_add(x, b); y = fe_add(y, b); }
    if constexpr (V == 1) { x = add_asm1(x, b); y = add_asm1(y, b); }
    if constexpr (V == 2) { fe r1, r2; add_asm2(x, b, y, b, r1, r2); x = r1; y = r2; }
}
template <int V>
__global__ void k_check(const fe *a, const fe *b, fe *o, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) { fe x = a[i], y = b[i]; op2<V>(x, y, b[i]); o[2 * i] = x; o[2 * i + 1] = y; }
}
template <int V>
__global__ void __launch_bounds__(256) k_tput(uint64_t *out, uint32_t seed) {
    fe a[4], b = fe_make(threadIdx.x + seed, 12345);
    for (int i = 0; i < 4; i++) a[i] = fe_make(i + 1, blockIdx.x);
    for (int it = 0; it < 1024; it++) {
        op2<V>(a[0], a[1], b);
        op2<V>(a[2], a[3], b);
    }
    uint64_t s = 0;
    for (int i = 0; i < 4; i++) s ^= a[i].lo ^ a[i].hi;
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
static const char *names[] = {"library fe_add", "asm, one add, 2 chains", "asm, two adds, 4 chains"};
template <int V>
static int run(uint64_t *out, const fe *da, const fe *db, fe *dout, const std::vector<fe> &ha, const std::vector<fe> &hb, float tadd) {
    const size_t n = ha.size();
    hipLaunchKernelGGL(k_check<V>, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, dout, n);
    std::vector<fe> ho(2 * n);
    (void)hipMemcpy(ho.data(), dout, 2 * n * sizeof(fe), hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) {
        const fe w1 = fe_add(ha[i], hb[i]), w2 = fe_add(hb[i], hb[i]);
        bad += !fe_eq(w1, ho[2 * i]) || !fe_eq(w2, ho[2 * i + 1]);
    }
    const float t = tk(k_tput<V>, out, 256 * 8);
    printf("%-28s %s, %.1f add-equivalents per fe_add\n", names[V], bad ? "WRONG" : "bit-exact", t / tadd * 65536.0 / 4096.0);
    return bad != 0;
}
int main() {
    std::vector<fe> ha, hb;
    uint64_t st = 0x9e3779b97f4a7c15ull;
    auto rnd = [&] { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
    const fe edge[] = {fe_zero(), fe_one(), fe{ZK_P_LO - 1, ZK_P_HI}, fe{ZK_P_LO - 2, ZK_P_HI}, fe{0, 1}, fe{~0ull, 0},
                       fe{0xffffffffull, 0}, fe{ZK_P_LO - 1 - ZK_C, ZK_P_HI}, fe{1ull << 63, 1ull << 63}, fe{ZK_C, 0}, fe{ZK_C + 1, 0}};
    for (auto x : edge) for (auto y : edge) { ha.push_back(x); hb.push_back(y); }
    for (int i = 0; i < (1 << 20); i++) {
        fe x{rnd(), rnd()}, y{rnd(), rnd()};
        if (x.hi == ~0ull && x.lo >= ZK_P_LO) x.lo -= ZK_C + 1;
        if (y.hi == ~0ull && y.lo >= ZK_P_LO) y.lo -= ZK_C + 1;
        if ((i & 3) == 1) x.hi = ~0ull, x.lo = ZK_P_LO - 1 - (rnd() >> 16);
        if ((i & 3) == 2) y.hi = ~0ull, y.lo = ZK_P_LO - 1 - (rnd() >> 16);
        ha.push_back(x); hb.push_back(y);
    }
    const size_t n = ha.size();
    fe *da, *db, *dout; uint64_t *out;
    (void)hipMalloc(&da, n * sizeof(fe)); (void)hipMalloc(&db, n * sizeof(fe)); (void)hipMalloc(&dout, 2 * n * sizeof(fe));
    (void)hipMalloc(&out, sizeof(uint64_t) * 256 * 8 * 256);
    (void)hipMemcpy(da, ha.data(), n * sizeof(fe), hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb.data(), n * sizeof(fe), hipMemcpyHostToDevice);
    const float tadd = tk(k_add, out, 256 * 8);
    int r = run<0>(out, da, db, dout, ha, hb, tadd);
    r |= run<1>(out, da, db, dout, ha, hb, tadd);
    r |= run<2>(out, da, db, dout, ha, hb, tadd);
    return r;
}
