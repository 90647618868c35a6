// fri_small.hpp -- the FRI fold's small inverse DFT, shared by the single-GPU fold (kernels.hip) and the sharded
// prover's layer-0 fold over its own cosets (shard.hip).
#pragma once
#include "f128.hpp"

namespace zk {
// V_m = sum_k v_k * zeta^(-k m), m < F: in-register radix-2 DIT on bit-reversed input (zinv[t] = zeta^-t);
// the j = 0 twiddles are compile-time 1, so F = 8 costs 5 multiplies instead of 64.
template <int F>
__device__ __forceinline__ void idft_small(fe v[F], const fe *zinv) {
    constexpr int LOGF = F == 2 ? 1 : F == 4 ? 2 : F == 8 ? 3 : 4;
    fe w[F];
#pragma unroll
    for (int k = 0; k < F; k++) {
        int r = 0;
#pragma unroll
        for (int b = 0; b < LOGF; b++) r |= ((k >> b) & 1) << (LOGF - 1 - b);
        w[r] = v[k];
    }
#pragma unroll
    for (int len = 2; len <= F; len <<= 1) {
#pragma unroll
        for (int start = 0; start < F; start += len) {
#pragma unroll
            for (int j = 0; j < len / 2; j++) {
                const fe u = w[start + j];
                const fe t = j == 0 ? w[start + j + len / 2] : fe_mul(w[start + j + len / 2], zinv[j * (F / len)]);
                w[start + j] = fe_add(u, t);
                w[start + j + len / 2] = fe_sub(u, t);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < F; k++) v[k] = w[k];
}

}  // namespace zk
