// air_shape.hpp -- ProcessorAir metadata shared by the prover and the verifier (host only).
#pragma once
#include <stddef.h>

#include <algorithm>

#include "../../include/zkvm_gpu.h"
#include "ext2.hpp"

namespace zk {
// num_constraint_composition_columns for the ProcessorAir transition degrees (air/src/lib.rs:69-90;
// winter-air TransitionConstraintDegree::get_evaluation_degree, cycle length 16) [DESIGN P6]:
// ceil((max evaluation degree - divisor degree) / n), divisor degree n - 2 (two exemptions)
inline int num_comp_cols(size_t n) {
    static const int base[20] = {1, 5, 2, 6, 6, 6, 7, 7, 6, 6, 6, 6, 4, 7, 4, 4, 2, 2, 2, 2};
    static const int cyc[20] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1};
    size_t hi = 0;
    for (int k = 0; k < 20; k++) hi = std::max(hi, (size_t)base[k] * (n - 1) + (cyc[k] ? (n / 16) * 15 : 0));
    size_t c = (hi - (n - 2) + n - 1) / n;
    return (int)std::max<size_t>(c, 1);
}
// verifier.cpp: the out-of-domain constraint identity at z (ood = [T(z)]_W ++ [T(zg)]_W ++ [H_j(z)]_C;
// ct: 20 transition, cb: 22 boundary composition coefficients), over E (base values lift with b = 0)
bool ood_identity(const fe2 *ood, int C, const fe2 *ct, const fe2 *cb, fe2 z, size_t n, const zk_pub_inputs *pub);
}  // namespace zk
