// ext2.hpp -- the quadratic extension E = F[X]/(X^2 - X - 1) of the f128 field, for gfx950 and
// host: winter-math `ExtensibleField<2> for f128::BaseElement` (FieldExtension::Quadratic in
// ProofOptions; vm/src/lib.rs:20 uses None, SURVEY.md config 5 needs Quadratic for 128 bits).
//
// An fe2 is a + b*X, serialized as the two base elements a, b (32 bytes).  Base-field values lift
// with b = 0.  Multiplication is Karatsuba with X^2 = X + 1 (3 base multiplications):
//   (a0 + a1 X)(b0 + b1 X) = (a0 b0 + a1 b1) + ((a0 + a1)(b0 + b1) - a0 b0) X
#pragma once
#include "f128.hpp"

struct fe2 {
    fe a, b;
};

ZK_HD fe2 fe2_make(fe a, fe b) { return fe2{a, b}; }
ZK_HD fe2 fe2_lift(fe a) { return fe2{a, fe_zero()}; }
ZK_HD fe2 fe2_zero() { return fe2{fe_zero(), fe_zero()}; }
ZK_HD fe2 fe2_one() { return fe2{fe_one(), fe_zero()}; }
ZK_HD bool fe2_eq(fe2 x, fe2 y) { return fe_eq(x.a, y.a) && fe_eq(x.b, y.b); }
ZK_HD fe2 fe2_add(fe2 x, fe2 y) { return fe2{fe_add(x.a, y.a), fe_add(x.b, y.b)}; }
ZK_HD fe2 fe2_sub(fe2 x, fe2 y) { return fe2{fe_sub(x.a, y.a), fe_sub(x.b, y.b)}; }
ZK_HD fe2 fe2_mul(fe2 x, fe2 y) {
    const fe z = fe_mul(x.a, y.a);
    return fe2{fe_add(z, fe_mul(x.b, y.b)), fe_sub(fe_mul(fe_add(x.a, x.b), fe_add(y.a, y.b)), z)};
}
ZK_HD fe2 fe2_mulb(fe2 x, fe s) { return fe2{fe_mul(x.a, s), fe_mul(x.b, s)}; }
// X * (a + bX) = b + (a + b) X
ZK_HD fe2 fe2_mulX(fe2 v) { return fe2{v.b, fe_add(v.a, v.b)}; }
// (a + bX)^-1 = ((a + b) - bX) / (a^2 + ab - b^2)
ZK_HD fe2 fe2_inv(fe2 x) {
    const fe d = fe_sub(fe_add(fe_mul(x.a, x.a), fe_mul(x.a, x.b)), fe_mul(x.b, x.b));
    const fe di = fe_inv(d);
    return fe2{fe_mul(fe_add(x.a, x.b), di), fe_neg(fe_mul(x.b, di))};
}
ZK_HD fe2 fe2_exp(fe2 x, uint64_t e) {
    fe2 r = fe2_one();
    while (e) {
        if (e & 1) r = fe2_mul(r, x);
        x = fe2_mul(x, x);
        e >>= 1;
    }
    return r;
}
