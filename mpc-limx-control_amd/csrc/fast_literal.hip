// fast_literal.hip -- the reference-literal 13/3 model (include/mpcQP.h:154-181) at N = 20
// and N = 10 (fast_pair.hip adds the paired kernel for nf <= 30).
#define MPCQP_FAST_TU
// the dual loop's divisions by v_rcp_f64 + two Newton steps (wave_ops.hpp fdiv): L 2.36 -> 2.32
// ms, parity suite unchanged; within noise for C / E / B standing, which keep the IEEE division
#ifndef MPCQP_FAST_DIV
#define MPCQP_FAST_DIV 1
#endif
#include "fast_kernels.hpp"

namespace mpcqp {

bool pick_fast_literal(int N, int nfmax, FastKernels &k) {
    if (N == 20 && nfmax <= 64) { k = make_fast<13, 3, 20, 1, false, 60>(); return true; }
    if (N == 10 && nfmax <= 32) { k = make_fast<13, 3, 10, 1, false, 32>(); return true; }
    return false;
}

}  // namespace mpcqp
