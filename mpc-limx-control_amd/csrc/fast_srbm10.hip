// fast_srbm10.hip -- SRBM 13/6/10 instantiations (BASELINE config B, the metric; box or
// friction rows): one-QP-per-wave kernels for NF <= 32 / 64 (fast_pair.hip adds the paired
// kernel for nf <= 30).
#define MPCQP_FAST_TU
#include "fast_kernels.hpp"

namespace mpcqp {

bool pick_fast_srbm10(bool fric, int nfmax, FastKernels &k) {
    if (nfmax <= 32) {
        k = fric ? make_fast<13, 6, 10, 0, true, 32>() : make_fast<13, 6, 10, 0, false, 32>();
        return true;
    }
    if (nfmax <= 64) {
        k = fric ? make_fast<13, 6, 10, 0, true, 64>() : make_fast<13, 6, 10, 0, false, 64>();
        return true;
    }
    return false;
}

}  // namespace mpcqp
