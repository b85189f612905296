// fast_srbm20.hip -- SRBM 13/6/20 instantiations (BASELINE config C: box + friction rows).
#define MPCQP_FAST_TU
#include "fast_kernels.hpp"

namespace mpcqp {

bool pick_fast_srbm20(bool fric, int nfmax, FastKernels &k) {
    if (nfmax > 64) return false;
    k = fric ? make_fast<13, 6, 20, 0, true, 64>() : make_fast<13, 6, 20, 0, false, 64>();
    return true;
}

}  // namespace mpcqp
