// fast_srbm20.hip -- SRBM 13/6/20 instantiations (BASELINE config C: box + friction rows).
#define MPCQP_FAST_TU
#include "fast_kernels.hpp"

namespace mpcqp {

// NF = 60 = 3N: one foot in contact per step (calculateGait's alternating schedule) -- the
// register arrays hold exactly those, lane 63 is free to carry g through the inverse sweep;
// double support / standing instances (up to 6N) overflow to the workgroup kernel
bool pick_fast_srbm20(bool fric, int nfmax, FastKernels &k) {
    if (nfmax > 64) return false;
    k = fric ? make_fast<13, 6, 20, 0, true, 60>() : make_fast<13, 6, 20, 0, false, 60>();
    return true;
}

}  // namespace mpcqp
