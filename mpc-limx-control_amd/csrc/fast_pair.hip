// fast_pair.hip -- the two-QPs-per-wavefront fused kernels (mpc_pair.hpp) for configurations
// with at most 30 free variables: SRBM 13/6/10 box (config B, explicit and generated inputs)
// and the reference-literal 13/3/10.
#include <hip/hip_runtime.h>

#include "../../include/mpcqp.h"
#include "fast_kernels.hpp"
#include "mpc_pair.hpp"

namespace mpcqp {
namespace {

// grid = ceil(B / 2): lanes 0-31 solve instance 2w, lanes 32-63 instance 2w + 1.  W: the
// register budget, waves per SIMD (the LDS layout, 9,984 B per wave at config B, fits 16 per
// CU either way): W = 4 hides more latency on a full chip, W = 3 runs a lone wave's chain
// faster (fewer code-motion fences, no spills) -- the library picks by batch size
template <int NU, int N, int MODEL, bool GEN, int W>
__global__ void __launch_bounds__(64, W) k_mpc_pair(MpcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_p[];
    pair_mpc<NU, N, MODEL, GEN, W>(a, smem_p);
}

template <int NU, int N, int MODEL>
void add_pair(FastKernels &k) {
    k.pair = (const void *)&k_mpc_pair<NU, N, MODEL, false, 3>;
    k.pair_w4 = (const void *)&k_mpc_pair<NU, N, MODEL, false, 4>;
    if constexpr (MODEL == 0) {
        k.pair_gen = (const void *)&k_mpc_pair<NU, N, MODEL, true, 3>;
        k.pair_gen_w4 = (const void *)&k_mpc_pair<NU, N, MODEL, true, 4>;
    }
    k.pair_lds = PairLayout<NU, N, MODEL>::lds_bytes;
    k.crash_k = MPCQP_PAIR_CRASH ? kPairCrashK : 0;
    k.crash_p = MPCQP_PAIR_CRASH ? kPairCrashP : 0;
}

}  // namespace

bool add_fast_pair(int model, int N, bool fric, int nfmax, FastKernels &k) {
    static_assert(kPairNF == kPairCap, "one capacity");
    // instances with more than kPairNF free forces go to the overflow list (or BAD_DIMS)
    (void)nfmax;
    if (fric || N != 10) return false;
    if (model == MPCQP_MODEL_SRBM && k.nu == 6) { add_pair<6, 10, 0>(k); return true; }
    if (model == MPCQP_MODEL_LITERAL && k.nu == 3) { add_pair<3, 10, 1>(k); return true; }
    return false;
}

}  // namespace mpcqp
