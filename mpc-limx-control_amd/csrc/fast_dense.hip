// fast_dense.hip -- the dense-model (whole-body, BASELINE config E) workgroup kernel,
// dense_wg.hpp: one 4-wave workgroup per QP, FP64 MFMA condensing.
#include <hip/hip_runtime.h>

#include "../../include/mpcqp.h"
#include "dense_wg.hpp"
#include "fast_kernels.hpp"

// waves per SIMD the register budget is sized for (2: what the 72.8 KB of LDS per workgroup
// allows, 256 registers; 1: 512 registers incl. AGPRs, one workgroup per CU)
#ifndef MPCQP_DENSE_W
#define MPCQP_DENSE_W 2
#endif

namespace mpcqp {
namespace {

template <int NX, int NU, int N, bool TOEP>
__global__ void __launch_bounds__(WgShape<NU * N>::THREADS, MPCQP_DENSE_W) k_dense_wg(MpcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_d[];
    // one workgroup per QP (grid = B): no grid-stride loop, so nothing is hoisted out of a loop
    // and kept live across the whole body
    const int b = xcd_order((int)blockIdx.x, (int)gridDim.x);
    if (b < a.B) dense_mpc_one<NX, NU, N, TOEP>(a, b, smem_d);
}

template <int NX, int NU, int N, bool TOEP>
void add_dense(FastKernels &k) {
    k.dense = (const void *)&k_dense_wg<NX, NU, N, TOEP>;
    k.dense_lds = DenseLayout<NX, NU, N, TOEP>::lds_bytes;
    k.dense_threads = WgShape<NU * N>::THREADS;
    k.nx = NX;
    k.nu = NU;
}

}  // namespace

// MPCQP_DENSE_TOEP=0: always the recursion (A/B builds)
#ifndef MPCQP_DENSE_TOEP
#define MPCQP_DENSE_TOEP 1
#endif

bool pick_fast_dense(int nx, int nu, int N, bool toep, FastKernels &k) {
    if (nx == 24 && nu == 6 && N == 16) {  // config E
        k.crash_k_wg = kWgCrashK;
        k.crash_p_wg = kWgCrashP;
        if (toep && MPCQP_DENSE_TOEP) add_dense<24, 6, 16, true>(k);
        else add_dense<24, 6, 16, false>(k);
        return true;
    }
    return false;
}

}  // namespace mpcqp
