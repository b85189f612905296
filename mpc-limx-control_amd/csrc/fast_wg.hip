// fast_wg.hip -- the workgroup-per-QP fused kernels (mpc_wg.hpp): every contact schedule of the
// SRBM 13/6/{10,20} configurations (double support, standing: up to 6N free forces), run on
// the instances the one-wave kernels append to the context's overflow list.
#include <hip/hip_runtime.h>

#include "../../include/mpcqp.h"
#include "fast_kernels.hpp"
#include "mpc_wg.hpp"

#ifndef MPCQP_OVF_ONEWAVE
#define MPCQP_OVF_ONEWAVE 1
#endif

namespace mpcqp {
namespace {

// one 4-wave workgroup per QP; list != nullptr: the overflow list, else the whole batch
template <int NU, int N, int MODEL, bool FRIC, bool GEN, int NF>
__global__ void __launch_bounds__(WgShape<NF>::THREADS, (NF <= 64 ? 2 : 1))
    k_mpc_wg(MpcArgs a, int *list, int *rearm) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_w[];
    wg_mpc_grid<NU, N, MODEL, FRIC, GEN, NF>(a, list, rearm, smem_w);
}

// explicit-input kernels only: calculateGait (the generated-input path) puts one foot down
// per step, so a generated schedule never exceeds the one-wave capacity
template <int N, bool FRIC, int NF>
void add_wg(FastKernels &k) {
    k.wg = (const void *)&k_mpc_wg<6, N, 0, FRIC, false, NF>;
    k.wg_lds = WgSrbmLayout<6, N, FRIC, NF>::lds_bytes;
    k.wg_threads = WgShape<NF>::THREADS;
}

}  // namespace

bool add_fast_wg(int model, int N, bool fric, FastKernels &k) {
    if (model != MPCQP_MODEL_SRBM || k.nu != 6) return false;
    // the crash start runs on box-only problems (no friction rows), and in these kernels only
    // when built with MPCQP_WG_SRBM_CRASH=1: at B standing its working sets average 21 bounds,
    // and their solves cost more than the dual passes they replace
    const bool crash = !fric && MPCQP_WG_SRBM_CRASH;
    k.crash_k_wg = crash ? kWgCrashK : 0;
    k.crash_p_wg = crash ? kWgCrashP : 0;
    // N = 10 behind the paired kernel: at most 6N = 60 free forces, which the one-QP-per-wave
    // k_mpc<.., 64> holds -- its list form takes the overflow (MPCQP_OVF_ONEWAVE);
    // 0: the workgroup kernel (A/B builds)
    if (N == 10 && MPCQP_OVF_ONEWAVE && k.pair && k.mpc_list && k.nf >= 6 * N) {
        k.wg = k.mpc_list;
        k.wg_lds = k.mpc_lds;
        k.wg_threads = 64;
        k.crash_k_wg = k.crash_p_wg = 0;
        return true;
    }
    if (N == 10) { fric ? add_wg<10, true, 64>(k) : add_wg<10, false, 64>(k); return true; }
    if (N == 20) { fric ? add_wg<20, true, 128>(k) : add_wg<20, false, 128>(k); return true; }
    return false;
}

}  // namespace mpcqp
