// fast_kernels.hpp -- the compile-time-dimension kernels of the fused hot path and their
// per-configuration instantiation.  Each configuration family is instantiated in its own
// translation unit (fast_srbm10.hip, fast_srbm20.hip, fast_literal.hip, fast_pair.hip) so the
// library builds in parallel; mpcqp_kernels.hip picks one through pick_fast().
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mpcqp.h"

#ifdef MPCQP_VARIANT_TAG  // set only on a variant build's translation unit (build_variants.sh)
extern "C" const char *mpcqp_variant_tag_fn(void) { return MPCQP_VARIANT_TAG; }
#endif

#ifndef MPCQP_W32
#define MPCQP_W32 3  // waves per SIMD the NF <= 32 fused kernel is register-budgeted for
#endif
#ifndef MPCQP_W64
#define MPCQP_W64 2  // the same for NF = 64
#endif
#include "condense.hpp"
#include "fused.hpp"
#include "mpc_fused.hpp"

namespace mpcqp {

struct FastKernels {
    const void *mpc_gen = nullptr;
    const void *pair = nullptr, *pair_gen = nullptr;  // two QPs per wave (nf <= 30)
    // the same at a 4-wave register budget, used from pair_w4_min instances per launch
    const void *pair_w4 = nullptr, *pair_gen_w4 = nullptr;
    int pair_w4_min = 0;
    size_t pair_lds = 0;
    const void *wg = nullptr;  // workgroup per QP for the overflow list (nf <= 6N)
    size_t wg_lds = 0;
    int wg_threads = 0;
    const void *dense = nullptr;  // dense model (whole body): workgroup per QP, MFMA condensing
    size_t dense_lds = 0;
    int dense_threads = 0;
    const void *disc = nullptr, *cs = nullptr, *mpc = nullptr;
    const void *mpc_list = nullptr;  // k_mpc on the overflow list (SRBM): the paired kernel's overflow
    size_t disc_lds = 0, cs_lds = 0, mpc_lds = 0;
    int nx = 0, nu = 0;
    int prim_nf = 0;  // free variables the one-wave kernel holds (kPairCap or its NF)
    int nf = 0;       // NF the one-wave kernel is instantiated for
    int crash_k = 0, crash_p = 0;  // the one-wave kernel's crash start (0: none)
    int crash_k_wg = 0, crash_p_wg = 0;  // the workgroup solver's (overflow / dense kernels)
};

constexpr int kPairCap = 30;  // free variables of one half of the paired kernel (mpc_pair.hpp)
// batches from which the paired kernel runs at its 4-wave register budget (fast_pair.hip): below,
// fewer than ~3 waves per SIMD are resident and the 3-wave build's shorter chain wins
#ifndef MPCQP_PAIR_W4_MIN
#define MPCQP_PAIR_W4_MIN 16384
#endif
constexpr int kPairW4Min = MPCQP_PAIR_W4_MIN;

// per-family pickers (one translation unit each); false = not instantiated
bool pick_fast_srbm10(bool fric, int nfmax, FastKernels &k);
bool pick_fast_srbm20(bool fric, int nfmax, FastKernels &k);
bool pick_fast_literal(int N, int nfmax, FastKernels &k);
// two-QPs-per-wave kernels (fast_pair.hip), added to k for nf <= 30 configurations
bool add_fast_pair(int model, int N, bool fric, int nfmax, FastKernels &k);
// workgroup-per-QP kernels (fast_wg.hip) for the instances beyond the one-wave capacity
bool add_fast_wg(int model, int N, bool fric, FastKernels &k);
// dense-model kernels (fast_dense.hip): config E, 24/6/16
// toep: Q and P have symmetric factors (the Toeplitz condensing, dense_wg.hpp); otherwise the
// Riccati-style recursion
bool pick_fast_dense(int nx, int nu, int N, bool toep, FastKernels &k);

#ifdef MPCQP_FAST_TU
namespace {

template <int NX, int NU, int MODEL>
__global__ void __launch_bounds__(64) k_discretize(FastArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem_f[];
    if ((int)blockIdx.x >= a.B) return;
    fast_discretize<NX, NU, MODEL>(a, smem_f);
}

template <int NX, int NU, int N, int MODEL, bool FRIC, int NFMAX>
__global__ void __launch_bounds__(64) k_condense_solve(FastArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_c[];
    if ((int)blockIdx.x >= a.B) return;
    fast_condense_solve<NX, NU, N, MODEL, FRIC, NFMAX>(a, smem_c);
}

template <int NU, int N, int MODEL, bool FRIC, int NF>
__global__ void __launch_bounds__(64, (NF <= 32 ? MPCQP_W32 : MPCQP_W64)) k_mpc(MpcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_m[];
    if ((int)blockIdx.x >= a.B) return;
    fast_mpc<NU, N, MODEL, FRIC, NF>(a, smem_m);
}

// the overflow list's one-QP-per-wave kernel (instances the paired kernel defers: more than its
// 30 free forces per half, at most NF): the same fused step as k_mpc on the listed instances,
// a resident grid striding over the list; re-arms the other list and, in the fused selection,
// commits each workgroup's minimum key and finalizes the record (as wg_mpc_grid, mpc_wg.hpp)
template <int NU, int N, int MODEL, bool FRIC, int NF>
__global__ void __launch_bounds__(64, (NF <= 32 ? MPCQP_W32 : MPCQP_W64))
    k_mpc_list(MpcArgs a, int *list, int *rearm) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_l[];
    if (blockIdx.x == 0 && threadIdx.x < kListSubs)
        __hip_atomic_store(&rearm[threadIdx.x * kListStride], 0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const OvfView ov = ovf_view(list, a.ovf_cap);
    const int count = ov.total;
    unsigned long long kmin = kSelNone;
    for (int i = blockIdx.x; i < count; i += gridDim.x) {
        unsigned long long k = kSelNone;
        fast_mpc<NU, N, MODEL, FRIC, NF>(a, smem_l, ov.id(i), &k);
        kmin = k < kmin ? k : kmin;
        wave_sync();
    }
    if (a.sel) {
        const int groups = count <= 0 ? 1 : (count < (int)gridDim.x ? count : (int)gridDim.x);
        if ((int)blockIdx.x >= groups) return;
        sel_commit(a, kmin, NU * N, (int)blockIdx.x < count,
                   reinterpret_cast<unsigned long long *>(smem_l), groups, count <= 0);
    }
}

// device-generated inputs: the same fused step, x0/xref/lin/contact
// built on chip from per-state data, gait candidates and commands
template <int NU, int N, int MODEL, bool FRIC, int NF>
__global__ void __launch_bounds__(64, (NF <= 32 ? 3 : MPCQP_W64)) k_mpc_gen(MpcArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_g[];
    if ((int)blockIdx.x >= a.B) return;
    fast_mpc<NU, N, MODEL, FRIC, NF, true>(a, smem_g);
}

}  // namespace

template <int NX, int NU, int N, int MODEL, bool FRIC, int NFMAX>
FastKernels make_fast() {
    FastKernels k;
    k.disc = (const void *)&k_discretize<NX, NU, MODEL>;
    k.cs = (const void *)&k_condense_solve<NX, NU, N, MODEL, FRIC, NFMAX>;
    k.disc_lds = sizeof(double) * disc_lds_doubles<NX, NU>();
    k.cs_lds = CSLayout<NX, NU, N, FRIC, NFMAX>::lds_bytes;
    k.mpc = (const void *)&k_mpc<NU, N, MODEL, FRIC, NFMAX>;
    if constexpr (MODEL == 0) {
        k.mpc_gen = (const void *)&k_mpc_gen<NU, N, MODEL, FRIC, NFMAX>;
        k.mpc_list = (const void *)&k_mpc_list<NU, N, MODEL, FRIC, NFMAX>;
    }
    k.mpc_lds = MpcLayout<NU, N, FRIC, NFMAX>::lds_bytes;
    k.nx = NX;
    k.nu = NU;
    k.nf = NFMAX;
    return k;
}
#endif  // MPCQP_FAST_TU

}  // namespace mpcqp
