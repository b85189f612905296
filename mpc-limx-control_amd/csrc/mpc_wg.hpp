// mpc_wg.hpp -- the fused per-tick step (mpc_fused.hpp) for instances with more free forces
// than the one-wave kernels hold: up to NF = 64 at N = 10 and NF = 128 at N = 20, i.e. every
// contact schedule including double support and standing (nf = 6 N).  One workgroup (2 waves for
// NF <= 64, 4 above) per QP: wave 0 runs the same input / model / condensed-term phases as fast_mpc, every thread
// then builds its half-row of H_FF from the closed form and gi_run_wg (gi_wg.hpp) solves.
//
// Reference: mpcQP::mpcQP + buildSystemModel (include/mpcQP.h:35-119, 121-182),
// QPSolver::discretizeSystem / buildQPParams / solveQP (src/QPSolver.cpp:21-106); qpOASES
// takes the dense nV = NU*N problem whatever the bound pattern (src/QPSolver.cpp:87-96).
//
// Routing: the one-wave kernels (k_mpc_pair, k_mpc) append an instance whose free-variable
// count exceeds their register capacity to the context's overflow list (64 sub-lists, one
// atomic per deferring wavefront, mpc_fused.hpp) and
// leave its outputs alone; k_mpc_wg, launched right after on the same stream with a resident
// grid, solves the listed instances and writes their outputs; the last workgroup to finish
// re-arms the list.  An empty list costs one short launch.
#pragma once
#include "gi_wg.hpp"
#include "mpc_fused.hpp"

namespace mpcqp {

template <int NU, int N, bool FRIC, int NF>
struct WgSrbmLayout {
    static constexpr int NX = 13, NV = NU * N;
    static constexpr int NFRIC = FRIC ? 4 * N * 2 : 0;
    static constexpr int MT = 2 * NF + NFRIC;
    // live for the whole solve: x mirror (one per row), fixed values, the bounds' b
    static constexpr int oXS = 0;
    static constexpr int oXF = oXS + WgShape<NF>::RW;
    static constexpr int oMisc = oXF + NV;                 // nf and status for waves 1-3
    static constexpr int oCB = oMisc + 2;
    static constexpr int oU = (oCB + 2 * NF + 1) & ~1;     // shared region (16-B aligned)
    // front view (wave 0), as MpcLayout's early + condensed views
    static constexpr int oT = oU;
    static constexpr int oX0 = oT + NX * (NX + NU);
    static constexpr int oX1 = oX0 + NX * NU;
    static constexpr int oAx = oX1 + NX * NU;
    static constexpr int oXr = oAx + 2 * NX;
    static constexpr int oX0v = oXr + NX * (N + 1);
    static constexpr int oS = (oX0v + NX + 1) & ~1;
    static constexpr int oUV = oS + 4 * NU * NU;
    static constexpr int oRm = oUV + (N + 1) * 2 * NU;
    static constexpr int nFront = oRm + NU * NU - oU;
    // solver view (after every thread holds its H_FF half-row)
    static constexpr int oW = oU;
    static constexpr int nSolver = WgLayout<NF>::work;
    static constexpr int nDoubles = oU + (nFront > nSolver ? nFront : nSolver);
    static constexpr size_t bytes =
        sizeof(double) * nDoubles + sizeof(int) * (NF + NV) + ((MT + 15) & ~15);
    static constexpr size_t lds_bytes = (bytes + 15) & ~(size_t)15;
};

template <int NU, int N, int MODEL, bool FRIC, bool GEN, int NF>
__device__ __forceinline__ void wg_mpc_one(const MpcArgs &a, int b, unsigned char *smem) {
    using Lay = WgSrbmLayout<NU, N, FRIC, NF>;
    constexpr int NV = Lay::NV, NH = NF / 2;
    const WgIds T = wg_ids<WgShape<NF>::RW>();
    double *D = reinterpret_cast<double *>(smem);

    SolveProblem P;
    P.nV = NV;
    P.H = nullptr; P.f = nullptr; P.lb = nullptr; P.ub = nullptr;
    P.gen_bounds = 1;
    P.model = MODEL; P.nu = NU; P.N = N; P.nfeet = 2;
    P.fz_min = a.fz_min; P.fz_max = a.fz_max; P.fxy_max = a.fxy_max;
    P.u_min = a.u_min; P.u_max = a.u_max;
    P.contact = (MODEL != 0) ? 0ull
              : GEN ? gait_mask_wave(N, a.Ts, a.phase[b], a.swing, a.stance) : a.contact[b];
    P.friction = FRIC ? 1 : 0;
    P.mu = a.mu;
    P.mA = 0; P.A = nullptr; P.a_colmajor = 0; P.lbA = nullptr; P.ubA = nullptr;
    P.max_iter = a.max_iter;
    GiCtx C;
    C.wide = 1;
    C.crash_p = (FRIC || !MPCQP_WG_SRBM_CRASH) ? 0 : a.crash_p_wg;
    C.stamps = a.stamps;
    C.cut = a.cut >= 100 ? a.cut - 100 : 0;  // (cuts build) MPCQP_CUT=100+k: the workgroup solver's cut k
    MPCQP_STAMP_INIT(tst);
    C.P = &P;
    C.nfmax = NF;
    C.L.ld = NF | 1;
    C.L.R = nullptr;
    C.L.J = nullptr;
    C.L.g = nullptr;
    C.L.xs = D + Lay::oXS;
    C.L.xfull = D + Lay::oXF;
    C.L.rowfix = D + Lay::oMisc;
    C.L.ys = D + Lay::oMisc;
    int *ip = reinterpret_cast<int *>(D + Lay::nDoubles);
    C.L.fid = ip;
    C.L.pos = ip + NF;
    C.L.st = reinterpret_cast<unsigned char *>(ip + NF + NV);
    C.L.cb = D + Lay::oCB;

    if (T.wv == 0) {
        double lin[8];
        mpc_load_inputs<Lay, NU, N, GEN>(a, b, D, lin);
        mpc_model_terms<Lay, NU, MODEL>(a, D, lin);
        gi_setup(C);  // free map + constraint states (up to NF free)
        if (C.nf > a.max_free) C.status = ST_BAD_DIMS;
        mpc_condensed_terms<Lay, NU, N, MODEL>(a, D);
        if (T.ln == 0) {
            D[Lay::oMisc] = (double)C.nf;
            D[Lay::oMisc + 1] = (double)C.status;
        }
    }
    __syncthreads();
    C.nf = (int)D[Lay::oMisc];
    C.status = (int)D[Lay::oMisc + 1];
    C.nfric = FRIC ? 4 * N * 2 : 0;
    C.mt = 2 * C.nf + C.nfric;
    C.c0 = 0.0;
    MPCQP_STAMP(a.stamps, 0, tst);

    // ---- H_FF half-rows (lower triangle; identity padding beyond nf) and g
    const int nf = C.nf, r = T.r, h = T.h;
    const bool ok = C.status == ST_OK && nf > 0;
    double hr[NH];
    double g = 0.0;
    if (ok && r < nf) {
        const int vi = C.L.fid[r];
#pragma unroll
        for (int j = 0; j < NH; ++j) {
            const int c = 2 * j + h;  // interleaved columns (gi_run_wg's factorisation layout)
            hr[j] = (c < nf && c <= r) ? mpc_h_entry<Lay, NU, N>(D, vi, C.L.fid[c]) : 0.0;
            step_fence();  // one entry at a time (the entries share no work)
        }
        g = mpc_g_entry<Lay, NU, N>(D, vi);
    } else {
#pragma unroll
        for (int j = 0; j < NH; ++j) hr[j] = (r == 2 * j + h) ? 1.0 : 0.0;
    }
    __syncthreads();  // the solver's workspace overlays the condensed terms
    MPCQP_STAMP(a.stamps, 3, tst);
    gi_run_wg<NF, !FRIC && MPCQP_WG_SRBM_CRASH>(C, hr, g, D + Lay::oW);
    MPCQP_STAMP_INIT(tw);
    SolveOut O;
    O.x = a.U + (size_t)b * NV;
    O.cost = a.cost + b;
    O.status = a.status + b;
    O.iters = a.iters + b;
    O.y = nullptr;
    gi_write_wg<NF>(C, O);
    MPCQP_STAMP(a.stamps, 9, tw);
}

// list == nullptr: instance b = blockIdx.x (+ grid stride) of the whole batch.  Otherwise the
// instances of the overflow list the one-wave kernel just filled; the context alternates two
// lists, and this launch re-arms the other one (its last reader was the previous launch, its
// next writer the next one-wave launch), so no exit ticket is needed.
template <int NU, int N, int MODEL, bool FRIC, bool GEN, int NF>
__device__ __forceinline__ void wg_mpc_grid(const MpcArgs &a, int *list, int *rearm,
                                            unsigned char *smem) {
    if (!list) {
        for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
            wg_mpc_one<NU, N, MODEL, FRIC, GEN, NF>(a, b, smem);
            __syncthreads();
        }
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x < kListSubs)
        __hip_atomic_store(&rearm[threadIdx.x * kListStride], 0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const OvfView ov = ovf_view(list, a.ovf_cap);
    const int count = ov.total;
    for (int i = blockIdx.x; i < count; i += gridDim.x) {
        wg_mpc_one<NU, N, MODEL, FRIC, GEN, NF>(a, ov.id(i), smem);
        __syncthreads();
    }
    if (a.sel) {
        // fused selection (list mode: the launch after the one-wave kernel): thread 0 reads
        // back the keys of the block's instances (its own stores, gi_write_wg) once the solves
        // are done; the solves' LDS is dead, the finalizer's scratch.  Only the workgroups that
        // had an instance take a ticket (workgroup 0 alone when the list is empty: the usual
        // case, where the launch is then little more than its dispatch)
        const int groups = count <= 0 ? 1 : (count < (int)gridDim.x ? count : (int)gridDim.x);
        if ((int)blockIdx.x >= groups) return;
        unsigned long long kmin = kSelNone;
        for (int i = blockIdx.x; i < count; i += gridDim.x) {
            const int b = ov.id(i);
            const unsigned long long k = sel_key(a.status[b], a.cost[b], a.sel_base + b);
            kmin = k < kmin ? k : kmin;
        }
        sel_commit(a, kmin, NU * N, (int)blockIdx.x < count,
                   reinterpret_cast<unsigned long long *>(smem), groups, count <= 0);
    }
}

}  // namespace mpcqp
