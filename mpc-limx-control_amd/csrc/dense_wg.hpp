// dense_wg.hpp -- the per-tick step for a DENSE continuous model (BASELINE config E: the
// 24-state whole-body linearisation of TRON1, NU = 6 joint torques, N = 16), one 4-wave
// workgroup per QP:
//
//   discretisation   [Ad | Bd] = top block of exp([[Ac, Bc], [0, 0]] Ts): Eigen's Pade degree
//                    selection + scaling and squaring (wg_expm, expm_wg.hpp: the products on
//                    the matrix cores over the workgroup)
//                                                            QPSolver::discretizeSystem,
//                                                            src/QPSolver.cpp:21-29
//   condensing       H = 2 (B'QB + R), f = 2 B'Q (A x0 - xref)   QPSolver::buildQPParams,
//                    src/QPSolver.cpp:31-81 -- the reference's dense (nx(N+1))^2 product is
//                    restructured into genuinely dense NX x NX contractions on the FP64
//                    matrix cores (mfma_ops.hpp):
//                      Phi_a = Ad^a Bd                 (a = 0..N-1, by doubling: Ad^2, Ad^4 ..)
//                      Z_{N-1} = P,  Z_i = Q + Ad' Z_{i+1} Ad      (backward recursion)
//                      Y_i = Bd' Z_i,  H(i,j) = 2 (Y_i Phi_{i-j} + R [i == j])   (i >= j)
//                    and f by the matching vector recursion s_i = W_{i+1} e_{i+1} + Ad' s_{i+1},
//                    f_i = 2 Bd' s_i (e_m = Ad^m x0 - xref_m) on the VALU
//   solve            box u_min <= u <= u_max (src/QPSolver.cpp:67-68), every input free:
//                    gi_run_wg (gi_wg.hpp) on the NV = 96 free variables
//
// The H rows reach the solver's registers through 16-row tiles of M = [Y_0; ..; Y_{N-1}] Phi
// staged in LDS (H(r, c) = 2 M(r, (k_r - k_c) NU + c mod NU)), so no NV x NV matrix is ever
// stored.  Per instance: [Ac | Bc] (NX x NS), x0, xref in; U, cost, status, iterations out.
//
// TOEP (Q = F_Q F_Q', P = F_P F_P' factored on the host at context creation, mpcqp_ctx_create):
// the recursion's 16 dependent steps are replaced by one product with no chain,
//   H = 2 (G' G + R),  G = blockdiag(F_Q', .., F_Q', F_P') Bbar,  Bbar(m, j) = Phi_{m-1-j}
// (block lower-triangular Toeplitz), i.e. H(i, j) = 2 sum_{mb >= max(i_b, j_b)}
// Psi(mb)_{mb-i_b}' Psi(mb)_{mb-j_b} with Psi_a = F' Phi_a: the 16 x 16 output tiles of H's
// lower triangle run their K = NX (N - mb0) loops on the matrix cores straight out of the two
// NX x NV Psi panels (the Toeplitz map is an address offset per lane), two row tiles per round
// (7 tiles over the 4 waves).  The gradient takes the same panels: with E = [e_1 .. e_N]
// (e_m = Ad^m x0 - xref_m; Ad^m x0 rides along the Phi doubling as extra columns),
// Gamma = Psi' F' E and f_(i_b, c) = 2 sum_{mb >= i_b} Gamma((mb - i_b) NU + c, mb).
#pragma once
#include "condense.hpp"
#include "expm_wg.hpp"
#include "gi_wg.hpp"
#include "mfma_ops.hpp"
#include "mpc_fused.hpp"

namespace mpcqp {

template <int NX, int NU, int N, bool TOEP = false>
struct DenseLayout {
    static constexpr int NS = NX + NU, NV = NU * N, NF = NV;
    static constexpr int RW = WgShape<NF>::RW;
    static constexpr int LD = NX + 1;   // odd leading dimension of the NX-row operands
    static constexpr int LY = NV + 1;   // the Y stack (NV x NX)
    static constexpr int LS = 17;       // a staged 16-row tile of M (16 x NV)
    static constexpr int MT = 2 * NF;
    // live for the whole solve: x mirror, fixed values, misc (nf, status), the bounds' b
    static constexpr int oXS = 0, oXF = oXS + RW, oMisc = oXF + NV, oCB = oMisc + 2;
    static constexpr int oU = (oCB + 2 * NF + 1) & ~1;
    // front: [Ad | Bd], x0, xref, f, then a region the phases take turns on
    static constexpr int oAB = oU;
    static constexpr int oX0 = oAB + NX * NS;
    static constexpr int oXr = oX0 + NX;
    static constexpr int oF = oXr + NX * (N + 1);
    static constexpr int oRm = oF + NV;                  // R, NU x NU (the H rows' diagonal blocks)
    static constexpr int oR = (oRm + NU * NU + 1) & ~1;
    //   discretisation view
    static constexpr int oT = oR;                       // [Ac | Bc] Ts
    static constexpr int oWs = oT + NX * NS;            // wave_expm scratch (7 NX NS)
    static constexpr int nExpm = oWs + 7 * NX * NS - oR;
    //   condensing view
    static constexpr int oPhi = oR;                     // Phi_a, NX x NV (ld LD)
    static constexpr int oPw = oPhi + LD * NV;          // 3 NX x NX (ld LD): powers, Z, Z', Z Ad
    static constexpr int oY = oPw + 3 * LD * NX;        // Y stack, NV x NX (ld LY)
    static constexpr int oXf = oY + LY * NX;            // e_m = Ad^m x0 - xref_m, NX x (N+1)
    static constexpr int oSv = oXf + NX * (N + 1);      // s_i, NX x N
    static constexpr int nCondR = oSv + NX * N - oR;
    static_assert(LS * NV <= 3 * LD * NX, "the staged M tile fits the Z region");
    //   Toeplitz condensing view: [Phi | X] (X_a = Ad^(a+1) x0, then e_(a+1)), Psi = F_Q' [Phi | E],
    //   Psi_P = F_P' [Phi | e_N]; Gamma and the H staging reuse the [Phi | X] panel once Psi is in
    static constexpr int NC = NV + N;
    static constexpr int oPx = oR;
    static constexpr int oPs = oPx + LD * NC;
    static constexpr int oPp = oPs + LD * NC;
    static constexpr int LG = NV + 1;                   // Gamma, NV x N
    static constexpr int nCondT = oPp + LD * (NV + 1) - oR;
    static constexpr int TR = (NV + 15) / 16;           // row tiles of H
    static_assert(LG * N <= LD * NC, "Gamma fits the [Phi | X] panel");
    static_assert(LS * 16 * (TR + 1 + 2) <= LD * NC,
                  "two staged row tiles and two split tiles' halves fit the [Phi | X] panel");
    static_assert(!TOEP || NX % 4 == 0, "K steps of 4 per Psi block");
    static constexpr int nCond = TOEP ? nCondT : nCondR;
    static constexpr int nFront = oR - oU + (nExpm > nCond ? nExpm : nCond);
    // solver view (after every thread holds its H_FF row part and g)
    static constexpr int nSolver = WgLayout<NF>::work;
    static constexpr int nDoubles = oU + (nFront > nSolver ? nFront : nSolver);
    static constexpr size_t bytes =
        sizeof(double) * nDoubles + sizeof(int) * (NF + NV) + ((MT + 15) & ~15);
    static constexpr size_t lds_bytes = (bytes + 15) & ~(size_t)15;
};

// One 16 x 16 tile (I, J), J <= I, of G' G (TOEP): lane li's A row i = 16 I + li and B column
// j = 16 J + li take block mb's K = NX slice from Psi(mb) at Psi_{mb - i_b}(:, c_i) -- a per-lane
// offset -- and read 0 where mb < i_b (j_b); mb starts at the tile's first row block (i >= j).
// 1: block mb + 1's operands are loaded while block mb's MFMAs run, and even / odd K steps
// go to two accumulators (measured 1.5 % slower at config E, 16,384: off)
// 0: tile t of a round to wave t % 4, no K split (A/B builds)
#ifndef MPCQP_TOEP_LPT
#define MPCQP_TOEP_LPT 1
#endif
#ifndef MPCQP_TOEP_PIPE
#define MPCQP_TOEP_PIPE 0
#endif
#ifndef MPCQP_TOEP_SPLIT
#define MPCQP_TOEP_SPLIT 1
#endif
// The H-row rounds' tile schedule (which wave takes which tile / K half, in the greedy order
// below) depends only on the shape: computed at compile time, each wave walks its own list
// (MPCQP_TOEP_SCHED; 0: every wave replays the greedy over all tiles at run time, A/B).  Same
// tiles, K ranges and waves as the run-time form (bit-identical).  E 4.60 -> 4.52 ms (r06t).
#ifndef MPCQP_TOEP_SCHED
#define MPCQP_TOEP_SCHED 1
#endif
template <int NU, int N, int TR>
struct ToepSched {
    static constexpr int R = (TR + 1) / 2, MAXE = 2 * TR + 4;
    int n[R][4];
    signed char I[R][4][MAXE], J[R][4][MAXE], lo[R][4][MAXE], hi[R][4][MAXE], fl[R][4][MAXE];
    constexpr ToepSched() : n{}, I{}, J{}, lo{}, hi{}, fl{} {
        for (int rho = 0; rho < R; ++rho) {
            const int Ia = rho, Ib = TR - 1 - rho;
            const int na = Ia + 1, nt_ = Ia == Ib ? na : na + Ib + 1;
            const int Ka = N - (16 * Ia) / NU, Kb = Ia == Ib ? 0 : N - (16 * Ib) / NU;
            const int avg = (na * Ka + (nt_ - na) * Kb + 3) / 4;
            const bool split = MPCQP_TOEP_LPT && na <= 2 && Ka > avg;
            int l[4] = {0, 0, 0, 0};
            for (int t = 0; t < nt_; ++t) {
                const int I_ = t < na ? Ia : Ib, J_ = t < na ? t : t - na;
                const int m0 = (16 * I_) / NU, K = N - m0;
                const int parts = (split && t < na) ? 2 : 1;
                for (int part = 0; part < parts; ++part) {
                    const int lo_ = part ? m0 + K / 2 : m0, hi_ = parts == 2 && !part ? m0 + K / 2 : N;
                    const int m01 = l[1] < l[0] ? l[1] : l[0], m23 = l[3] < l[2] ? l[3] : l[2];
                    const int w = !MPCQP_TOEP_LPT ? t % 4
                                                  : m23 < m01 ? (l[3] < l[2] ? 3 : 2) : (l[1] < l[0] ? 1 : 0);
                    l[w] += hi_ - lo_;
                    const int k = n[rho][w]++;
                    I[rho][w][k] = (signed char)I_;
                    J[rho][w][k] = (signed char)J_;
                    lo[rho][w][k] = (signed char)lo_;
                    hi[rho][w][k] = (signed char)hi_;
                    fl[rho][w][k] = (signed char)(part | (t < na ? 2 : 0));
                }
            }
        }
    }
};
template <int NU, int N, int TR>
__constant__ constexpr ToepSched<NU, N, TR> kToepSched{};

template <int NX, int NU, int N, int LD>
__device__ __forceinline__ dx4 toep_tile(const double *Ps, const double *Pp, int I, int J, int mlo,
                                         int mhi) {
    constexpr int NV = NU * N, KS = NX / 4;
    const int ln = lane(), li = ln & 15, lk = ln >> 4;
    const int i = 16 * I + li, j = 16 * J + li;
    const int ib = i < NV ? i / NU : N, jb = j < NV ? j / NU : N;
    const int offa = (i % NU - ib * NU) * LD + lk, offb = (j % NU - jb * NU) * LD + lk;
    const int mb0 = mlo;
    auto load = [&](int mb, double (&av)[KS], double (&bv)[KS]) {
        const double *P = (mb == N - 1 ? Pp : Ps) + mb * NU * LD;
        const bool va = mb >= ib, vb = mb >= jb;
        const double *pa = P + (va ? offa : lk), *pb = P + (vb ? offb : lk);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const double x = pa[4 * s], y = pb[4 * s];
            av[s] = va ? x : 0.0;
            bv[s] = vb ? y : 0.0;
        }
    };
    dx4 acc = {0.0, 0.0, 0.0, 0.0};
    if (MPCQP_TOEP_PIPE) {
        dx4 acc1 = {0.0, 0.0, 0.0, 0.0};
        double av[KS], bv[KS];
        load(mb0, av, bv);
        for (int mb = mb0; mb < mhi; ++mb) {
            double an[KS], bn[KS];
            load(mb + 1 < mhi ? mb + 1 : mb, an, bn);  // (the last block's re-read is discarded)
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                if (s & 1) acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc1, 0, 0, 0);
                else acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
            }
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                av[s] = an[s];
                bv[s] = bn[s];
            }
        }
        return acc + acc1;
    }
    // MPCQP_TOEP_SPLIT: from the first block where every row of both tiles is live (wave-uniform:
    // the tiles' last rows' step) the operands load without the zero selects (the same values)
    const int mfull = MPCQP_TOEP_SPLIT ? max(16 * I + 15 < NV ? (16 * I + 15) / NU : N,
                                             16 * J + 15 < NV ? (16 * J + 15) / NU : N)
                                       : N;
    const int msel = mfull < mhi ? mfull : mhi;
    for (int mb = mb0; mb < msel; ++mb) {
        double av[KS], bv[KS];
        load(mb, av, bv);
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
    }
    for (int mb = mb0 > msel ? mb0 : msel; mb < mhi; ++mb) {
        const double *P = (mb == N - 1 ? Pp : Ps) + mb * NU * LD;
        const double *pa = P + offa, *pb = P + offb;
        double av[KS], bv[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            av[s] = pa[4 * s];
            bv[s] = pb[4 * s];
        }
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
    }
    return acc;
}

template <int NX, int NU, int N, bool TOEP = false>
__device__ __forceinline__ void dense_mpc_one(const MpcArgs &a, int b, unsigned char *smem) {
    using Lay = DenseLayout<NX, NU, N, TOEP>;
    constexpr int NS = Lay::NS, NV = Lay::NV, NF = Lay::NF, RW = Lay::RW, NH = NF / 2;
    constexpr int LD = Lay::LD, LY = Lay::LY, LS = Lay::LS, NT = 2 * RW;
    const WgIds T = wg_ids<RW>();
    const int tid = T.tid, wv = T.wv, ln = T.ln, r = T.r, h = T.h;
    double *D = reinterpret_cast<double *>(smem);
    double *AB = D + Lay::oAB, *Ad = AB, *Bd = AB + NX * NX;
    double *x0 = D + Lay::oX0, *xr = D + Lay::oXr, *fv = D + Lay::oF;

    SolveProblem P;
    P.nV = NV;
    P.H = nullptr; P.f = nullptr; P.lb = nullptr; P.ub = nullptr;
    P.gen_bounds = 1;
    P.model = 2; P.nu = NU; P.N = N; P.nfeet = 2;  // input box u_min .. u_max (gen_bound)
    P.fz_min = a.fz_min; P.fz_max = a.fz_max; P.fxy_max = a.fxy_max;
    P.u_min = a.u_min; P.u_max = a.u_max;
    P.contact = 0ull;
    P.friction = 0;
    P.mu = 0.0;
    P.mA = 0; P.A = nullptr; P.a_colmajor = 0; P.lbA = nullptr; P.ubA = nullptr;
    P.max_iter = a.max_iter;
    GiCtx C;
    C.wide = 1;
    C.crash_p = a.crash_p_wg;
    C.stamps = a.stamps;
    C.cut = a.cut >= 100 ? a.cut - 100 : 0;  // (cuts build) MPCQP_CUT=100+k: the workgroup solver's cut k
    C.P = &P;
    C.nfmax = NF;
    C.L.ld = NF | 1;
    C.L.R = nullptr; C.L.J = nullptr; C.L.g = nullptr;
    C.L.xs = D + Lay::oXS;
    C.L.xfull = D + Lay::oXF;
    C.L.rowfix = D + Lay::oMisc;
    C.L.ys = D + Lay::oMisc;
    int *ip = reinterpret_cast<int *>(D + Lay::nDoubles);
    C.L.fid = ip;
    C.L.pos = ip + NF;
    C.L.st = reinterpret_cast<unsigned char *>(ip + NF + NV);
    C.L.cb = D + Lay::oCB;
    MPCQP_STAMP_INIT(tst);

    // ---- inputs: [Ac | Bc] Ts, x0, xref (coalesced over the workgroup)
    {
        const double *abg = a.lin + (size_t)b * NX * NS;
        for (int e = tid; e < NX * NS; e += NT) D[Lay::oT + e] = abg[e] * a.Ts;
        for (int e = tid; e < NX; e += NT) x0[e] = a.x0[(size_t)b * NX + e];
        const double *xrg = a.xref + (size_t)b * NX * (N + 1);
        for (int e = tid; e < NX * (N + 1); e += NT) xr[e] = xrg[e];
        for (int e = tid; e < NU * NU; e += NT) D[Lay::oRm + e] = a.rmat[e];
    }
    __syncthreads();
    // ---- discretisation (the workgroup, matrix cores) and the free map / bounds (wave 0)
    // (the free map and bounds touch only the solve-lifetime region and the int maps: the last
    //  wave sets them up while the first solves the Pade quotient; C's fields are re-read from
    //  oMisc / set uniformly below)
    wg_expm(NX, NS, D + Lay::oT, D + Lay::oWs, AB, tid, NT, wv, NT / 64, a.stamps, [&]() {
        gi_setup(C);
        if (C.nf > a.max_free) C.status = ST_BAD_DIMS;
        if (ln == 0) {
            D[Lay::oMisc] = (double)C.nf;
            D[Lay::oMisc + 1] = (double)C.status;
        }
    });
    __syncthreads();
    MPCQP_STAMP(a.stamps, 11, tst);
    MPCQP_CUT(a.cut, 91);  // (cuts build: inputs + expm + free map)

    double hr[NH];
#pragma unroll
    for (int j = 0; j < NH; ++j) hr[j] = (r == 2 * j + h) ? 1.0 : 0.0;
    int nf = 0;
    bool ok = false;
    if constexpr (TOEP) {
        // ---- [Phi | X]: Phi_a = Ad^a Bd and X_a = Ad^(a+1) x0, a = 0..N-1, by doubling
        constexpr int NC = Lay::NC;
        double *Px = D + Lay::oPx, *Ps = D + Lay::oPs, *Pp = D + Lay::oPp;
        double *Pw0 = Ps, *Pw1 = Ps + LD * NX;  // the powers of Ad, in the (not yet written) Psi
        for (int e = tid; e < NX * NU; e += NT) Px[(e / NX) * LD + e % NX] = Bd[e];
        mfma_gemm<false>(NX, 1, NX, Ad, NX, x0, NX, Px + NV * LD, LD, nullptr, 0, 1.0, wv, 2, 2);
        __syncthreads();
        {
            const double *pw = Ad;
            int ldp = NX;
            double *nxt = Pw0, *oth = Pw1;
            for (int p2 = 1; p2 < N; p2 *= 2) {
                const int nb = p2 < N - p2 ? p2 : N - p2;
                const bool more = 2 * p2 < N;
                mfma_gemm<false>(NX, nb * NU, NX, pw, ldp, Px, LD, Px + p2 * NU * LD, LD, nullptr, 0,
                                 1.0, wv, 0, 4);
                mfma_gemm<false>(NX, nb, NX, pw, ldp, Px + NV * LD, LD, Px + (NV + p2) * LD, LD,
                                 nullptr, 0, 1.0, wv, 2, 2);
                if (more)
                    mfma_gemm<false>(NX, NX, NX, pw, ldp, pw, ldp, nxt, LD, nullptr, 0, 1.0, wv, 0, 4);
                __syncthreads();
                if (more) {
                    pw = nxt;
                    ldp = LD;
                    double *t_ = nxt;
                    nxt = oth;
                    oth = t_;
                }
            }
        }
        // e_m = Ad^m x0 - xref_m in place of X_(m-1)
        for (int e = tid; e < NX * N; e += NT) Px[(NV + e / NX) * LD + e % NX] -= xr[NX + e];
        __syncthreads();
        // ---- Psi = F_Q' [Phi | E], Psi_P = F_P' [Phi | e_N] (F from global memory)
        mfma_gemm<true>(NX, NC, NX, a.fq, NX, Px, LD, Ps, LD, nullptr, 0, 1.0, wv, 0, 4);
        mfma_gemm<true>(NX, NV, NX, a.fp, NX, Px, LD, Pp, LD, nullptr, 0, 1.0, wv, 0, 4);
        mfma_gemm<true>(NX, 1, NX, a.fp, NX, Px + (NC - 1) * LD, LD, Pp + NV * LD, LD, nullptr, 0,
                        1.0, wv, 2, 2);
        __syncthreads();
        MPCQP_STAMP(a.stamps, 1, tst);
        // ---- gradient: Gamma(:, mb) = Psi(mb)' w_mb (the e columns of Psi / Psi_P), then
        //      f_(i_b, c) = 2 sum_{mb >= i_b} Gamma((mb - i_b) NU + c, mb)
        double *G = Px;
        constexpr int LG = Lay::LG;
        mfma_gemm<true>(NV, N - 1, NX, Ps, LD, Ps + NV * LD, LD, G, LG, nullptr, 0, 1.0, wv, 0, 4);
        mfma_gemm<true>(NV, 1, NX, Pp, LD, Pp + NV * LD, LD, G + (N - 1) * LG, LG, nullptr, 0, 1.0,
                        wv, 0, 4);
        __syncthreads();
        for (int e = tid; e < NV; e += NT) {
            const int ib = e / NU, c = e % NU;
            double s = 0.0;
            for (int mb = ib; mb < N; ++mb) s += G[mb * LG + (mb - ib) * NU + c];
            fv[e] = 2.0 * s;
        }
        __syncthreads();
        C.nf = (int)D[Lay::oMisc];
        C.status = (int)D[Lay::oMisc + 1];
        nf = C.nf;
        ok = C.status == ST_OK && nf > 0;
        MPCQP_STAMP(a.stamps, 4, tst);
        MPCQP_CUT(a.cut, 92);  // (cuts build: + [Phi | X], Psi, gradient)
        // ---- H rows: rounds of two row tiles (rho, TR-1-rho): their 16 I + 16 tiles of G' G
        //      over the waves, staged (rows of I at stg, of I' after them), then every thread
        //      takes H(r, c) = 2 (G'G(r, c) + R(c_c, c_r) [k_r == k_c]), c = 2j + h <= r
        constexpr int TR = Lay::TR;
        double *stg = Px;
        MPCQP_STAMP_INIT(th);  // diagnostic build: tiles (slot 2) and row pickup (slot 10)
        for (int rho = 0; rho < (TR + 1) / 2; ++rho) {
            const int Ia = rho, Ib = TR - 1 - rho;
            const int na = Ia + 1, nt_ = Ia == Ib ? na : na + Ib + 1;
            double *sb = stg + LS * 16 * na;
            // the K blocks of a tile: mb = its first row block .. N-1.  Greedy over the waves in
            // tile order (the first row tile's K are the larger); when the first row tile's K
            // exceeds a quarter of the round (only for <= 2 tiles: the staging room), its tiles
            // go out as two K halves, the second half staged apart (ex) and added before pickup
            const int Ka = N - (16 * Ia) / NU, Kb = Ia == Ib ? 0 : N - (16 * Ib) / NU;
            const int avg = (na * Ka + (nt_ - na) * Kb + 3) / 4;
            const bool split = MPCQP_TOEP_LPT && na <= 2 && Ka > avg;
            double *ex = stg + LS * 16 * (Ia == Ib ? na : na + Ib + 1);
            if constexpr (MPCQP_TOEP_SCHED) {
                const auto &TS = kToepSched<NU, N, TR>;
                const int ne = TS.n[rho][wv];
                for (int k = 0; k < ne; ++k) {
                    const int I = TS.I[rho][wv][k], J = TS.J[rho][wv][k], f = TS.fl[rho][wv][k];
                    const dx4 acc = toep_tile<NX, NU, N, LD>(Ps, Pp, I, J, TS.lo[rho][wv][k],
                                                             TS.hi[rho][wv][k]);
                    double *st_ = (f & 1) ? ex + J * 16 * LS : ((f & 2) ? stg : sb) + 16 * J * LS;
#pragma unroll
                    for (int q = 0; q < 4; ++q) st_[(ln & 15) * LS + (ln >> 4) + 4 * q] = acc[q];
                }
            }
            int l0 = 0, l1 = 0, l2 = 0, l3 = 0;  // K blocks handed to each wave so far
            for (int t = 0; t < (MPCQP_TOEP_SCHED ? 0 : nt_); ++t) {
                const int I = t < na ? Ia : Ib, J = t < na ? t : t - na;
                const int m0 = (16 * I) / NU, K = N - m0;
                const int parts = (split && t < na) ? 2 : 1;
                for (int part = 0; part < parts; ++part) {
                    const int lo = part ? m0 + K / 2 : m0, hi = parts == 2 && !part ? m0 + K / 2 : N;
                    const int m01 = l1 < l0 ? l1 : l0, m23 = l3 < l2 ? l3 : l2;
                    const int w = !MPCQP_TOEP_LPT ? t % 4 : m23 < m01 ? (l3 < l2 ? 3 : 2) : (l1 < l0 ? 1 : 0);
                    l0 += w == 0 ? hi - lo : 0;
                    l1 += w == 1 ? hi - lo : 0;
                    l2 += w == 2 ? hi - lo : 0;
                    l3 += w == 3 ? hi - lo : 0;
                    if (w != wv) continue;
                    const dx4 acc = toep_tile<NX, NU, N, LD>(Ps, Pp, I, J, lo, hi);
                    double *st_ = part ? ex + J * 16 * LS : (t < na ? stg : sb) + 16 * J * LS;
#pragma unroll
                    for (int q = 0; q < 4; ++q) st_[(ln & 15) * LS + (ln >> 4) + 4 * q] = acc[q];
                }
            }
            __syncthreads();
            if (split) {  // the second K halves onto the first (same tile layout)
                for (int e = tid; e < na * 16 * LS; e += NT) stg[e] += ex[e];
                __syncthreads();
            }
            MPCQP_STAMP(a.stamps, 2, th);
            const int Ir = r >> 4;
            if (ok && (Ir == Ia || Ir == Ib) && r < nf) {
                const double *st_ = Ir == Ia ? stg : sb;
                const int kr = r / NU, cr = r % NU, rr = r & 15;
#pragma unroll
                for (int j = 0; j < NH; ++j) {
                    const int c = 2 * j + h;
                    if (c <= r) {
                        const int kc = c / NU, cc = c % NU;
                        double v = st_[c * LS + rr];
                        if (kr == kc) v += D[Lay::oRm + cc * NU + cr];
                        hr[j] = 2.0 * v;
                    }
                    if ((j & 7) == 7) step_fence();
                }
            }
            __syncthreads();
            MPCQP_STAMP(a.stamps, 10, th);
        }
    } else {
        // ---- Phi_a = Ad^a Bd, a = 0..N-1, by doubling: Phi[p .. p+nb) = Ad^p Phi[0 .. nb)
        double *Phi = D + Lay::oPhi, *Pw0 = D + Lay::oPw, *Pw1 = Pw0 + LD * NX, *Pw2 = Pw1 + LD * NX;
        for (int e = tid; e < NX * NU; e += NT) Phi[(e / NX) * LD + e % NX] = Bd[e];
        __syncthreads();
        {
            const double *pw = Ad;
            int ldp = NX;
            double *nxt = Pw0, *oth = Pw1;
            for (int p2 = 1; p2 < N; p2 *= 2) {
                const int nb = p2 < N - p2 ? p2 : N - p2;
                const bool more = 2 * p2 < N;
                mfma_gemm<false>(NX, nb * NU, NX, pw, ldp, Phi, LD, Phi + p2 * NU * LD, LD, nullptr, 0,
                                 1.0, wv, 0, more ? 2 : 4);
                if (more)
                    mfma_gemm<false>(NX, NX, NX, pw, ldp, pw, ldp, nxt, LD, nullptr, 0, 1.0, wv, 2, 2);
                __syncthreads();
                if (more) {
                    pw = nxt;
                    ldp = LD;
                    double *t_ = nxt;
                    nxt = oth;
                    oth = t_;
                }
            }
        }
        // ---- Z_{N-1} = P, Z_i = Q + Ad' Z_{i+1} Ad;  Y_i = Bd' Z_i into the stack's rows i NU ..
        double *Y = D + Lay::oY;
        for (int e = tid; e < NX * NX; e += NT) Pw0[(e / NX) * LD + e % NX] = a.pm[e];
        __syncthreads();
        {
            double *Zc = Pw0, *Zn = Pw1;
            for (int i = N - 1; i >= 0; --i) {
                mfma_gemm<true>(NU, NX, NX, Bd, NX, Zc, LD, Y + i * NU, LY, nullptr, 0, 1.0, wv, 0, 2);
                if (i > 0)
                    mfma_gemm<false>(NX, NX, NX, Zc, LD, Ad, NX, Pw2, LD, nullptr, 0, 1.0, wv, 2, 2);
                __syncthreads();
                if (i > 0) {
                    mfma_gemm<true>(NX, NX, NX, Ad, NX, Pw2, LD, Zn, LD, a.qm, NX, 1.0, wv, 0, 4);
                    __syncthreads();
                    double *t_ = Zc;
                    Zc = Zn;
                    Zn = t_;
                }
            }
        }
        MPCQP_STAMP(a.stamps, 1, tst);
        // ---- gradient (wave 0): e_m = Ad^m x0 - xref_m, s_{N-1} = P e_N,
        //      s_i = Q e_{i+1} + Ad' s_{i+1}, f_i = 2 Bd' s_i
        if (wv == 0) {
            double *xf = D + Lay::oXf, *sv = D + Lay::oSv;
            if (ln < NX) xf[ln] = x0[ln];
            wave_sync();
            for (int m = 1; m <= N; ++m) {
                if (ln < NX) {
                    double s = 0.0;
#pragma unroll
                    for (int l = 0; l < NX; ++l) s += Ad[l * NX + ln] * xf[(m - 1) * NX + l];
                    xf[m * NX + ln] = s;
                }
                wave_sync();
            }
            for (int e = ln; e < NX * N; e += kWave) xf[NX + e] -= xr[NX + e];
            wave_sync();
            for (int i = N - 1; i >= 0; --i) {
                if (ln < NX) {
                    const double *W = (i + 1 < N) ? a.qm : a.pm;
                    double s = 0.0;
#pragma unroll
                    for (int l = 0; l < NX; ++l) s += W[l * NX + ln] * xf[(i + 1) * NX + l];
                    if (i + 1 < N) {
#pragma unroll
                        for (int l = 0; l < NX; ++l) s += Ad[ln * NX + l] * sv[(i + 1) * NX + l];
                    }
                    sv[i * NX + ln] = s;
                }
                wave_sync();
            }
            for (int e = ln; e < NV; e += kWave) {
                const int i = e / NU, c = e % NU;
                double s = 0.0;
#pragma unroll
                for (int l = 0; l < NX; ++l) s += Bd[c * NX + l] * sv[i * NX + l];
                fv[e] = 2.0 * s;
            }
        }
        __syncthreads();
        C.nf = (int)D[Lay::oMisc];
        C.status = (int)D[Lay::oMisc + 1];
        nf = C.nf;
        ok = C.status == ST_OK && nf > 0;
        MPCQP_STAMP(a.stamps, 4, tst);

        // ---- H rows: 16-row tiles of M = Y Phi staged over the Z region; thread (r, h) takes
        //      H(r, c) = 2 (M(r, (k_r - k_c) NU + c mod NU) + R(c_r, c_c) [k_r == k_c]), c = 2j + h
        //      <= r (gi_run_wg's interleaved factorisation layout; identity beyond nf)
        double *stg = Pw0;
        for (int r0 = 0; r0 < NV; r0 += 16) {
            const int nrow = NV - r0 < 16 ? NV - r0 : 16;
            const int ncol = ((r0 + nrow - 1) / NU + 1) * NU;  // columns a NU + c with a <= k_r
            mfma_gemm<false, false>(nrow, ncol, NX, Y + r0, LY, Phi, LD, stg, LS, nullptr, 0, 1.0, wv, 0, 4);
            __syncthreads();
            if (ok && r >= r0 && r < r0 + nrow && r < nf) {
                const int kr = r / NU, cr = r % NU;
#pragma unroll
                for (int j = 0; j < NH; ++j) {
                    const int c = 2 * j + h;
                    if (c <= r) {
                        const int kc = c / NU, cc = c % NU;
                        double v = stg[((kr - kc) * NU + cc) * LS + (r - r0)];
                        if (kr == kc) v += a.rmat[cc * NU + cr];
                        hr[j] = 2.0 * v;
                    }
                    if ((j & 7) == 7) step_fence();
                }
            }
            __syncthreads();
        }
    }
    C.nfric = 0;
    C.mt = 2 * C.nf;
    C.c0 = 0.0;
    const double g = (ok && r < nf) ? fv[C.L.fid[r]] : 0.0;
    __syncthreads();  // the solver's workspace overlays the front
    MPCQP_STAMP(a.stamps, 3, tst);
    MPCQP_CUT(a.cut, 93);  // (cuts build: + the H rows)
    gi_run_wg<NF, true>(C, hr, g, D + Lay::oU);
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

}  // namespace mpcqp
