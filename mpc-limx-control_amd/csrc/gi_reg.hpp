// gi_reg.hpp -- register-resident Goldfarb-Idnani solve for up to NF <= 64 free variables.
//
// Same algorithm, constraint order and tolerances as gi_run (gi_solver.hpp) and the CPU
// oracle; only the storage differs:
//   * lane i holds row i of H_FF, then of L (Cholesky, right-looking, in place) -- h[NF];
//     g rides along as an extra column, so the same sweep leaves t = L^-1 g on the lanes
//   * L is parked in LDS (row-major packed), then lane c computes column c of L^-1 by
//     forward substitution; since J = L^-T, that column is row c of J, which lane c keeps in
//     registers -- Jr[NF]; the unconstrained minimum is x = -J t, objective -|t|^2 / 2
//   * R lives in LDS, column-major packed with one sub-diagonal slot per column (the drop
//     step's Hessenberg entry), reusing the parked-L space: NF(NF+3)/2 doubles in total
//   * an add step updates J by a Householder reflection (2 NF FMAs), a drop step by Givens
//     rotations (as the oracle); the two differ from the oracle's Givens-chain add only in
//     rounding
//   * x is mirrored in LDS (xs) for the constraint sweeps, with the constraint states
// All loops over columns are unrolled to NF with wave-uniform predicates, so every register
// index is a compile-time constant (no scratch), and cross-lane reads are v_readlane with
// constant lane indices.
#pragma once
#include "chol_reg.hpp"
#include "gi_crash_reg.hpp"
#include "gi_solver.hpp"

namespace mpcqp {

// packed R: column j holds rows 0..j+1 (j+1 = the Hessenberg slot of the drop step)
__device__ __forceinline__ int roff(int j) { return j * (j + 3) / 2; }
// packed L (parked for the inverse): row i holds columns 0..i
__host__ __device__ constexpr int lrow(int i) { return i * (i + 1) / 2; }
// column-major packed L kept during the factorisation: column k holds rows k..NF-1 and
// starts 16-byte aligned (two doubles)
__host__ __device__ constexpr int ccol(int k, int nf) {
    return k == 0 ? 0 : ccol(k - 1, nf) + ((nf - (k - 1) + 1) & ~1);
}
template <int NF>
struct RegPack {
    static constexpr int doubles = NF * (NF + 3) / 2;  // >= lrow(NF): L fits in R's space
    static_assert(ccol(NF, NF) <= doubles, "column-packed L fits the R space");
};

// Row-broadcast of J: d_j = c0 J(a0, j) [+ c1 J(a1, j)] on lane j.  The owning lanes publish
// their J rows to LDS (buf[0, NF) and buf[NF, 2NF)); every lane reads its column.
template <int NF>
__device__ __forceinline__ double reg_project(const double (&Jr)[NF], int a0, double c0,
                                              int a1, double c1, double *buf) {
    const int ln = lane();
    if (ln == a0) {
#pragma unroll
        for (int c = 0; c < NF; ++c) buf[c] = Jr[c];
    }
    if (a1 >= 0 && ln == a1) {
#pragma unroll
        for (int c = 0; c < NF; ++c) buf[NF + c] = Jr[c];
    }
    wave_sync();
    double d = 0.0;
    if (ln < NF) {
        d = c0 * buf[ln];
        if (a1 >= 0) d += c1 * buf[NF + ln];
    }
    wave_sync();
    return d;
}

template <int NF>
__device__ __forceinline__ void gi_project_reg(const GiCtx &C, const double (&Jr)[NF], int id, double x,
                                      double &dj, double &sp, double *rowbuf) {
    const SolveProblem &P = *C.P;
    const GiLds &L = C.L;
    const int nf = C.nf, nfric = C.nfric, ln = lane();
    const double b = id < 2 * nf ? L.cb[id] : gi_cons_b(C, id);
    if (id < 2 * nf) {
        const int a = id < nf ? id : id - nf;
        const double sg = id < nf ? 1.0 : -1.0;
        dj = reg_project<NF>(Jr, a, sg, -1, 0.0, rowbuf);
        sp = sg * readlane(x, a) - b;
    } else {
        // friction row (the fast path has no dense rows)
        const int r = id - 2 * nf, ks = r >> 2, t = r & 3;
        const int k = ks / P.nfeet, sft = ks % P.nfeet;
        const int pz = L.pos[k * P.nu + 3 * sft + 2], pt = L.pos[k * P.nu + 3 * sft + (t >> 1)];
        const double sg = (t & 1) ? 1.0 : -1.0;
        double nx_ = 0.0;
        if (pz >= 0 && pt >= 0) {
            dj = reg_project<NF>(Jr, pz, P.mu, pt, sg, rowbuf);
            nx_ = P.mu * readlane(x, pz) + sg * readlane(x, pt);
        } else if (pz >= 0) {
            dj = reg_project<NF>(Jr, pz, P.mu, -1, 0.0, rowbuf);
            nx_ = P.mu * readlane(x, pz);
        } else {
            dj = reg_project<NF>(Jr, pt, sg, -1, 0.0, rowbuf);
            nx_ = sg * readlane(x, pt);
        }
        sp = nx_ - b;
    }
    (void)nfric;
    if (ln >= nf) dj = 0.0;
}

// Warm start of the dual loop from the previous tick's active set (the closed-loop rollout,
// SURVEY.md 8f row 2; QPSolver::updateState, src/QPSolver.cpp:108-111, then the next tick's
// solveQP).  words: bit v = lower bound of input v, bit nV + v = its upper bound, bit
// 2 nV + 4 (k nfeet + s) + t = friction row t of foot s at step k (global numbering, so the
// set survives a change of the free-variable map).  The previous horizon shifted by one step
// (step k here = step k + 1 there; the last step repeats) marks guessed constraints; while any
// guessed constraint is violated the selection takes the lowest-id one of those instead of
// the most violated one, and each is guessed only once.  The optimum is the same unique point;
// only the order of the adds (and so the number of drops) changes.  The final active set is
// written back over the same words.
struct WarmSet {
    unsigned long long *words;  // this instance's words (read at the start, written at the end)
    int n;                      // words per instance
};
__device__ __forceinline__ bool warm_bit(const unsigned long long *w, int i) {
    return (w[i >> 6] >> (i & 63)) & 1ull;
}

// h: lane p holds row p of H_FF (columns < nf meaningful), g: lane p holds g_p.
// rowbuf: 5 NF doubles of LDS (16-byte aligned): row / column broadcast buffers, the
// rotation pairs and 1/R(j,j).  Broadcasts go through LDS (one ds_read_b128 brings two values to every
// lane) rather than v_readlane pairs, which cost VALU issue slots.  Fills C.{status,x,u,fval,act,q,iters}.
// TILES: the start comes from the packed H_FF in L.R (Hb) through the blocked MFMA
// factorisation of chol_reg.hpp instead of the column sweeps over h (h unused).
// The dual loop keeps R^-1 (column-major packed, (i, j) at lrow(j) + i, in L.R) instead of R:
// r = R^-1 d is a product whose loads pipeline instead of a back substitution whose every step
// waits on the previous one; the add writes column q = (-r / r_qq, 1 / r_qq); a drop computes
// every Givens rotation at once from a prefix sum over row k of R^-1 and each lane carries its
// row through the columns (gi_wg.hpp, mpc_pair.hpp).  0 keeps R (A/B builds).
#ifndef MPCQP_REG_RINV
#define MPCQP_REG_RINV 1
#endif

template <int NF, bool TILES = false>
__device__ __forceinline__ void gi_run_reg(GiCtx &C, double (&h)[NF], double g, double *rowbuf,
                                           const WarmSet *warm = nullptr) {
    static_assert(NF <= kWave, "register path holds at most 64 free variables");
    GiLds &L = C.L;
    const SolveProblem &P = *C.P;
    const int nf = C.nf, ln = lane(), mt = C.mt;
    int status = C.status;
    double fval = 0.0, x = 0.0, u = 0.0;
    int iters = 0, q = 0, act = -1;
    double Jr[NF];
    constexpr bool T63 = NF < kWave;  // lane 63 computes t = L^-1 g in the inverse sweep
    double gv = g;     // lane i: g_i, then t_i = (L^-1 g)_i (fused path, NF == 64)
    double *colb = rowbuf + NF, *rot = rowbuf + 2 * NF, *rinv = rowbuf + 4 * NF;
    double *Lc = L.R;  // column-packed L (the R space is free until the dual loop)
    MPCQP_STAMP_INIT(tst);

    if constexpr (TILES) {
        if (status == ST_OK && nf > 0) {
            bool bad = false;
            double tt = 0.0;
            static_assert(RegPack<NF>::doubles >= 608, "chol_reg.hpp scratch fits the R space");
            reg_chol_inverse_mfma<NF>(L.R, nf, g, L.R, Jr, tt, bad);
            if (bad) status = ST_NOT_PD;
            gv = (ln < NF) ? tt : 0.0;
            if (ln < NF) colb[ln] = gv;
            wave_sync();
        }
        MPCQP_STAMP(C.stamps, 5, tst); MPCQP_CUT(C.cut, 4);
    }
    if (!TILES && status == ST_OK && nf > 0) {
        // ---- Cholesky, right-looking; lane i owns row i.  h is padded with the identity
        //      beyond nf (and g with 0), so every step runs unpredicated (upper-triangle junk
        //      is never read).  The forward solve L t = g runs in the same sweep.
        //      Look-ahead: lane k+1's own L(k+1,k) gives the next pivot without waiting for
        //      the LDS broadcast, so the pivot's rsqrt overlaps the step's bulk update.
        //      With NF < 64, lane 63 is free: it carries g as an extra column through the
        //      inverse sweep instead (T63), which keeps the forward solve out of this loop.
        double piv = readlane(h[0], 0);
        bool bad = !(piv > 0.0);
        double ik = rsqrt_nr(piv);
        //      Columns go in pairs: column k+1 is finished in registers from column k's
        //      broadcast entry L(k+1, k), so one LDS write -> read round trip serves two
        //      columns.  Per element the operations and their order are those of two
        //      single-column steps.
        static_assert(NF % 2 == 0, "column pairs");
#pragma unroll
        for (int k = 0; k < NF; k += 2) {
            // on lane k, h[k] is the pivot itself, so lik there is L(k,k) = piv / sqrt(piv)
            const double lik = h[k] * ik;
            h[k] = lik;
            const double ck1 = readlane(lik, k + 1);  // L(k+1, k)
            h[k + 1] -= lik * ck1;                    // column k's update of column k+1
            const double piv1 = readlane(h[k + 1], k + 1);
            bad |= !(piv1 > 0.0);
            const double ik1 = rsqrt_nr(piv1);
            const double lik1 = h[k + 1] * ik1;
            h[k + 1] = lik1;
            if constexpr (!T63) {
                const double tk = readlane(gv, k) * ik;
                gv = (ln == k) ? tk : ((ln > k) ? gv - lik * tk : gv);
                const double tk1 = readlane(gv, k + 1) * ik1;
                gv = (ln == k + 1) ? tk1 : ((ln > k + 1) ? gv - lik1 * tk1 : gv);
            }
            double pivn = 1.0, ikn = 1.0;
            if (k + 2 < NF) {
                const double hk2 = h[k + 2 < NF ? k + 2 : k] - lik * lik;  // on lane k+2
                pivn = readlane(hk2 - lik1 * lik1, k + 2);
                bad |= !(pivn > 0.0);
                ikn = rsqrt_nr(pivn);
            }
            // columns k, k+1 of L (diagonal first) into LDS: the broadcasts for this step's
            // update and, kept, the operands of the inverse sweep; 1/L(k,k) beside them
            if (ln >= k && ln < NF) Lc[ccol(k, NF) + ln - k] = lik;
            if (ln >= k + 1 && ln < NF) Lc[ccol(k + 1, NF) + ln - k - 1] = lik1;
            if (ln == 0) { rowbuf[k] = ik; rowbuf[k + 1] = ik1; }
            wave_sync();
#pragma unroll
            for (int j = 0; j < NF; ++j)
            {
                if (j > k + 1) {
                    h[j] -= lik * Lc[ccol(k, NF) + j - k];
                    h[j] -= lik1 * Lc[ccol(k + 1, NF) + j - k - 1];
                }
                if ((j & 3) == 3 && j > k + 1) step_fence();  // bound the loads in flight
            }
#pragma unroll
            for (int j = 0; j < NF; ++j)
                if (j >= k) pin(h[j]);  // the pair's updates happen in the pair's step
            if constexpr (!T63) pin(gv);
            piv = pivn;
            ik = ikn;
            pin(piv);
            pin(ik);
            step_fence();
        }
        if (bad) status = ST_NOT_PD;
    }
    if constexpr (!TILES) { MPCQP_STAMP(C.stamps, 5, tst); MPCQP_CUT(C.cut, 4); }
    if (status == ST_OK && nf > 0) {
      if constexpr (!TILES) {
        // ---- columns of L^-1, right-looking: lane c solves L y = e_c (lane 63: L t = g when
        //      NF < 64) column by column of L, whose entries are uniform-address LDS
        //      broadcasts; a step's updates are independent FMAs.  y = column c of L^-1 =
        //      row c of J, kept in registers.  Lanes >= NF start from 0 and stay 0.
        if constexpr (T63) {
            if (ln < NF) colb[ln] = gv;  // g, the right-hand side of lane 63
        }
        wave_sync();
#pragma unroll
        for (int l = 0; l < NF; ++l) {
            Jr[l] = (ln == l) ? 1.0 : 0.0;
            if constexpr (T63) Jr[l] = (ln == kWave - 1) ? colb[l] : Jr[l];
        }
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            Jr[i] *= rowbuf[i];
#pragma unroll
            for (int l = 0; l < NF; ++l) {
                if (l > i) Jr[l] -= Lc[ccol(i, NF) + l - i] * Jr[i];
                if ((l & 15) == 15 && l > i) step_fence();  // bound the loads in flight
            }
#pragma unroll
            for (int l = 0; l < NF; ++l)
                if (l >= i) pin(Jr[l]);
            step_fence();  // keep step i's loads and arithmetic in step i
        }
        MPCQP_STAMP(C.stamps, 6, tst); MPCQP_CUT(C.cut, 5);
        // ---- unconstrained minimum x = -J t, objective -|t|^2/2 (t_j = 0 beyond nf)
        if constexpr (T63) {
            wave_sync();
            if (ln == kWave - 1) {  // lane 63 publishes t (its Jr row); its Jr is junk from now
#pragma unroll
                for (int j = 0; j < NF; ++j) colb[j] = Jr[j];
            }
        } else {
            if (ln < NF) colb[ln] = gv;
        }
        wave_sync();
        if constexpr (T63) gv = (ln < NF) ? colb[ln] : 0.0;
      }
        double s4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            s4[j & 3] += Jr[j] * colb[j];
            if ((j & 7) == 7) step_fence();
        }
        x = (ln < nf) ? -((s4[0] + s4[1]) + (s4[2] + s4[3])) : 0.0;
        fval = -0.5 * wave_sum(ln < nf ? gv * gv : 0.0);
        if (ln < nf) L.xs[ln] = x;
        wave_sync();
    }
    MPCQP_STAMP(C.stamps, 7, tst); MPCQP_CUT(C.cut, 6);

    // ---- dual active-set loop, flattened: one pass = one step (add or drop).  J changes at
    //      the end of the pass in wave-uniform code (a reflection for an add, a rotation
    //      sequence read from LDS for a drop), so the register allocator keeps one copy of Jr.
    const int max_iter = P.max_iter > 0 ? P.max_iter : 10 * (mt + nf + 1);
    bool done = (status != ST_OK) || nf == 0;
    bool fresh = true;  // select a new violated constraint
    int p = 0;
    // Lane l evaluates the constraints of its own variable: its two bounds (ids l, l + nf)
    // and, when it is the vertical force of a foot in contact, that foot-step's four friction
    // rows (ids fbase .. fbase + 3).  A foot in contact has all three forces free (the fast
    // path's bounds guarantee it), at consecutive positions l-2, l-1, l, so the rows' x comes
    // from the two lanes below by DPP and their b is 0 (no fixed part): one LDS round trip for
    // the states instead of a strided sweep with dependent position / mirror reads.  Same
    // slack arithmetic, same (value, id) order as that sweep (gi_cons_b / gi_fric_nx_lane).
    int fbase = -1;
    if (C.nfric > 0 && status == ST_OK && ln < nf) {
        const int v = L.fid[ln], k = v / P.nu, c = v % P.nu, sft = c / 3;
        if (c % 3 == 2 && ((P.contact >> (2 * k + sft)) & 1ull))
            fbase = 2 * nf + 4 * (k * P.nfeet + sft);
    }
    int gmask = 0;  // guessed constraints of this lane: bit 0 lower, 1 upper, 2 + t friction row t
    if (warm && status == ST_OK && ln < nf) {
        const unsigned long long *w = warm->words;
        const int v = L.fid[ln], k = v / P.nu, c = v % P.nu;
        const int ks = k + 1 < P.N ? k + 1 : k;
        const int vs = ks * P.nu + c;
        if (warm_bit(w, vs)) gmask |= 1;
        if (warm_bit(w, P.nV + vs)) gmask |= 2;
        if (fbase >= 0) {
            const int fb = 2 * P.nV + 4 * (ks * P.nfeet + c / 3);
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (warm_bit(w, fb + t)) gmask |= 4 << t;
        }
    }
// (off: on config C's friction problems the primal-dual iteration stalls on the degenerate
//  pyramid apex of unloaded feet -- tools/crash_sim_friction.py: even the optimum's own active
//  set converges for 209 of 256 instances, the rest cycle -- so the rollouts measured 1.03x the
//  cold loop's iterations with it against 0.89x without)
#ifndef MPCQP_REG_WARM_CRASH
#define MPCQP_REG_WARM_CRASH 0
#endif
    // warm start: the seeded set solved in one working-set step (gi_crash_reg.hpp); the dual
    // loop below runs only if that start gives up (then exactly as without it)
    if constexpr (RegCrashLayout<NF>::end <= RegPack<NF>::doubles) {  // (NF = 60, 64)
        if (MPCQP_REG_WARM_CRASH && warm && !done && __ballot(gmask != 0) != 0ull) {
            if (reg_warm_crash<NF>(C, Jr, fbase, gmask, x, fval, iters, L.R)) done = true;
            gmask = 0;  // (after a give-up the dual loop runs cold)
        }
    }
    MPCQP_SUB_INIT(tsub);
    while (!done) {
        MPCQP_SUB(tsub, 3);
        if (fresh) {
            // ---- step 1: most violated inactive constraint (lowest id on ties)
            double best = INFINITY;
            int bid = 0x7fffffff;
            const bool qsel = C.nfric > 0 && P.contact != 0ull;  // (gi_sel_key)
            if (ln < nf) {
                const unsigned char s0 = L.st[ln], s1 = L.st[ln + nf];
                const double b0 = L.cb[ln], b1 = L.cb[ln + nf];
                if (s0 == 1) {
                    const double sl_ = x - b0;
                    if (sl_ < -kFeasTol * (1.0 + fabs(b0))) {
                        best = (gmask & 1) ? -INFINITY : gi_sel_key(sl_, qsel);
                        bid = ln;
                    }
                }
                if (s1 == 1) {
                    const double sl_ = -x - b1;
                    const double kv = (gmask & 2) ? -INFINITY : gi_sel_key(sl_, qsel);
                    if (sl_ < -kFeasTol * (1.0 + fabs(b1)) && kv < best) { best = kv; bid = ln + nf; }
                }
            }
            if (C.nfric > 0) {
                const double xm1 = wave_prev(x), xm2 = wave_prev(xm1);  // x_{l-1} (fy), x_{l-2} (fx)
                if (fbase >= 0) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        if (L.st[fbase + t] != 1) continue;
                        const double sg = (t & 1) ? 1.0 : -1.0;
                        double s = 0.0;
                        s += P.mu * x;
                        s += sg * ((t >> 1) ? xm1 : xm2);
                        const double sl_ = s - 0.0;
                        const double kv = (gmask & (4 << t)) ? -INFINITY : gi_sel_key(sl_, qsel);
                        if (sl_ < -kFeasTol * (1.0 + fabs(0.0)) && kv < best) { best = kv; bid = fbase + t; }
                    }
                }
            }
            wave_argmin(best, bid);
            if (bid == 0x7fffffff) break;  // optimal
            p = bid;
            if (ln == q) u = 0.0;
            fresh = false;
            if (gmask) {  // a guess is used once
                if (p < nf) { if (ln == p) gmask &= ~1; }
                else if (p < 2 * nf) { if (ln == p - nf) gmask &= ~2; }
                else if (fbase >= 0 && p >= fbase && p < fbase + 4) gmask &= ~(4 << (p - fbase));
            }
        }
        double dj, sp;
        MPCQP_SUB(tsub, 0);
        gi_project_reg<NF>(C, Jr, p, x, dj, sp, rowbuf);
        MPCQP_SUB(tsub, 1);
        // ---- step 2
        if (iters >= max_iter) { status = ST_ITER_LIMIT; break; }
        ++iters;
        double dd = ln < nf ? dj * dj : 0.0;
        double zn = (ln >= q && ln < nf) ? dj * dj : 0.0;
        double zq = (ln > q && ln < nf) ? dj * dj : 0.0;  // |d2|^2 without d_q
        wave_sum3(dd, zn, zq);
        if (ln < NF) colb[ln] = (ln >= q) ? dj : 0.0;  // d_j = 0 for j >= nf
        if (MPCQP_REG_RINV && ln < NF) rinv[ln] = dj;   // d (the R^-1 product reads it)
        wave_sync();
        double z4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            z4[j & 3] += Jr[j] * colb[j];
            if ((j & 7) == 7) step_fence();
        }
        double z = (z4[0] + z4[1]) + (z4[2] + z4[3]);
        pin(z);  // here, not sunk to its use after the R solve: the row would stay live
        // r = R^-1 d(0:q) (R in LDS, 1/R(j,j) kept beside it); nothing to do while q == 0
        double r = 0.0, t1 = INFINITY;
        int kslot = 0x7fffffff;
        if (MPCQP_REG_RINV && q > 0) {
            // r_i = sum_{j = i}^{q-1} R^-1(i, j) d_j: lane i reads row i of R^-1 against the
            // broadcast d_j; two accumulators, the loads of four columns issued together
            double a0 = 0.0, a1 = 0.0;
            int j = 0;
            for (; j + 1 < q; j += 2) {
                const double v0 = L.R[ln <= j ? lrow(j) + ln : 0], d0 = rinv[j];
                const double v1 = L.R[ln <= j + 1 ? lrow(j + 1) + ln : 0], d1 = rinv[j + 1];
                a0 = fma(ln <= j ? v0 : 0.0, d0, a0);
                a1 = fma(ln <= j + 1 ? v1 : 0.0, d1, a1);
            }
            if (j < q) {
                const double v0 = L.R[ln <= j ? lrow(j) + ln : 0];
                a0 = fma(ln <= j ? v0 : 0.0, rinv[j], a0);
            }
            r = (ln < q) ? a0 + a1 : 0.0;
            const double rmax = wave_max(fabs(r));
            if (ln < q && r > kRTol * rmax) { t1 = fdiv(u, r); kslot = ln; }
            wave_argmin(t1, kslot);
        }
        if (!MPCQP_REG_RINV && q > 0) {
            // the chain from one step to the next is v_readlane -> mul -> FMA in registers:
            // 1/R(j,j) comes out of a register (lane j), R's columns are loaded four at a time
            // one block ahead; the FMA runs on every lane (a lane at or past its slot only
            // changes a value already read)
            double val = dj;
            const double ril = rinv[ln < NF ? ln : 0];
            auto colR = [&](int jj) { return (jj >= 0 && ln < jj) ? L.R[roff(jj) + ln] : 0.0; };
            int j = q - 1;
            double cc[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) cc[t] = colR(j - t);
            for (; j >= 0; j -= 4) {
                double nc[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) nc[t] = colR(j - 4 - t);
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int jj = j - t;
                    if (jj >= 0) {
                        const double rj = readlane(val, jj) * readlane(ril, jj);
                        if (ln == jj) r = rj;
                        val -= cc[t] * rj;
                    }
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) cc[t] = nc[t];
            }
            const double rmax = wave_max(ln < q ? fabs(r) : 0.0);
            if (ln < q && r > kRTol * rmax) { t1 = fdiv(u, r); kslot = ln; }
            wave_argmin(t1, kslot);
        }
        const bool dep = !(zn > kDepTol * dd);
        const double t2 = dep ? INFINITY : fdiv(-sp, zn);
        const double t = t1 < t2 ? t1 : t2;
        if (isinf(t)) { status = ST_INFEASIBLE; break; }
        MPCQP_SUB(tsub, 2);
        const double uq = readlane(u, q);
        if (!isinf(t2)) {
            if (ln < nf) { x += t * z; L.xs[ln] = x; }
            fval += t * zn * (0.5 * t + uq);
        }
        if (ln < q) u -= t * r;
        if (ln == q) u += t;
        const bool add = !isinf(t2) && t2 <= t1;
        double beta = 0.0;
        if (add) {
            // ---- add p: J2 <- J2 (I - beta v v'), the Householder reflection with
            //      v = d2 - |d2| e_q (v_q by Parlett's cancellation-free form) that maps d2 to
            //      |d2| e_q.  Same new column J2 d2 / |d2| and R column as the Givens chain;
            //      the trailing columns are another orthonormal basis of the same subspace,
            //      which every later GI quantity (z = J2 J2' n, d1 = J1' n, r) is invariant
            //      to.  colb holds d2 (zeros below q); v differs from it only at q.
            const double dq = readlane(dj, q);
            double rqq = dq, vq = 0.0;
            if (zq > 0.0) {  // otherwise d2 = d_q e_q: no reflection, r_qq = d_q
                const double nrm = sqrt(zn);
                rqq = nrm;
                vq = dq > 0.0 ? fdiv(-zq, dq + nrm) : dq - nrm;
                beta = fdiv(2.0, vq * vq + zq);
            }
            wave_sync();
            if (ln == q) colb[q] = vq;
            if (MPCQP_REG_RINV) {
                // R^-1 of [[R, d1], [0, r_qq]]: column q = (-R^-1 d1 / r_qq, 1 / r_qq), and
                // R^-1 d1 is this pass's r
                const double irq = fdiv(1.0, rqq);
                if (ln < q) L.R[lrow(q) + ln] = -r * irq;
                if (ln == q) { L.R[lrow(q) + q] = irq; act = p; }
            } else {
                if (ln < q) L.R[roff(q) + ln] = dj;
                if (ln == q) { L.R[roff(q) + q] = rqq; rinv[q] = 1.0 / rqq; act = p; }
            }
            if (ln == 0) L.st[p] = 2;
            ++q;
            fresh = true;
        } else {
            // ---- drop slot kslot: shift u/act and the R columns left, then restore R to
            //      triangular with Givens rotations whose (c, s) go to LDS for J
            const int k = kslot;
            const int dropped = readlane(act, k);
            if (ln == 0) L.st[dropped] = 1;
            {
                const int src = ln + 1 < kWave ? ln + 1 : ln;
                const double un = __shfl(u, src, kWave);
                const int an = __shfl(act, src, kWave);
                if (ln >= k && ln < q) { u = un; act = an; }
            }
            if (MPCQP_REG_RINV) {
                // R^-1 G' with the rotations that zero row k of R^-1 left of column q-1 (the G
                // that restores R without column k), row k deleted, the last column dropped.
                // Rotation j (lane j): hypotenuse sqrt(R^-1(k,k)^2 + sum_{i <= j} R^-1(k,i+1)^2)
                // from one DPP prefix sum; c = R^-1(k,j+1) / h_j, s = -h_{j-1} / h_j.
                const int qn = q - 1;
                const double ra0 = L.R[lrow(k) + k];
                const bool on = ln >= k && ln < qn;
                const double rb = on ? L.R[lrow(ln + 1) + k] : 0.0;
                double pf = wave_prefix_sum(rb * rb);
                pin(pf);  // the DPP moves with every lane active (a disabled source lane reads 0)
                const double H = sqrt(ra0 * ra0 + pf);
                double hp = wave_prev(H);
                pin(hp);
                if (ln < NF) {
                    const double ih = fdiv(1.0, H);
                    rot[2 * ln] = on ? rb * ih : 1.0;
                    rot[2 * ln + 1] = on ? -(ln == k ? ra0 : hp) * ih : 0.0;
                }
                wave_sync();
                // lane i carries row i: column j's rotated value is final (stored at row i, or
                // i - 1 past the deleted row k); the carry is column j + 1 as rotated so far
                double cr = (ln <= k) ? L.R[lrow(k) + ln] : 0.0;
                int j = k;
                for (; j + 4 <= qn; j += 4) {
                    double c4[4], s4[4], y4[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        c4[t] = rot[2 * (j + t)];
                        s4[t] = rot[2 * (j + t) + 1];
                        const double y = L.R[ln <= j + t + 1 ? lrow(j + t + 1) + ln : 0];
                        y4[t] = (ln <= j + t + 1) ? y : 0.0;
                    }
                    step_fence();  // every load of the block before its stores (other lanes')
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const double o = c4[t] * cr + s4[t] * y4[t];
                        cr = -s4[t] * cr + c4[t] * y4[t];
                        if (ln <= j + t + 1 && ln != k) L.R[lrow(j + t) + ln - (ln > k ? 1 : 0)] = o;
                    }
                    step_fence();
                }
                for (; j < qn; ++j) {
                    const double c = rot[2 * j], s_ = rot[2 * j + 1];
                    const double y0 = L.R[ln <= j + 1 ? lrow(j + 1) + ln : 0];
                    const double y = (ln <= j + 1) ? y0 : 0.0;
                    step_fence();
                    const double o = c * cr + s_ * y;
                    cr = -s_ * cr + c * y;
                    if (ln <= j + 1 && ln != k) L.R[lrow(j) + ln - (ln > k ? 1 : 0)] = o;
                    step_fence();
                }
                --q;
            }
            // R's columns k+1.. move one left: lane l moves its own entries (rows <= j + 1 of
            //      column j + 1), so no lane waits on another -- four columns per round trip
            for (int j = k; !MPCQP_REG_RINV && j < q - 1; j += 4) {
                double v[4];
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    v[t] = (j + t < q - 1 && ln <= j + t + 1) ? L.R[roff(j + t + 1) + ln] : 0.0;
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (j + t < q - 1 && ln <= j + t + 1) L.R[roff(j + t) + ln] = v[t];
            }
            if (!MPCQP_REG_RINV) {
                --q;
                if (ln < NF) { rot[2 * ln] = 1.0; rot[2 * ln + 1] = 0.0; }
            }
            wave_sync();
            // Givens back to triangular.  Rotation j mixes rows j and j+1 of the columns
            // l > j (lane l - j - 1).  Row j+1 is untouched until then (prefetchable from LDS);
            // row j's entries are the previous rotation's second outputs, one lane up (DPP
            // wave_shl), and the next pivot R(j+1, j+1) is lane 0's second output: the chain
            // from one rotation to the next stays in registers.  Same arithmetic as the
            // LDS round-trip form.
            if (!MPCQP_REG_RINV && k < q) {
                double carry = 0.0;  // row j of columns j+1+ln, after the previous rotation
                {
                    const int l = k + 1 + ln;
                    carry = (l < q) ? L.R[roff(l) + k] : 0.0;
                }
                double a = L.R[roff(k) + k];
                for (int j = k; j < q; ++j) {
                    const int l = j + 1 + ln;
                    const double bb = L.R[roff(j) + j + 1];
                    const double r1 = (l < q) ? L.R[roff(l) + j + 1] : 0.0;
                    const double r0 = carry;
                    double n1 = r1;
                    if (bb != 0.0) {
                        const double hh = sqrt(a * a + bb * bb);
                        const double ih = fdiv(1.0, hh);
                        const double c = a * ih, s_ = bb * ih;
                        n1 = -s_ * r0 + c * r1;
                        if (l < q) {
                            L.R[roff(l) + j] = c * r0 + s_ * r1;
                            L.R[roff(l) + j + 1] = n1;
                        }
                        if (ln == 0) {
                            L.R[roff(j) + j] = hh;
                            L.R[roff(j) + j + 1] = 0.0;
                            rinv[j] = ih;
                            rot[2 * j] = c;
                            rot[2 * j + 1] = s_;
                        }
                    } else {
                        if (ln == 0) rinv[j] = 1.0 / a;  // the shifted column's diagonal as it is
                    }
                    a = readlane(n1, 0);    // R(j+1, j+1) after this rotation
                    carry = wave_next(n1);  // row j+1 of columns j+2+ln
                }
            }
        }
        wave_sync();
        // ---- the pass's update of J: add -> the reflection (J_j -= beta (J . v) v_j),
        //      drop -> rotations (j, j+1) for j = 0 .. NF-2, identity where (c, s) = (1, 0)
        //      Two independent uniform steps, not an if / else: the two arms' definitions of
        //      Jr would meet in a phi that the register allocator resolves with a second copy
        //      of the 2 NF registers (and spills)
        if (__builtin_amdgcn_readfirstlane((int)(add && beta != 0.0))) {
            double w4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                w4[j & 3] += Jr[j] * colb[j];
                if ((j & 7) == 7) step_fence();
            }
            const double f = beta * ((w4[0] + w4[1]) + (w4[2] + w4[3]));
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                Jr[j] -= f * colb[j];
                if ((j & 7) == 7) step_fence();
            }
        }
        if (__builtin_amdgcn_readfirstlane((int)!add)) {
#pragma unroll
            for (int j = 0; j < NF - 1; ++j) {
                const double c = rot[2 * j], s_ = rot[2 * j + 1];
                const double x0 = Jr[j], x1 = Jr[j + 1];
                Jr[j] = c * x0 + s_ * x1;
                Jr[j + 1] = -s_ * x0 + c * x1;
                if ((j & 7) == 7) step_fence();
            }
        }
        wave_sync();
    }
    MPCQP_SUB(tsub, 3);
    MPCQP_SUB_FLUSH(C.stamps, tsub);
    MPCQP_STAMP(C.stamps, 8, tst); MPCQP_CUT(C.cut, 7);
    if (warm) {
        // this tick's active set, in the global numbering, for the next tick
        unsigned long long *wl = reinterpret_cast<unsigned long long *>(rowbuf);
        wave_sync();
        if (ln < warm->n) wl[ln] = 0ull;
        wave_sync();
        if (status == ST_OK && ln < nf) {
            const int v = L.fid[ln], k = v / P.nu, c = v % P.nu;
            if (L.st[ln] == 2) atomicOr(&wl[v >> 6], 1ull << (v & 63));
            if (L.st[ln + nf] == 2) atomicOr(&wl[(P.nV + v) >> 6], 1ull << ((P.nV + v) & 63));
            if (fbase >= 0) {
                const int fb = 2 * P.nV + 4 * (k * P.nfeet + c / 3);
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (L.st[fbase + t] == 2) atomicOr(&wl[(fb + t) >> 6], 1ull << ((fb + t) & 63));
            }
        }
        wave_sync();
        if (ln < warm->n) warm->words[ln] = wl[ln];
    }
    C.status = status;
    C.x = x;
    C.u = u;
    C.fval = fval;
    C.act = act;
    C.q = q;
    C.iters = iters;
}

}  // namespace mpcqp
