// gi_wg.hpp -- Goldfarb-Idnani solve of ONE QP by a 4-wave workgroup, for up to NF <= 128
// free variables: the instances the one-wave kernels cannot hold (double support / standing
// at N = 10 and 20, up to 6N = 120 free forces) and the whole-body configuration E
// (nV = 96).  Replaces qpOASES in QPSolver::solveQP (src/QPSolver.cpp:83-106), which the
// reference calls on the dense nV = NU*N problem whatever the bound pattern (:87-96).
//
// Same algorithm, constraint order and tolerances as gi_run_reg (gi_reg.hpp), gi_run
// (gi_solver.hpp) and the CPU oracle; only the distribution over threads differs:
//   * 256 threads = rows 0..127 x two column halves.  Thread (r, h) (h = tid / 128, waves 0-1
//     are half 0, waves 2-3 half 1) hands in row r of H_FF (columns 2j + h <= r) and holds
//     columns [h NF/2, (h+1) NF/2) of row r of J = L^-T Q.  NF/2 <= 64 doubles per thread.
//   * Cholesky and J = L^-T: the blocked FP64-MFMA factorisation and triangular inverse of
//     chol_mfma.hpp on 16 x 16 tiles in LDS (three barriers per 16 columns), then every thread
//     reads its J row part (J(r, c) = X(c, r), X = L^-1) and t = L^-1 g = X g.
//   * Dual loop: the most violated constraint is found by the rows of half 0 (bounds of their
//     own variable and, for a foot's vertical force, that foot-step's friction rows); the
//     constraint's normal n is published as J rows (d = J' n); z = J2 d2 is a per-half dot
//     product summed over the two halves through LDS; r = R^-1 d1 and the slot bookkeeping
//     (u, active ids, R packed in LDS) run on wave 0 (two slots per lane); the add step is
//     the Householder reflection of gi_reg.hpp, the drop step Givens rotations whose chain
//     crosses the half boundary once.
//   * Sums across threads are combined in a fixed order (half 0 + half 1, wave 0 + wave 1),
//     so both halves hold bit-identical copies of x, z and every scalar.
#pragma once
#include "chol_mfma.hpp"
#include "gi_reg.hpp"

namespace mpcqp {

// rows per column half: one wave for NF <= 64, two waves for NF <= 128
template <int NF>
struct WgShape {
    static constexpr int RW = NF <= 64 ? 64 : 128;
    static constexpr int THREADS = 2 * RW;  // two or four waves
    static constexpr int NWH = RW / 64;      // waves per half
};

// column k of the parked L, rows k..NF-1 (column-major packed, no padding)
template <int NF>
__device__ __forceinline__ int wg_lcol(int k) { return k * NF - (k * (k - 1)) / 2; }

template <int NF>
struct WgLayout {
    static_assert(NF % 2 == 0 && NF >= 2 && NF <= 128, "two column halves of <= 64");
    static constexpr int NH = NF / 2, RW = WgShape<NF>::RW;
    static constexpr int NRP = NF * (NF + 3) / 2;    // packed L, then packed R (roff)
    static constexpr int CBW = RW + 2;               // column broadcast: RW rows + g slot
    static constexpr int oL = 0;
    static constexpr int oCol = (NRP + 1) & ~1;      // [2][CBW]; then the rotations (2 NF)
    static constexpr int oD = oCol + 2 * CBW;        // d = J' n (published rows)
    static constexpr int oDq = oD + RW;              // d masked to c >= q, then the reflector v
    static constexpr int oD2 = oDq + RW;             // second friction row; drop carry
    static constexpr int oPart = oD2 + RW;           // [2][RW] per-half partial sums
    static constexpr int oT = oPart + 2 * RW;        // t = L^-1 g; drop carry
    static constexpr int oRinv = oT + RW;            // 1/L(k,k), then 1/R(j,j)
    static constexpr int oUs = oRinv + RW;           // slot multipliers u
    static constexpr int oRed = oUs + RW;            // reduction slots
    static constexpr int oAct = oRed + 32;           // slot constraint ids (int)
    static constexpr int oRp = oAct + RW / 2;        // [waves][RW] partial products R^-1 d
    static constexpr int doubles = oRp + 2 * RW * (RW / 64);
    static_assert(2 * CBW >= 2 * NF, "rotations fit the column buffers");
    // the blocked factorisation (chol_mfma.hpp) overlays the whole workspace before the loop
    static constexpr int work = doubles > TileFact<NF>::doubles ? doubles : TileFact<NF>::doubles;
};

struct WgIds {
    int tid, h, r, wv, ln;
};
template <int RW>
__device__ __forceinline__ WgIds wg_ids() {
    WgIds t;
    t.tid = (int)threadIdx.x;
    // opaque per call: the index arithmetic (and every LDS address derived from it) is
    // recomputed per instance instead of being hoisted out of a persistent kernel's instance
    // loop and held in registers across the whole solve
    asm volatile("" : "+v"(t.tid));
    // the half and the wave index are wave-uniform: in SGPRs, so the per-column LDS addresses
    // and masks of the unrolled loops are scalar (not a VGPR per column held across the loop)
    t.h = __builtin_amdgcn_readfirstlane(t.tid / RW);
    t.r = t.tid & (RW - 1);
    t.wv = __builtin_amdgcn_readfirstlane(t.tid >> 6);
    t.ln = lane();
    return t;
}

// lexicographic (value, id) minimum of the NWH half-0 wave results in red[o..o+2 NWH)
template <int NWH>
__device__ __forceinline__ void wg_pick(const double *red, int o, double &v, int &id) {
    v = red[o];
    id = (int)red[o + 1];
    if constexpr (NWH == 2) {
        const double v1 = red[o + 2];
        const int i1 = (int)red[o + 3];
        const bool take1 = v1 < v || (v1 == v && i1 < id);
        v = take1 ? v1 : v;
        id = take1 ? i1 : id;
    }
}

// hr: thread (r, h) holds H_FF(r, 2 j + h) for c <= r (columns interleaved over the halves;
// rows / columns >= nf padded with the identity, so every step runs unpredicated; entries
// above the diagonal are never read).
// g: g_r on both halves of row r (0 beyond nf).  W: WgLayout<NF>::doubles of LDS.
// C.L must provide xs (128), cb, st, fid, pos, xfull.  Fills C.{status, x, fval, q, iters};
// every thread returns x_r of its row.
// The dual loop keeps R^-1 (column-major packed, (i, j) at lrow(j) + i) instead of R: r = R^-1 d
// is a product over the slots instead of a back substitution whose every step waits on the
// previous one (see mpc_pair.hpp for the add / drop updates); 0 keeps R (A/B builds)
#ifndef MPCQP_WG_RINV
#define MPCQP_WG_RINV 1
#endif
// 1: every wave takes every (2 NWH)-th column of the R^-1 product, the partials meet in LDS
// behind the barrier that follows anyway and every wave finishes r, max |r| and t1 itself
#ifndef MPCQP_WG_RSPLIT
#define MPCQP_WG_RSPLIT 1
#endif
// 1: the J products skip 8-column blocks the step leaves untouched -- columns c < q of d2 and
// of the reflector are zero, and a drop rotates only columns k .. q
#ifndef MPCQP_WG_SKIP
#define MPCQP_WG_SKIP 1
#endif
// 1: a drop's rotations all at once (rotation j's hypotenuse is sqrt(R^-1(k,k)^2 + the prefix
// sum of R^-1(k, k+1 .. j+1)^2), then each lane carries its row through the columns with the
// column loads issued four at a time; 0: one rotation after the other, an LDS round trip and a
// sqrt / divide on the chain per column
// 1: the selection's bound states and b in registers at NF > 64 (below)
#ifndef MPCQP_WG_STREG
#define MPCQP_WG_STREG 1
#endif
#ifndef MPCQP_WG_PDROP
#define MPCQP_WG_PDROP 1
#endif

// ---- crash start of the workgroup solver (box constraints only; the paired kernel's
//      speculative primal-dual active-set start, mpc_pair.hpp / oracle box_crash, at the
//      workgroup's scale).  Thread (r, 0) owns variable r's bounds and working-set state; the
//      rows of J in A are published to the dead workspace, M = J_A J_A' is computed entry by
//      entry over the whole workgroup (its lower triangle, mirrored), the k x k system by
//      Gauss-Jordan over the workgroup (one barrier per pivot), y = J_A' w by column and
//      dx = J y as each row's two half products.  Returns true when the working set settled (x,
//      fval, iterations set, L.xs updated); false: nothing changed but the iteration count.
#ifndef MPCQP_WG_CRASH_K
#define MPCQP_WG_CRASH_K 32
#endif
#ifndef MPCQP_WG_CRASH_P
#define MPCQP_WG_CRASH_P 8
#endif
constexpr int kWgCrashK = MPCQP_WG_CRASH_K, kWgCrashP = MPCQP_WG_CRASH_P;
#ifndef MPCQP_WG_SRBM_CRASH
#define MPCQP_WG_SRBM_CRASH 0  // the SRBM overflow kernels (mpc_wg.hpp) without the crash
#endif

template <int NF>
struct WgCrashLayout {
    static constexpr int KC = kWgCrashK, RW = WgShape<NF>::RW;
    static constexpr int LDW = NF + 1;  // odd row stride: the Gram's per-thread row reads
    static constexpr int LDM = KC + 2;  // column KC: the right-hand side
    static constexpr int oWr = 0, oM = oWr + KC * LDW, oW = oM + KC * LDM, oY = oW + KC;
    static constexpr int oP = oY + NF, oR0 = oP + 2 * RW, oRed = oR0 + KC;
    static constexpr int oRho = oRed + 16;  // int [RW]
    static constexpr int doubles = oRho + RW / 2 + 1;
};

// rank of a flagged owner thread (h = 0: rows r = tid < RW, waves 0 .. NWH-1) among the flagged
// ones in row order, and their count; one barrier
template <int NWH>
__device__ __forceinline__ int wg_rank(bool f, int *cnt, int wv, int ln, int &total) {
    const uint64_t b = __ballot(f);
    if (ln == 0) cnt[wv] = __popcll(b);
    __syncthreads();
    int base = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < NWH; ++w) {
        base += (w < wv) ? cnt[w] : 0;
        total += cnt[w];
    }
    return base + __popcll(b & ((1ull << ln) - 1ull));
}

template <int NF>
__device__ __forceinline__ bool wg_crash(GiCtx &C, const double (&Jr)[NF / 2], double &x,
                                         double &fval, int &iters, double *W) {
    using CL = WgCrashLayout<NF>;
    static_assert(CL::doubles <= WgLayout<NF>::work, "the crash fits the solver's workspace");
    // after a give-up the dual loop reuses the buffers from oCol on (column broadcast, reflector,
    // R^-1 slots, multipliers, reductions, active ids) without re-deriving them: the crash's
    // scratch must stay in the packed L / R region below (NF = 96 fits, the NF = 64
    // SRBM overflow kernel does not, so MPCQP_WG_SRBM_CRASH=1 builds refuse to compile)
    static_assert(CL::doubles <= WgLayout<NF>::oCol,
                  "the crash's scratch overlaps the dual loop's buffers (NF = 64: keep "
                  "MPCQP_WG_SRBM_CRASH=0)");
    constexpr int KC = CL::KC, NH = NF / 2, RW = WgShape<NF>::RW, NWH = WgShape<NF>::NWH;
    constexpr int NT = 2 * RW, LDW = CL::LDW, LDM = CL::LDM;
    GiLds &L = C.L;
    const WgIds T = wg_ids<RW>();
    const int h = T.h, r = T.r, wv = T.wv, ln = T.ln, tid = T.tid, nf = C.nf, PC = C.crash_p;
    double *Wr = W + CL::oWr, *M = W + CL::oM, *Wv = W + CL::oW, *Yv = W + CL::oY,
           *Pp = W + CL::oP, *R0 = W + CL::oR0, *red = W + CL::oRed;
    int *rho_of = reinterpret_cast<int *>(W + CL::oRho);
    int *cnt = reinterpret_cast<int *>(red + 8);
    const bool owner = h == 0 && r < nf;
    double b0 = 0.0, b1 = 0.0;
    int s0 = 0, s1 = 0;
    if (owner) {
        s0 = L.st[r];
        s1 = L.st[r + nf];
        b0 = L.cb[r];
        b1 = L.cb[r + nf];
    }
    const double x0 = x, f0 = fval;
    double xc = x0, lam = 0.0, fc = f0;
    int side = 0, cit = 0, solves = 0;
    bool settled = false;
    for (;;) {
        int nw = side;
        if (owner) {
            if (side == 0) {
                if (s0 == 1 && xc - b0 < -kFeasTol * (1.0 + fabs(b0))) nw = 1;
                else if (s1 == 1 && -xc - b1 < -kFeasTol * (1.0 + fabs(b1))) nw = -1;
            } else if (lam < 0.0) {
                nw = 0;
            }
        }
        if (!__syncthreads_or(owner && nw != side)) { settled = true; break; }
        if (cit >= PC) break;  // give up
        {   // at most KC bounds: those already in A, then the lowest variable ids
            int tot = 0, kept = 0;
            (void)wg_rank<NWH>(owner && nw != 0, cnt, wv, ln, tot);
            __syncthreads();
            if (tot > KC) {
                (void)wg_rank<NWH>(owner && nw != 0 && side != 0, cnt, wv, ln, kept);
                __syncthreads();
                int nadd = 0;
                const int rk = wg_rank<NWH>(owner && nw != 0 && side == 0, cnt, wv, ln, nadd);
                __syncthreads();
                if (owner && nw != 0 && side == 0 && rk >= KC - kept) nw = 0;
            }
        }
        if (owner) side = nw;
        ++cit;
        const bool inA = owner && side != 0;
        int k = 0;
        const int rho = wg_rank<NWH>(inA, cnt, wv, ln, k);
        if (k == 0) {  // (workgroup-uniform) the unconstrained minimum again
            xc = x0;
            lam = 0.0;
            fc = f0;
            __syncthreads();
            continue;
        }
        ++solves;
        const double bv = side > 0 ? b0 : -b1;
        if (h == 0) rho_of[r] = inA ? rho : -1;
        if (inA) {
            R0[rho] = x0 - bv;
            M[rho * LDM + KC] = x0 - bv;
        }
        __syncthreads();
        {   // publish the J rows of A (both halves of each row)
            const int rr = (r < nf) ? rho_of[r] : -1;
            if (rr >= 0) {
#pragma unroll
                for (int j = 0; j < NH; ++j) Wr[rr * LDW + h * NH + j] = Jr[j];
            }
        }
        __syncthreads();
        // M = J_A J_A': lower-triangle entries over the workgroup, mirrored
        const int ne = k * (k + 1) / 2;
        for (int e = tid; e < ne; e += NT) {
            int i = (int)((__builtin_sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
            i += ((i + 1) * (i + 2) / 2 <= e) ? 1 : 0;
            i -= (i * (i + 1) / 2 > e) ? 1 : 0;
            const int m = e - i * (i + 1) / 2;
            const double *wi = Wr + i * LDW, *wm = Wr + m * LDW;
            double s4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int c = 0; c < NF; ++c) {
                s4[c & 3] += wi[c] * wm[c];
                if ((c & 15) == 15) step_fence();
            }
            const double sv = (s4[0] + s4[1]) + (s4[2] + s4[3]);
            M[i * LDM + m] = sv;
            M[m * LDM + i] = sv;
        }
        __syncthreads();
        // Gauss-Jordan without pivoting (M positive definite), one barrier per pivot: step j
        // writes M(i, m) for i != j, m > j (and the right-hand side) and reads only column j and
        // row j, which it does not write
        bool bad = false;
        for (int j = 0; j < k; ++j) {
            const double d = M[j * LDM + j];
            bad |= !(d > 0.0);
            const double inv = 1.0 / d;
            const int ncol = k - j;  // columns j+1 .. k-1, then the right-hand side
            for (int e = tid; e < (k - 1) * ncol; e += NT) {
                const int ii = e / ncol, mm = e - ii * ncol;
                const int i = ii + (ii >= j ? 1 : 0), m = (mm < ncol - 1) ? j + 1 + mm : KC;
                const double l = M[i * LDM + j] * inv;
                M[i * LDM + m] -= l * M[j * LDM + m];
            }
            __syncthreads();
        }
        if (bad) break;  // (workgroup-uniform: every thread read the same pivots) give up
        if (tid < k) Wv[tid] = M[tid * LDM + KC] / M[tid * LDM + tid];
        __syncthreads();
        // y = J_A' w by column; f = f0 + w'(x0_A - b_A) / 2
        if (tid < NF) {
            double y = 0.0;
            for (int m = 0; m < k; ++m) y += Wr[m * LDW + tid] * Wv[m];
            Yv[tid] = y;
        }
        if (wv == NWH * 2 - 1) {
            double s = 0.0;
            for (int m = ln; m < k; m += 64) s += Wv[m] * R0[m];
            s = wave_sum(s);
            if (ln == 0) red[0] = s;
        }
        __syncthreads();
        {   // dx = J y: each row's two half products
            double s4[4] = {0.0, 0.0, 0.0, 0.0};
            const double *yv = Yv + h * NH;
#pragma unroll
            for (int j = 0; j < NH; ++j) {
                s4[j & 3] += Jr[j] * yv[j];
                if ((j & 7) == 7) step_fence();
            }
            Pp[h * RW + r] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
        }
        __syncthreads();
        if (owner) {
            xc = inA ? bv : x0 - (Pp[r] + Pp[RW + r]);
            lam = inA ? -(double)side * Wv[rho] : 0.0;
        }
        fc = f0 + 0.5 * red[0];
        __syncthreads();
    }
    iters = solves;
    if (!settled) return false;
    if (owner) L.xs[r] = xc;
    __syncthreads();
    x = (r < nf) ? L.xs[r] : 0.0;
    fval = fc;
    return true;
}

template <int NF, bool CRASH = false>
__device__ __forceinline__ void gi_run_wg(GiCtx &C, double (&hr)[NF / 2], double g, double *W) {
    using Lay = WgLayout<NF>;
    constexpr int NH = Lay::NH, RW = Lay::RW, NWH = WgShape<NF>::NWH;
    constexpr bool TWO = RW > 64;  // wave 0 keeps two slots per lane (ln, ln + 64)
    GiLds &L = C.L;
    const SolveProblem &P = *C.P;
    const WgIds T = wg_ids<RW>();
    const int h = T.h, r = T.r, wv = T.wv, ln = T.ln, tid = T.tid;
    const int nf = C.nf, mt = C.mt;
    int status = C.status;
    double *Lc = W + Lay::oL, *colb = W + Lay::oCol, *dB = W + Lay::oD, *dqB = W + Lay::oDq,
           *d2B = W + Lay::oD2, *part = W + Lay::oPart, *tB = W + Lay::oT,
           *rinv = W + Lay::oRinv, *us = W + Lay::oUs, *red = W + Lay::oRed;
    double *rot = colb;
    int *acts = reinterpret_cast<int *>(W + Lay::oAct);
    const bool live = r < NF;
    double x = 0.0, fval = 0.0;
    int iters = 0, q = 0;
    double Jr[NH];
    MPCQP_STAMP_INIT(tst);

    // ---- H_FF = L L' and X = L^-1 on the matrix cores (chol_mfma.hpp), tiles in LDS over the
    //      workspace; then J(r, c) = X(c, r) (c >= r) and t = X g per row
    double gv = (live && r < nf) ? g : 0.0;
    if (status == ST_OK && nf > 0) {
        using TF = TileFact<NF>;
        constexpr int TS = TF::TS;
        double *F = W;
        if (live) {
#pragma unroll
            for (int j = 0; j < NH; ++j) {
                const int c = 2 * j + h;  // the callers' interleaved row layout
                if (c <= r) {
                    const int ti = r >> 4, tj = c >> 4, ra = r & 15, cb_ = c & 15;
                    double *tl = F + TF::oTiles + TS * tix(ti, tj);
                    tl[64 * (cb_ >> 2) + 16 * (cb_ & 3) + ra] = hr[j];      // stored S = H_ij'
                    if (ti == tj && c < r) tl[64 * (ra >> 2) + 16 * (ra & 3) + cb_] = hr[j];
                }
            }
            if (h == 0) F[TF::oG + r] = gv;
        }
        if (tid == 0) F[TF::oFlag] = 0.0;
        __syncthreads();
        if (chol_inverse_mfma<NF, 2 * NWH>(F, wv)) status = ST_NOT_PD;
        MPCQP_STAMP(C.stamps, 5, tst);
        MPCQP_CUT(C.cut, 4);
#pragma unroll
        for (int j = 0; j < NH; ++j) {
            const int c = h * NH + j;
            Jr[j] = (live && c >= r) ? F[TF::xoff(c, r)] : 0.0;
            if ((j & 7) == 7) step_fence();
        }
        double tt = 0.0;
        if (live) {
            // t_r = sum_c X(r, c) g_c, block by block; lane r starts block cb at column
            // (r & 15): row reads of a slice-order tile stride 16 doubles across the lanes (8-way
            // bank conflicts in column order), rotated they hit 16 distinct bank pairs.  The
            // diagonal tile's entries above the diagonal are exact zeros.
            const double *xr = F + TF::oTiles + TS * tix(r >> 4, 0) + 16 * (r & 15);
            for (int cb = 0; cb <= (r >> 4); ++cb) {
                const double *gb = F + TF::oG + 16 * cb;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int cc = (k + r) & 15;
                    tt += xr[TS * cb + cc] * gb[cc];
                }
            }
        }
        gv = (live && r < nf) ? tt : 0.0;
        __syncthreads();  // the factorisation's tiles are dead: the loop's buffers overlay them
        if (h == 0) tB[r] = (r < nf) ? gv : 0.0;
        __syncthreads();
        MPCQP_STAMP(C.stamps, 6, tst);
        MPCQP_CUT(C.cut, 5);
        // ---- unconstrained minimum x = -J t, objective -|t|^2 / 2
        double s4[4] = {0.0, 0.0, 0.0, 0.0};
        const double *tb = tB + h * NH;
#pragma unroll
        for (int j = 0; j < NH; ++j) {
            s4[j & 3] += Jr[j] * tb[j];
            if ((j & 7) == 7) step_fence();
        }
        part[h * RW + r] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
        if (h == 0) {
            const double tt = wave_sum((r < nf) ? gv * gv : 0.0);
            if (ln == 0) red[wv] = tt;
        }
        __syncthreads();
        x = (r < nf) ? -(part[r] + part[RW + r]) : 0.0;
        fval = -0.5 * (NWH == 2 ? red[0] + red[1] : red[0]);
        if (h == 0) L.xs[r] = x;
        __syncthreads();
    }
    MPCQP_STAMP(C.stamps, 7, tst);
    MPCQP_CUT(C.cut, 6);

    // ---- dual active-set loop: one pass = one add or drop step
    const int max_iter = P.max_iter > 0 ? P.max_iter : 10 * (mt + nf + 1);
    bool done = (status != ST_OK) || nf == 0;
    if constexpr (CRASH) {
        // (workgroup-uniform condition: status, nf and the problem kind are the instance's)
        if (!done && C.nfric == 0 && C.crash_p > 0) done = wg_crash<NF>(C, Jr, x, fval, iters, W);
    }
    MPCQP_CUT(C.cut, 8);
    bool fresh = true;
    int p = 0;
    int fbase = -1;  // friction rows of the foot-step whose vertical force is variable r
    if (C.nfric > 0 && status == ST_OK && h == 0 && r < nf) {
        const int v = L.fid[r], k = v / P.nu, c = v % P.nu, sft = c / 3;
        if (c % 3 == 2 && ((P.contact >> (2 * k + sft)) & 1ull)) fbase = 2 * nf + 4 * (k * P.nfeet + sft);
    }
    // row r's two bound states and b in registers (half 0): an add sets them from the uniform
    // p, a drop's row re-reads them after the pass's last barrier; no LDS reads per selection.
    // Only for NF > 64 (at NF = 64 the four registers cost 8 more spilled VGPRs)
    constexpr bool kStReg = TWO && MPCQP_WG_STREG;
    int s0r = 0, s1r = 0;
    double b0r = 0.0, b1r = 0.0;
    if (kStReg && h == 0 && r < nf) {
        s0r = L.st[r];
        s1r = L.st[r + nf];
        b0r = L.cb[r];
        b1r = L.cb[r + nf];
    }
    MPCQP_SUB_INIT(tsub);
    while (!done) {
        MPCQP_SUB(tsub, 3);
        if (fresh) {
            // ---- step 1: most violated inactive constraint (lowest id on ties)
            double best = INFINITY;
            int bid = 0x7fffffff;
            const bool qsel = C.nfric > 0 && P.contact != 0ull;  // (gi_sel_key)
            if (h == 0 && r < nf) {
                const int s0 = kStReg ? s0r : L.st[r], s1 = kStReg ? s1r : L.st[r + nf];
                const double b0 = kStReg ? b0r : L.cb[r], b1 = kStReg ? b1r : L.cb[r + nf];
                if (s0 == 1) {
                    const double sl_ = x - b0;
                    if (sl_ < -kFeasTol * (1.0 + fabs(b0))) { best = gi_sel_key(sl_, qsel); bid = r; }
                }
                if (s1 == 1) {
                    const double sl_ = -x - b1;
                    const double kv = gi_sel_key(sl_, qsel);
                    if (sl_ < -kFeasTol * (1.0 + fabs(b1)) && kv < best) { best = kv; bid = r + nf; }
                }
                if (fbase >= 0) {
                    const double xm1 = L.xs[r - 1], xm2 = L.xs[r - 2];  // fy, fx of the foot
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        if (L.st[fbase + t] != 1) continue;
                        const double sg = (t & 1) ? 1.0 : -1.0;
                        double s = 0.0;
                        s += P.mu * x;
                        s += sg * ((t >> 1) ? xm1 : xm2);
                        const double kv = gi_sel_key(s, qsel);
                        if (s < -kFeasTol && kv < best) { best = kv; bid = fbase + t; }
                    }
                }
            }
            wave_argmin(best, bid);
            if (h == 0 && ln == 0) { red[4 + 2 * wv] = best; red[5 + 2 * wv] = (double)bid; }
            __syncthreads();
            wg_pick<NWH>(red, 4, best, bid);
            if (bid == 0x7fffffff) break;  // optimal
            p = bid;
            if (tid == 0) us[q] = 0.0;
            fresh = false;
        }
        MPCQP_SUB(tsub, 0);
        // ---- d = J' n_p (published J rows) and the slack of p
        int a0, a1 = -1;
        double c0, c1 = 0.0, bp;
        if (p < 2 * nf) {
            a0 = p < nf ? p : p - nf;
            c0 = p < nf ? 1.0 : -1.0;
            bp = L.cb[p];
        } else {
            const int rr = p - 2 * nf, ks = rr >> 2, t = rr & 3;
            const int k = ks / P.nfeet, sft = ks % P.nfeet;
            const int pz = L.pos[k * P.nu + 3 * sft + 2], pt = L.pos[k * P.nu + 3 * sft + (t >> 1)];
            const double sg = (t & 1) ? 1.0 : -1.0;
            a0 = pz >= 0 ? pz : pt;
            c0 = pz >= 0 ? P.mu : sg;
            if (pz >= 0 && pt >= 0) { a1 = pt; c1 = sg; }
            bp = gi_cons_b(C, p);
        }
        const double sp = c0 * L.xs[a0] + (a1 >= 0 ? c1 * L.xs[a1] : 0.0) - bp;
        if (a1 < 0) {
            if (r == a0) {
#pragma unroll
                for (int j = 0; j < NH; ++j) {
                    const int c = h * NH + j;
                    const double v = c0 * Jr[j];
                    dB[c] = v;
                    dqB[c] = (c >= q) ? v : 0.0;
                    if ((j & 7) == 7) step_fence();
                }
            }
        } else {
            if (r == a0) {
#pragma unroll
                for (int j = 0; j < NH; ++j) {
                    dB[h * NH + j] = c0 * Jr[j];
                    if ((j & 7) == 7) step_fence();
                }
            }
            if (r == a1) {
#pragma unroll
                for (int j = 0; j < NH; ++j) {
                    d2B[h * NH + j] = c1 * Jr[j];
                    if ((j & 7) == 7) step_fence();
                }
            }
            __syncthreads();
            if (tid < NF) {
                const double v = dB[tid] + d2B[tid];
                dB[tid] = v;
                dqB[tid] = (tid >= q) ? v : 0.0;
            }
        }
        __syncthreads();
        MPCQP_SUB(tsub, 0);
        const double uq = us[q];
        // ---- step 2
        if (iters >= max_iter) { status = ST_ITER_LIMIT; break; }
        ++iters;
        {   // z = J2 d2 (per-half partial sums)
            double z4[4] = {0.0, 0.0, 0.0, 0.0};
            const double *dq = dqB + h * NH;
            const int qb = __builtin_amdgcn_readfirstlane(q - h * NH);  // first column of d2 here
#pragma unroll
            for (int b = 0; b < NH; b += 8) {
                if (!MPCQP_WG_SKIP || b + 7 >= qb) {
#pragma unroll
                    for (int j = b; j < b + 8 && j < NH; ++j) z4[j & 3] += Jr[j] * dq[j];
                }
                step_fence();
            }
            part[h * RW + r] = (z4[0] + z4[1]) + (z4[2] + z4[3]);
        }
        if (h == 0) {  // |d|^2, |d2|^2, |d2|^2 without d_q: thread r owns d_r
            const double dv = (r < nf) ? dB[r] : 0.0;
            double dd = dv * dv, zn = (r >= q) ? dv * dv : 0.0, zq = (r > q) ? dv * dv : 0.0;
            wave_sum3(dd, zn, zq);
            if (ln == 0) { red[8 + 3 * wv] = dd; red[9 + 3 * wv] = zn; red[10 + 3 * wv] = zq; }
        }
        MPCQP_SUB(tsub, 1);
        double r0 = 0.0, r1 = 0.0;  // wave 0 (every wave with RSPLIT): r of slots ln and ln + 64
        // the slot multipliers t1 divides, read before the barrier (wave 0 updates them after it)
        double us0 = 0.0, us1 = 0.0;
        if (MPCQP_WG_RINV && MPCQP_WG_RSPLIT && q > 0) {
            // this wave's columns j = wv, wv + 2 NWH, ...; partials to LDS, summed after the
            // barrier in wave order
            constexpr int NW = 2 * NWH;
            double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
            int j = wv;
            for (; j + NW < q; j += 2 * NW) {
                const double dj = dB[j], dk = dB[j + NW];
                a0 = fma((ln <= j) ? Lc[lrow(j) + ln] : 0.0, dj, a0);
                b0 = fma((ln <= j + NW) ? Lc[lrow(j + NW) + ln] : 0.0, dk, b0);
                if constexpr (TWO) {
                    a1 = fma((ln + 64 <= j) ? Lc[lrow(j) + ln + 64] : 0.0, dj, a1);
                    b1 = fma((ln + 64 <= j + NW) ? Lc[lrow(j + NW) + ln + 64] : 0.0, dk, b1);
                }
            }
            if (j < q) {
                const double dj = dB[j];
                a0 = fma((ln <= j) ? Lc[lrow(j) + ln] : 0.0, dj, a0);
                if constexpr (TWO) a1 = fma((ln + 64 <= j) ? Lc[lrow(j) + ln + 64] : 0.0, dj, a1);
            }
            us0 = us[ln];
            if constexpr (TWO) us1 = us[ln + 64];
            double *rp = W + Lay::oRp + wv * RW;
            rp[ln] = a0 + b0;
            if constexpr (TWO) rp[ln + 64] = a1 + b1;
        }
        if (MPCQP_WG_RINV && !MPCQP_WG_RSPLIT && wv == 0 && q > 0) {
            // r = R^-1 d(0:q): slot i takes row i of R^-1 against the published d (uniform
            // addresses); independent products in two accumulators per slot
            double a0[2] = {0.0, 0.0}, a1[2] = {0.0, 0.0};
#pragma unroll 4
            for (int j = 0; j < q; ++j) {
                const double dj = dB[j];
                const double v0 = (ln <= j) ? Lc[lrow(j) + ln] : 0.0;
                a0[j & 1] = fma(v0, dj, a0[j & 1]);
                if constexpr (TWO) {
                    const double v1 = (ln + 64 <= j) ? Lc[lrow(j) + ln + 64] : 0.0;
                    a1[j & 1] = fma(v1, dj, a1[j & 1]);
                }
            }
            r0 = (ln < q) ? a0[0] + a0[1] : 0.0;
            r1 = (TWO && ln + 64 < q) ? a1[0] + a1[1] : 0.0;
        }
        if (!MPCQP_WG_RINV && wv == 0 && q > 0) {
            // r = R^-1 d(0:q), back substitution (R packed in LDS, 1/R(j,j) beside it).  The
            // chain from one step to the next is v_readlane -> mul -> FMA in registers: 1/R(j,j)
            // is read out of registers too, and R's columns are prefetched two steps ahead, so
            // no LDS latency sits on it; the FMA runs on every lane (a lane past its slot only
            // changes a value that was already read)
            double v0 = (ln < q) ? dB[ln] : 0.0, v1 = (TWO && ln + 64 < q) ? dB[ln + 64] : 0.0;
            const double ri0 = (ln < q) ? rinv[ln] : 0.0;
            const double ri1 = (TWO && ln + 64 < q) ? rinv[ln + 64] : 0.0;
            auto col0 = [&](int jj) { return (jj >= 0 && ln < jj) ? Lc[roff(jj) + ln] : 0.0; };
            auto col1 = [&](int jj) {
                return (TWO && jj >= 0 && ln + 64 < jj) ? Lc[roff(jj) + ln + 64] : 0.0;
            };
            int j = q - 1;
            if constexpr (TWO) {
                // slots >= 64: four columns per block as below (one wave per SIMD at NF = 128,
                // so the LDS latency of a two-step prefetch sat on the chain); a block's steps
                // below 64 are left to the loop after it, which restarts at column 63
                if (j >= 64) {
                    double ca[4], cb[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) { ca[t] = col0(j - t); cb[t] = col1(j - t); }
                    for (; j >= 64; j -= 4) {
                        double na[4], nb[4];
#pragma unroll
                        for (int t = 0; t < 4; ++t) { na[t] = col0(j - 4 - t); nb[t] = col1(j - 4 - t); }
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int jj = j - t;
                            if (jj >= 64) {
                                const double rj = readlane(v1, jj - 64) * readlane(ri1, jj - 64);
                                if (ln + 64 == jj) r1 = rj;
                                v0 -= ca[t] * rj;
                                v1 -= cb[t] * rj;
                            }
                        }
#pragma unroll
                        for (int t = 0; t < 4; ++t) { ca[t] = na[t]; cb[t] = nb[t]; }
                    }
                    j = 63;
                }
            }
            // four columns per block, the next block's loads issued before this block's chain
            double cc[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) cc[t] = col0(j - t);
            for (; j >= 0; j -= 4) {
                double nc[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) nc[t] = col0(j - 4 - t);
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int jj = j - t;
                    if (jj >= 0) {
                        const double rj = readlane(v0, jj) * readlane(ri0, jj);
                        if (ln == jj) r0 = rj;
                        v0 -= cc[t] * rj;
                    }
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) cc[t] = nc[t];
            }
        }
        if (!(MPCQP_WG_RINV && MPCQP_WG_RSPLIT) && wv == 0 && q > 0) {
            const double rmax = wave_max(fmax(ln < q ? fabs(r0) : 0.0, ln + 64 < q ? fabs(r1) : 0.0));
            double t1 = INFINITY;
            int ks = 0x7fffffff;
            if (ln < q && r0 > kRTol * rmax) { t1 = fdiv(us[ln], r0); ks = ln; }
            if (TWO && ln + 64 < q && r1 > kRTol * rmax) {
                const double tt = fdiv(us[ln + 64], r1);
                if (tt < t1) { t1 = tt; ks = ln + 64; }
            }
            wave_argmin(t1, ks);
            if (ln == 0) { red[16] = t1; red[17] = (double)ks; }
        }
        __syncthreads();
        double t1 = INFINITY;
        int kslot = 0x7fffffff;
        if (MPCQP_WG_RINV && MPCQP_WG_RSPLIT && q > 0) {
            const double *rp = W + Lay::oRp;
            constexpr int NW = 2 * NWH;
            double v0 = rp[ln], v1 = TWO ? rp[ln + 64] : 0.0;
#pragma unroll
            for (int w = 1; w < NW; ++w) {
                v0 += rp[w * RW + ln];
                if constexpr (TWO) v1 += rp[w * RW + ln + 64];
            }
            r0 = (ln < q) ? v0 : 0.0;
            r1 = (TWO && ln + 64 < q) ? v1 : 0.0;
            const double rmax = wave_max(fmax(fabs(r0), fabs(r1)));
            if (ln < q && r0 > kRTol * rmax) { t1 = fdiv(us0, r0); kslot = ln; }
            if (TWO && ln + 64 < q && r1 > kRTol * rmax) {
                const double tt = fdiv(us1, r1);
                if (tt < t1) { t1 = tt; kslot = ln + 64; }
            }
            wave_argmin(t1, kslot);
        } else if (q > 0) {
            t1 = red[16];
            kslot = (int)red[17];
        }
        MPCQP_SUB(tsub, 2);
        const double z = part[r] + part[RW + r];
        const double dd = NWH == 2 ? red[8] + red[11] : red[8];
        const double zn = NWH == 2 ? red[9] + red[12] : red[9];
        const double zq = NWH == 2 ? red[10] + red[13] : red[10];
        const bool dep = !(zn > kDepTol * dd);
        const double t2 = dep ? INFINITY : fdiv(-sp, zn);
        const double t = t1 < t2 ? t1 : t2;
        if (isinf(t)) { status = ST_INFEASIBLE; break; }
        if (!isinf(t2)) {
            if (r < nf) x += t * z;
            if (h == 0) L.xs[r] = x;
            fval += t * zn * (0.5 * t + uq);
        }
        if (wv == 0) {
            double u0 = us[ln];
            if (ln < q) u0 -= t * r0;
            if (ln == q) u0 += t;
            us[ln] = u0;
            if constexpr (TWO) {
                double u1 = us[ln + 64];
                if (ln + 64 < q) u1 -= t * r1;
                if (ln + 64 == q) u1 += t;
                us[ln + 64] = u1;
            }
        }
        const bool add = !isinf(t2) && t2 <= t1;
        if (kStReg && add) {  // (L.st[p] = 2 below, by wave 0)
            s0r = (p == r) ? 2 : s0r;
            s1r = (p == r + nf) ? 2 : s1r;
        }
        double beta = 0.0;
        if (add) {
            // ---- add p: the Householder reflection of gi_reg.hpp, v = d2 - |d2| e_q
            const double dq = dB[q];
            double rqq = dq, vq = 0.0;
            if (zq > 0.0) {
                const double nrm = sqrt(zn);
                rqq = nrm;
                vq = dq > 0.0 ? fdiv(-zq, dq + nrm) : dq - nrm;
                beta = fdiv(2.0, vq * vq + zq);
            }
            if (wv == 0) {
                if (MPCQP_WG_RINV) {
                    // R^-1 of [[R, d1], [0, rqq]]: new column q = (-R^-1 d1 / rqq, 1 / rqq), and
                    // R^-1 d1 is this pass's r (wave 0's r0 / r1)
                    const double irq = fdiv(1.0, rqq);
                    if (ln < q) Lc[lrow(q) + ln] = -r0 * irq;
                    if (TWO && ln + 64 < q) Lc[lrow(q) + ln + 64] = -r1 * irq;
                    if (ln == 0) {
                        Lc[lrow(q) + q] = irq;
                        acts[q] = p;
                        L.st[p] = 2;
                    }
                } else {
                    if (ln < q) Lc[roff(q) + ln] = dB[ln];
                    if (TWO && ln + 64 < q) Lc[roff(q) + ln + 64] = dB[ln + 64];
                    if (ln == 0) {
                        Lc[roff(q) + q] = rqq;
                        rinv[q] = fdiv(1.0, rqq);
                        acts[q] = p;
                        L.st[p] = 2;
                    }
                }
            }
            // the reflector's slot q: written by every wave for its own J update below (LDS is
            // in order within a wave, and no wave reads dqB between the barrier after the R
            // solve and that update), so the add step needs no workgroup barrier of its own
            if (ln == 0) dqB[q] = vq;
            ++q;
            fresh = true;
        } else {
            // ---- drop slot kslot (wave 0): shift the slots and R's columns left, then Givens
            //      back to triangular; the rotations go to LDS for J
            const int k = kslot;
            if (wv == 0) {
                const int dropped = acts[k];
                const double un0 = (ln + 1 < RW) ? us[ln + 1] : 0.0;
                const int an0 = (ln + 1 < RW) ? acts[ln + 1] : 0;
                const double un1 = (TWO && ln + 65 < RW) ? us[ln + 65] : 0.0;
                const int an1 = (TWO && ln + 65 < RW) ? acts[ln + 65] : 0;
                wave_sync();
                // slots k .. q-1 take their successor's entries; slot q-1 receives slot q's
                // u, the partial multiplier of the constraint being added
                if (ln >= k && ln < q) { us[ln] = un0; acts[ln] = an0; }
                if (TWO && ln + 64 >= k && ln + 64 < q) { us[ln + 64] = un1; acts[ln + 64] = an1; }
                if (ln == 0) L.st[dropped] = 1;
                if (MPCQP_WG_RINV && MPCQP_WG_PDROP) {
                    const int qn = q - 1;
                    const double ra0 = Lc[lrow(k) + k];
                    const int j0 = ln, j1 = ln + 64;
                    const double rb0 = (j0 >= k && j0 < qn) ? Lc[lrow(j0 + 1) + k] : 0.0;
                    const double rb1 = (TWO && j1 >= k && j1 < qn) ? Lc[lrow(j1 + 1) + k] : 0.0;
                    // the DPP moves run with every lane active: pinned here, not sunk into the
                    // selects' branches (a disabled source lane reads 0)
                    const double a2 = ra0 * ra0;
                    double p0 = wave_prefix_sum(rb0 * rb0);
                    pin(p0);
                    const double H0 = sqrt(a2 + p0);
                    double hp0 = wave_prev(H0);
                    pin(hp0);
                    if (j0 < NF) {
                        const bool on = j0 >= k && j0 < qn;
                        const double pv = (j0 == k) ? ra0 : hp0;
                        const double ih = fdiv(1.0, H0);
                        rot[2 * j0] = on ? rb0 * ih : 1.0;
                        rot[2 * j0 + 1] = on ? -pv * ih : 0.0;
                    }
                    if constexpr (TWO) {
                        double p1 = wave_prefix_sum(rb1 * rb1);
                        pin(p1);
                        const double H1 = sqrt(a2 + (p1 + readlane(p0, 63)));
                        double pw = wave_prev(H1);
                        pin(pw);
                        const double pv = (j1 == k) ? ra0 : (ln == 0 ? readlane(H0, 63) : pw);
                        const bool on = j1 >= k && j1 < qn;
                        const double ih = 1.0 / H1;
                        if (j1 < NF) {
                            rot[2 * j1] = on ? rb1 * ih : 1.0;
                            rot[2 * j1 + 1] = on ? -pv * ih : 0.0;
                        }
                    }
                    wave_sync();
                    // rows ln (and ln + 64): the rotated column j (row k deleted) is final once
                    // rotated; the carry is column j + 1 as rotated so far
                    double cr0 = (ln <= k) ? Lc[lrow(k) + ln] : 0.0;
                    double cr1 = (TWO && ln + 64 <= k) ? Lc[lrow(k) + ln + 64] : 0.0;
                    auto step = [&](int j, double c, double s_, double y0, double y1) {
                        const double o0 = c * cr0 + s_ * y0;
                        cr0 = -s_ * cr0 + c * y0;
                        if (ln <= j + 1 && ln != k) Lc[lrow(j) + ln - (ln > k ? 1 : 0)] = o0;
                        if constexpr (TWO) {
                            const int i1 = ln + 64;
                            const double o1 = c * cr1 + s_ * y1;
                            cr1 = -s_ * cr1 + c * y1;
                            if (i1 <= j + 1 && i1 != k) Lc[lrow(j) + i1 - (i1 > k ? 1 : 0)] = o1;
                        }
                    };
                    int j = k;
                    // every load of a block (columns j+1 .. j+4, original) before its stores
                    // (columns j .. j+3, rows shifted up past k): other lanes' stores land on
                    // rows this lane reads
                    for (; j + 4 <= qn; j += 4) {
                        double c[4], s4[4], y0[4], y1[4];
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            c[t] = rot[2 * (j + t)];
                            s4[t] = rot[2 * (j + t) + 1];
                            y0[t] = (ln <= j + t + 1) ? Lc[lrow(j + t + 1) + ln] : 0.0;
                            y1[t] = (TWO && ln + 64 <= j + t + 1) ? Lc[lrow(j + t + 1) + ln + 64] : 0.0;
                        }
                        step_fence();
#pragma unroll
                        for (int t = 0; t < 4; ++t) step(j + t, c[t], s4[t], y0[t], y1[t]);
                        step_fence();
                    }
                    for (; j < qn; ++j) {
                        const double c = rot[2 * j], s_ = rot[2 * j + 1];
                        const double y0 = (ln <= j + 1) ? Lc[lrow(j + 1) + ln] : 0.0;
                        const double y1 = (TWO && ln + 64 <= j + 1) ? Lc[lrow(j + 1) + ln + 64] : 0.0;
                        step_fence();
                        step(j, c, s_, y0, y1);
                        step_fence();
                    }
                } else if (MPCQP_WG_RINV) {
                    // R^-1 G' with the rotations that zero row k of R^-1 left of column q-1 (the
                    // same G as restores R without column k: mpc_pair.hpp), row k deleted and the
                    // last column dropped; each rotated column j is final once rotated
                    const int qn = q - 1;
                    for (int j = ln; j < NF; j += kWave) { rot[2 * j] = 1.0; rot[2 * j + 1] = 0.0; }
                    wave_sync();
                    double ra = Lc[lrow(k) + k];
                    for (int j = k; j < qn; ++j) {
                        const double rb = Lc[lrow(j + 1) + k];
                        double c = 1.0, s_ = 0.0;
                        if (ra != 0.0) {
                            const double hh = sqrt(ra * ra + rb * rb), ih = 1.0 / hh;
                            c = rb * ih;
                            s_ = -ra * ih;
                            ra = hh;
                        } else {
                            ra = rb;
                        }
                        const int i0 = ln, i1 = ln + 64;
                        const double y00 = (i0 <= j) ? Lc[lrow(j) + i0] : 0.0;
                        const double y10 = (i0 <= j + 1) ? Lc[lrow(j + 1) + i0] : 0.0;
                        double y01 = 0.0, y11 = 0.0;
                        if (TWO) {
                            y01 = (i1 <= j) ? Lc[lrow(j) + i1] : 0.0;
                            y11 = (i1 <= j + 1) ? Lc[lrow(j + 1) + i1] : 0.0;
                        }
                        if (i0 <= j + 1 && i0 != k) Lc[lrow(j) + i0 - (i0 > k ? 1 : 0)] = c * y00 + s_ * y10;
                        if (i0 <= j + 1) Lc[lrow(j + 1) + i0] = -s_ * y00 + c * y10;
                        if (TWO) {
                            if (i1 <= j + 1 && i1 != k) Lc[lrow(j) + i1 - (i1 > k ? 1 : 0)] = c * y01 + s_ * y11;
                            if (i1 <= j + 1) Lc[lrow(j + 1) + i1] = -s_ * y01 + c * y11;
                        }
                        if (ln == 0) {
                            rot[2 * j] = c;
                            rot[2 * j + 1] = s_;
                        }
                        wave_sync();
                    }
                }
                for (int j = k; !MPCQP_WG_RINV && j < q - 1; ++j) {
                    const double v0 = (ln <= j + 1) ? Lc[roff(j + 1) + ln] : 0.0;
                    const double v1 = (TWO && ln + 64 <= j + 1) ? Lc[roff(j + 1) + ln + 64] : 0.0;
                    if (ln <= j + 1) Lc[roff(j) + ln] = v0;
                    if (TWO && ln + 64 <= j + 1) Lc[roff(j) + ln + 64] = v1;
                }
                const int qn = q - 1;
                if (!MPCQP_WG_RINV)
                    for (int j = ln; j < NF; j += kWave) { rot[2 * j] = 1.0; rot[2 * j + 1] = 0.0; }
                wave_sync();
                for (int j = k; !MPCQP_WG_RINV && j < qn; ++j) {
                    const double a_ = Lc[roff(j) + j], bb = Lc[roff(j) + j + 1];
                    if (bb != 0.0) {
                        const double hh = sqrt(a_ * a_ + bb * bb);
                        const double ih = 1.0 / hh;
                        const double c = a_ * ih, s_ = bb * ih;
#pragma unroll
                        for (int o = 0; o < (TWO ? 2 : 1); ++o) {
                            const int l = j + 1 + ln + 64 * o;
                            if (l < qn) {
                                const double y0 = Lc[roff(l) + j], y1 = Lc[roff(l) + j + 1];
                                Lc[roff(l) + j] = c * y0 + s_ * y1;
                                Lc[roff(l) + j + 1] = -s_ * y0 + c * y1;
                            }
                        }
                        if (ln == 0) {
                            Lc[roff(j) + j] = hh;
                            Lc[roff(j) + j + 1] = 0.0;
                            rinv[j] = ih;
                            rot[2 * j] = c;
                            rot[2 * j + 1] = s_;
                        }
                    } else if (ln == 0) {
                        rinv[j] = 1.0 / a_;  // the shifted column's diagonal as it is
                    }
                    wave_sync();
                }
            }
            --q;
        }
        // ---- the pass's update of J, as two sequential workgroup-uniform steps (not the arms
        //      of the if / else above): one definition chain of Jr, so the register allocator
        //      keeps a single copy of it
        if (__builtin_amdgcn_readfirstlane((int)(add && beta != 0.0))) {
            double w4[4] = {0.0, 0.0, 0.0, 0.0};
            const double *v = dqB + h * NH;
            // the reflector is zero left of the slot just added (q - 1)
            const int qb = __builtin_amdgcn_readfirstlane(q - 1 - h * NH);
#pragma unroll
            for (int b = 0; b < NH; b += 8) {
                if (!MPCQP_WG_SKIP || b + 7 >= qb) {
#pragma unroll
                    for (int j = b; j < b + 8 && j < NH; ++j) w4[j & 3] += Jr[j] * v[j];
                }
                step_fence();
            }
            // partial sums into d2B / tB (dead on the add path), not part: a lagging wave may
            // still be reading this pass's z out of part
            (h ? tB : d2B)[r] = (w4[0] + w4[1]) + (w4[2] + w4[3]);
            __syncthreads();
            const double f = beta * (d2B[r] + tB[r]);
#pragma unroll
            for (int b = 0; b < NH; b += 8) {
                if (!MPCQP_WG_SKIP || b + 7 >= qb) {
#pragma unroll
                    for (int j = b; j < b + 8 && j < NH; ++j) Jr[j] -= f * v[j];
                }
                step_fence();
            }
        }
        if (__builtin_amdgcn_readfirstlane((int)!add)) {
            // J columns: rotations (j, j+1), j = 0 .. NF-2, identity where (c, s) = (1, 0) -- all
            // but j = kslot .. q-1 (q after the drop).  Half 0 applies 0 .. NH-1 (the last one
            // needs column NH from half 1), then half 1 continues from the carried column NH;
            // when rotation NH-1 is the identity the halves run at once, no carry.  8-rotation
            // blocks outside kslot .. q-1 are skipped (uniform branches; the block's loads issue
            // together)
            const int jlo = __builtin_amdgcn_readfirstlane(kslot), jhi = __builtin_amdgcn_readfirstlane(q - 1);
            auto live_blk = [&](int j0, int j1) { return !MPCQP_WG_SKIP || (j1 >= jlo && j0 <= jhi); };
            auto rot_half = [&](int base) {  // rotations base + j, j = 0 .. NH-2, in registers
#pragma unroll
                for (int b = 0; b < NH - 1; b += 8) {
                    if (live_blk(base + b, base + b + 7)) {
#pragma unroll
                        for (int j = b; j < b + 8 && j < NH - 1; ++j) {
                            const double c = rot[2 * (base + j)], s_ = rot[2 * (base + j) + 1];
                            const double y0 = Jr[j], y1 = Jr[j + 1];
                            Jr[j] = c * y0 + s_ * y1;
                            Jr[j + 1] = -s_ * y0 + c * y1;
                        }
                    }
                }
            };
            const bool cross = !MPCQP_WG_SKIP || (jlo <= NH - 1 && jhi >= NH - 1);
            if (cross && h == 1) d2B[r] = Jr[0];
            __syncthreads();  // wave 0's rotations (and the carried column) are in LDS
            if (h == 0) rot_half(0);
            if (cross) {
                if (h == 0) {
                    const double c = rot[2 * (NH - 1)], s_ = rot[2 * (NH - 1) + 1];
                    const double y0 = Jr[NH - 1], y1 = d2B[r];
                    Jr[NH - 1] = c * y0 + s_ * y1;
                    tB[r] = -s_ * y0 + c * y1;
                }
                __syncthreads();
                if (h == 1) Jr[0] = tB[r];
            }
            if (h == 1) rot_half(NH);
        }
        __syncthreads();
        if (kStReg && !add && h == 0 && r < nf) {  // a drop set L.st[dropped] = 1 (wave 0, before the barrier)
            s0r = L.st[r];
            s1r = L.st[r + nf];
        }
    }
    MPCQP_SUB(tsub, 3);
    MPCQP_SUB_FLUSH(C.stamps, tsub);
    MPCQP_STAMP(C.stamps, 8, tst);
    MPCQP_CUT(C.cut, 7);
    C.status = status;
    C.x = x;
    C.fval = fval;
    C.q = q;
    C.iters = iters;
    C.u = 0.0;
    C.act = -1;
}

// outputs of a workgroup solve: x of the free variables from the rows of half 0, fixed values,
// cost / status / iterations (gi_write's conventions)
template <int NF>
__device__ __forceinline__ void gi_write_wg(GiCtx &C, const SolveOut &O) {
    constexpr int RW = WgShape<NF>::RW;
    const SolveProblem &P = *C.P;
    GiLds &L = C.L;
    const WgIds T = wg_ids<RW>();
    const int nV = P.nV, nf = C.nf;
    const bool have_map = nf <= C.nfmax;
    for (int v = T.tid; v < nV; v += 2 * RW) {
        const int pv = L.pos[v];
        if (pv < 0 || !have_map) O.x[v] = (pv < 0) ? L.xfull[v] : 0.0;
    }
    if (have_map && T.h == 0 && T.r < nf) O.x[L.fid[T.r]] = C.x;
    if (T.tid == 0) {
        *O.cost = C.fval + C.c0;
        *O.status = C.status;
        *O.iters = C.iters;
    }
}

}  // namespace mpcqp
