// gi_crash_reg.hpp -- warm-started working-set start of the one-QP register solver (gi_reg.hpp;
// configs C and L in the closed-loop rollout).
//
// The dual loop adds one constraint per pass, so a warm start that only reorders its adds
// (gi_reg.hpp WarmSet) cannot take fewer passes than the active set has members.  This start
// solves the previous tick's active set (one horizon step later) as equalities in ONE step and
// iterates the primal-dual active-set rule on it: drop the constraints whose multiplier is
// negative, add the ones the new x violates; an unchanged set is the optimum (the KKT point of
// the strictly convex QP within the dual loop's tolerances, the point the dual loop reaches).
// After kRegCrashP sets, more than kRegCrashK constraints or a non-positive pivot it gives up
// and the dual loop runs from the unconstrained minimum exactly as without it.
//
// Constraint c of lane l (the variable of slot l): c = 0 its lower bound x_l >= b, c = 1 its
// upper bound -x_l >= b, c = 2 + t friction row t of the foot-step whose vertical force is l:
// mu x_l + sg x_(l-2+(t>>1)) >= 0, sg = t odd ? +1 : -1 (gi_project_reg's rows; the foot's
// forces sit at consecutive slots l-2, l-1, l).  With N the normals of the set A and
// v_a = J' n_a (J J' = H^-1): M = N' H^-1 N = V V', M w = N' x0 - b, x = x0 - J V' w, the
// multipliers lambda = -w, the objective f0 + w' (N' x0 - b) / 2.
//   * the rows v_a go to LDS (stride kRegCrashLD: rows four banks apart); a friction row is
//     mu J_l written by lane l, then + sg J_ft added by the lane of f_t
//   * M = V V' is ONE 16 x 16 tile of v_mfma_f64_16x16x4_f64 (K = NF): lane l supplies
//     V(l & 15, 4s + (l >> 4)), which is A and B at once
//   * Gauss-Jordan without pivoting (M is positive definite) on the tile in the accumulator
//     registers, one pivot row and column published per step
#pragma once
#include "gi_solver.hpp"
#include "mfma_ops.hpp"

namespace mpcqp {

constexpr int kRegCrashK = 16;   // constraints per working set (one MFMA tile of M)
constexpr int kRegCrashP = 6;    // working sets before giving up
constexpr int kRegCrashLD = 66;  // published row stride (doubles): 132 dwords = 4 banks apart

// LDS (doubles, in the R space, free until the dual loop's first add): rows [K][LD], the pivot
// row and column [K] each, w, the right-hand sides (eliminated, original) by rank [K] each, y [NF]
template <int NF>
struct RegCrashLayout {
    static constexpr int K = kRegCrashK, LD = kRegCrashLD;
    static constexpr int oW = 0, oPv = oW + K * LD, oWv = oPv + 2 * K, oRv = oWv + K,
                         oRs = oRv + K, oY = oRs + K, end = oY + NF;
    static_assert(NF <= LD - 2 && NF % 4 == 0, "rows fit the stride; the MFMA K steps are whole");
};

// lane l's slack of constraint c at x (x_l on this lane, x_(l-1), x_(l-2) from the lanes below)
__device__ __forceinline__ double crash_slack(int c, double x, double xm1, double xm2, double blo,
                                              double bhi, double mu) {
    if (c == 0) return x - blo;
    if (c == 1) return -x - bhi;
    const int t = c - 2;
    const double sg = (t & 1) ? 1.0 : -1.0;
    double s = 0.0;
    s += mu * x;
    s += sg * ((t >> 1) ? xm1 : xm2);
    return s;
}

template <int NF>
__device__ __forceinline__ bool reg_warm_crash(GiCtx &C, const double (&Jr)[NF], int fbase,
                                               int gmask, double &x, double &fval, int &iters,
                                               double *S) {
    using Lay = RegCrashLayout<NF>;
    constexpr int KC = kRegCrashK, LD = kRegCrashLD;
    GiLds &L = C.L;
    const SolveProblem &P = *C.P;
    const int nf = C.nf, ln = lane(), li = ln & 15, lk = ln >> 4;
    double *W = S + Lay::oW, *Pv = S + Lay::oPv, *Wv = S + Lay::oWv, *Rv = S + Lay::oRv,
           *Rs = S + Lay::oRs, *Yv = S + Lay::oY;
    const double mu = P.mu;
    // this lane's constraints: eligibility (state 1: inactive, may be added) and b
    int elig = 0;
    double blo = 0.0, bhi = 0.0;
    if (ln < nf) {
        if (L.st[ln] == 1) elig |= 1;
        if (L.st[ln + nf] == 1) elig |= 2;
        blo = L.cb[ln];
        bhi = L.cb[ln + nf];
        if (fbase >= 0) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (L.st[fbase + t] == 1) elig |= 4 << t;
        }
    }
    const double tlo = -kFeasTol * (1.0 + fabs(blo)), thi = -kFeasTol * (1.0 + fabs(bhi)),
                 trow = -kFeasTol;
    const double x0 = x, f0 = fval;
    const double x0m1 = wave_prev(x0), x0m2 = wave_prev(x0m1);
    double xc = x0, fc = f0;
    int sel = 0, negb = 0;
    for (int it = 0;; ++it) {
        // ---- the next set: drop negative multipliers, add what xc violates (and, first, the seed)
        const double xm1 = wave_prev(xc), xm2 = wave_prev(xm1);
        int nsel = 0;
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            const int bit = 1 << c;
            if (!(elig & bit) && !(sel & bit)) continue;
            const double s = crash_slack(c, xc, xm1, xm2, blo, bhi, mu);
            const double tol = c == 0 ? tlo : (c == 1 ? thi : trow);
            const bool keep = (sel & bit) && !(negb & bit);
            const bool add = !(sel & bit) && (s < tol || (it == 0 && (gmask & bit)));
            if (keep || add) nsel |= bit;
        }
        const bool changed = __ballot(nsel != sel) != 0ull;
        if (!changed) {  // the optimum (for it == 0: x0 itself, nothing seeded or violated)
            x = xc;
            fval = fc;
            if (ln < nf) {
                L.xs[ln] = x;
                if (sel & 1) L.st[ln] = 2;
                if (sel & 2) L.st[ln + nf] = 2;
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (sel & (4 << t)) L.st[fbase + t] = 2;
            }
            wave_sync();
            return true;
        }
        if (it >= kRegCrashP) return false;
        sel = nsel;
        // ---- ranks: (lane, constraint) order; k constraints in all
        int k = 0, rb = 0;
        const unsigned long long below = (1ull << ln) - 1ull;
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            const unsigned long long m = __ballot((sel >> c) & 1);
            k += __popcll(m);
            rb += __popcll(m & below);
        }
        if (k > KC) return false;
        if (k == 0) {  // (every member dropped: back to the unconstrained minimum)
            xc = x0;
            fc = f0;
            negb = 0;
            continue;
        }
        ++iters;
        // ---- rows v_a and right-hand sides s_a(x0) by rank
        {
            int r = rb;
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                if (sel & (1 << c)) {
                    // (the scale made opaque inside the loop: hoisted out of it, the loop-invariant
                    //  products mu J and -J took 240 registers across the whole start)
                    double sc = c == 0 ? 1.0 : (c == 1 ? -1.0 : mu);
                    asm volatile("" : "+v"(sc));
#pragma unroll
                    for (int q = 0; q < NF; ++q) {
                        W[r * LD + q] = sc * Jr[q];
                        if ((q & 7) == 7) step_fence();  // (bounds the products held for stores)
                    }
                    Rv[r] = Rs[r] = crash_slack(c, x0, x0m1, x0m2, blo, bhi, mu);
                    ++r;
                }
            }
        }
        wave_sync();
        {   // the f_t part of friction rows: lane l is f_x of the foot-step at l + 2 (rows 0, 1)
            // and f_y of the one at l + 1 (rows 2, 3); each row is touched by one lane here
            const int s1 = __shfl_down(sel, 1, kWave), s2 = __shfl_down(sel, 2, kWave);
            const int r1 = __shfl_down(rb, 1, kWave), r2 = __shfl_down(rb, 2, kWave);
            const bool v1 = ln + 1 < kWave, v2 = ln + 2 < kWave;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int ss = t < 2 ? s2 : s1, rr = t < 2 ? r2 : r1;
                const bool vv = t < 2 ? v2 : v1;
                if (vv && ln < nf && (ss & (4 << t))) {
                    const int row = rr + __popc(ss & ((4 << t) - 1));
                    double sg = (t & 1) ? 1.0 : -1.0;
                    asm volatile("" : "+v"(sg));  // (not hoisted: see the rows above)
#pragma unroll
                    for (int q = 0; q < NF; ++q) {
                        W[row * LD + q] += sg * Jr[q];
                        if ((q & 7) == 7) step_fence();  // (bounds the loads in flight)
                    }
                }
            }
        }
        wave_sync();
        // ---- M = V V' on the matrix cores: one 16 x 16 tile, K = NF; lane l keeps
        //      M(lk + 4q, li) in its accumulator registers (q = 0..3)
        dx4 Mt = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < NF / 4; ++s) {
            const double v = li < k ? W[li * LD + 4 * s + lk] : 0.0;
            Mt = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, Mt, 0, 0, 0);
        }
        const bool inA = ln < k;
        const int kmax = k;  // (wave-uniform)
        // ---- Gauss-Jordan without pivoting on the tile in place (4 registers per lane): step j
        //      publishes row j and column j, every element (r, m), r != j, takes
        //      -= (M(r, j) / M(j, j)) M(j, m); the right-hand sides (LDS, by rank) likewise
        double *Pr = Pv, *Pc = Pv + 16;
        bool bad = false;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            if (j < kmax) {
                if (lk == (j & 3)) Pr[li] = Mt[j >> 2];
                if (li == j) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) Pc[lk + 4 * q] = Mt[q];
                }
                wave_sync();
                const double piv = Pr[j], ip = 1.0 / piv, pm = Pr[li], rj = Rv[j];
                bad |= !(piv > 0.0);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = lk + 4 * q;
                    if (r != j) Mt[q] -= (Pc[r] * ip) * pm;
                }
                if (inA && ln != j) Rv[ln] -= (Pc[ln] * ip) * rj;
                wave_sync();
            }
        }
        if (__ballot(bad) != 0ull) return false;
        // w = rhs / diagonal (the diagonal entry (r, r) lives on lane li = r, lk = r & 3, q = r >> 2)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (li == lk + 4 * q) Pr[li] = Mt[q];
        wave_sync();
        const double r0 = inA ? Rs[ln] : 0.0, rr = inA ? Rv[ln] : 0.0, dd = inA ? Pr[ln] : 1.0;
        const double w = inA ? rr / dd : 0.0;
        if (inA) Wv[ln] = w;
        const double wr = wave_sum(inA ? w * r0 : 0.0);
        wave_sync();
        // ---- y = V' w (lane q: column q), x = x0 - J y
        if (ln < NF) {
            double y = 0.0;
            for (int m = 0; m < kmax; ++m) y += W[m * LD + ln] * Wv[m];
            Yv[ln] = y;
        }
        wave_sync();
        double s4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < NF; ++q) {
            s4[q & 3] += Jr[q] * Yv[q];
            if ((q & 7) == 7) {  // (partial sums pinned: no more than 8 loads held at once)
                pin(s4[0]);
                pin(s4[1]);
                pin(s4[2]);
                pin(s4[3]);
                step_fence();
            }
        }
        xc = ln < nf ? x0 - ((s4[0] + s4[1]) + (s4[2] + s4[3])) : 0.0;
        if (sel & 1) xc = blo;  // (a bound in the set holds exactly)
        if (sel & 2) xc = -bhi;
        fc = f0 + 0.5 * wr;
        // multipliers of this lane's members (lambda = -w): negative -> dropped next
        negb = 0;
        {
            int r = rb;
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                if (sel & (1 << c)) {
                    if (-Wv[r] < 0.0) negb |= 1 << c;
                    ++r;
                }
            }
        }
        wave_sync();
    }
}

}  // namespace mpcqp
