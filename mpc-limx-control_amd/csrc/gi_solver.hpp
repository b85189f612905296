// gi_solver.hpp -- dense strictly-convex QP solve, one instance per 64-lane wavefront.
//
// Replaces the reference's qpOASES call in QPSolver::solveQP (src/QPSolver.cpp:83-106) by the
// Goldfarb-Idnani (1983) dual active-set method in its J = L^-T Q / R factored form.  The
// corrected QP (bounds + real inequality rows, no equality block) is strictly
// convex, so its optimum is unique; this is the same algorithm, constraint order and
// tolerances as the CPU oracle (oracle/mpcqp_oracle.c, gi_solve), so iteration counts match.
//
// Mapping: lane i owns row i of J and x_i; lane j owns active slot j (d_j, r_j, u_j, id_j).
// J and R live in LDS column-major with an odd leading dimension: column sweeps (lane i reads
// J(i, j)) are unit-stride and row gathers (lane j reads J(v, j)) stride ld, both conflict
// free for ds_read_b64.  x is mirrored in LDS (xs) for the constraint sweeps.
//   constraint ids: [0,nf) lower bounds, [nf,2nf) upper bounds,
//                   [2nf, 2nf+4*N*nfeet) friction rows (k, s, t), then dense rows (r, side).
//
// Stages (so the fused condense+solve kernel can build H_FF in LDS itself):
//   gi_setup      fixed variables, free index map, constraint states
//   gi_gather     H_FF, g = f_F + H_FB x_B from global memory (stand-alone solve)
//   gi_run        Cholesky, J = L^-T, unconstrained minimum, dual active-set loop
//   gi_write      x, cost, status, iterations, optional multipliers
#pragma once
#include "wave_ops.hpp"

namespace mpcqp {

constexpr double kInfty = 1e20;
constexpr double kFeasTol = 1e-11;  // violation threshold relative to (1 + |b|)
constexpr double kDepTol = 1e-20;   // |d2|^2 <= tol |d|^2  -> linearly dependent normal
constexpr double kRTol = 1e-12;     // r_j > tol * max|r| counts as blocking

enum { ST_OK = 0, ST_BAD_DIMS = 1, ST_INFEASIBLE = 2, ST_ITER_LIMIT = 3, ST_NOT_PD = 4 };

struct SolveProblem {
    int nV;                  // variables
    const double *H, *f;     // nV x nV column-major, nV
    const double *lb, *ub;   // nV each (used when gen_bounds == 0; nullptr = absent)
    // SRBM bound generation from the contact schedule
    int gen_bounds;
    int model, nu, N, nfeet;
    double fz_min, fz_max, fxy_max, u_min, u_max;
    uint64_t contact;
    // friction pyramid  mu fz -/+ fx >= 0, mu fz -/+ fy >= 0 for feet in contact
    int friction;
    double mu;
    // dense rows lbA <= A x <= ubA
    int mA;
    const double *A;         // row-major (a_colmajor = 0) or column-major
    int a_colmajor;
    const double *lbA, *ubA;
    int max_iter;
};

struct SolveOut {
    double *x;      // nV
    double *cost;   // 1
    int *status;    // 1
    int *iters;     // 1
    double *y;      // nullable: nV + mA multipliers (qpOASES convention)
    double *stage = nullptr;  // nullable: nV doubles of dead LDS; x is assembled there and
                              // written once, coalesced and non-temporal
};

// LDS workspace (bytes) for a free-variable cap and dims
__host__ __device__ inline size_t gi_lds_bytes(int nfmax, int nV, int mA, int nfric) {
    const int ld = nfmax | 1;
    const size_t mt = (size_t)2 * nfmax + nfric + 2 * mA;
    size_t b = 0;
    b += sizeof(double) * (size_t)2 * nfmax * ld;    // J, R
    b += sizeof(double) * (size_t)nfmax * 2;         // g, xs
    b += sizeof(double) * (size_t)nV;                // xfull
    b += sizeof(double) * (size_t)(mA > 0 ? mA : 1); // row fixed contributions
    b += sizeof(double) * (size_t)(nV + mA);         // y scratch
    b += sizeof(int) * (size_t)nfmax;                // fid
    b += sizeof(int) * (size_t)nV;                   // pos
    b += (mt + 15) & ~(size_t)15;                    // state byte per constraint id
    return (b + 15) & ~(size_t)15;
}

struct GiLds {
    double *J, *R, *g, *xs, *xfull, *rowfix, *ys;
    double *cb;  // nullable: b of every constraint id, precomputed by gi_setup (register solver)
    int *fid, *pos;
    unsigned char *st;  // 0 absent, 1 inactive, 2 active, 3 equality, 4 infeasible
    int ld;
};

// value of a fixed input (xfull == nullptr: the fused one-QP kernels, whose fixed inputs are 0)
__device__ __forceinline__ double xfixed(const GiLds &L, int v) {
    return L.xfull ? L.xfull[v] : 0.0;
}

__device__ __forceinline__ GiLds gi_carve(unsigned char *base, int nfmax, int nV, int mA) {
    GiLds L;
    L.ld = nfmax | 1;
    double *d = reinterpret_cast<double *>(base);
    L.J = d; d += nfmax * L.ld;
    L.R = d; d += nfmax * L.ld;
    L.g = d; d += nfmax;
    L.xs = d; d += nfmax;
    L.xfull = d; d += nV;
    L.rowfix = d; d += (mA > 0 ? mA : 1);
    L.ys = d; d += nV + mA;
    int *ip = reinterpret_cast<int *>(d);
    L.fid = ip; ip += nfmax;
    L.pos = ip; ip += nV;
    L.st = reinterpret_cast<unsigned char *>(ip);
    L.cb = nullptr;
    return L;
}

struct GiCtx {
    const SolveProblem *P;
    GiLds L;
    int nfmax, nf, nfric, mt;
    int status;
    double c0;     // objective contribution of the fixed variables
    // results of gi_run
    double x, u, fval;
    int act, q, iters;
    unsigned long long *stamps;  // diagnostic phase cycles (nullptr: off)
    int cut;                     // diagnostic cuts build only
    int wide;                    // 1: a workgroup solver (gi_wg.hpp) holds up to nfmax > 64
    int crash_p;                 // workgroup solver: crash start's working sets (0: none)
};

__device__ __forceinline__ double rowA(const SolveProblem &P, int r, int v) {
    return P.a_colmajor ? P.A[(size_t)v * P.mA + r] : P.A[(size_t)r * P.nV + v];
}

// SRBM / literal bounds of variable v (gen_bounds mode)
__device__ __forceinline__ void gen_bound(const SolveProblem &P, int v, double &lo, double &hi) {
    const int k = v / P.nu, c = v % P.nu;
    if (P.model != 0) { lo = P.u_min; hi = P.u_max; return; }  // literal / dense: input box
    const int s = c / 3, comp = c % 3;
    if ((P.contact >> (2 * k + s)) & 1ull) {
        if (comp == 2) { lo = P.fz_min; hi = P.fz_max; }
        else { lo = -P.fxy_max; hi = P.fxy_max; }
    } else { lo = 0.0; hi = 0.0; }
}

__device__ __forceinline__ void var_bounds(const SolveProblem &P, int v, double &lo, double &hi) {
    if (P.gen_bounds) { gen_bound(P, v, lo, hi); return; }
    lo = P.lb ? P.lb[v] : -kInfty;
    hi = P.ub ? P.ub[v] : kInfty;
}

// The most-violated selection's key when the QP has friction rows (qsel = nfric > 0 and a foot
// in contact): the violation with its low 20 mantissa bits cleared, so violations within ~2^-32
// relative tie and the lowest id wins, as for exact ties.  A pyramid's +- rows are exactly tied
// whenever the tangential force is zero, and rounding alone would otherwise pick one of them,
// differently here and in the oracle (gi_sel_key, oracle/mpcqp_oracle.c): same minimiser,
// different pass counts.  Box-only problems compare the violations themselves.
__device__ __forceinline__ double gi_sel_key(double s, bool qsel) {
    const long long b = __double_as_longlong(s) & ~0xFFFFFll;
    return qsel ? __longlong_as_double(b) : s;
}

// ---------------------------------------------------------------- constraint accessors
// b of the one-sided constraint id (normal' x_F >= b, fixed parts folded into b)
__device__ __forceinline__ double gi_cons_b(const GiCtx &C, int id) {
    const SolveProblem &P = *C.P;
    const GiLds &L = C.L;
    const int nf = C.nf, nfric = C.nfric;
    double lo, hi;
    if (id < nf) { var_bounds(P, L.fid[id], lo, hi); return lo; }
    if (id < 2 * nf) { var_bounds(P, L.fid[id - nf], lo, hi); return -hi; }
    if (id < 2 * nf + nfric) {
        const int r = id - 2 * nf, ks = r >> 2, t = r & 3;
        const int k = ks / P.nfeet, sft = ks % P.nfeet;
        const int vz = k * P.nu + 3 * sft + 2, vt = k * P.nu + 3 * sft + (t >> 1);
        const double sg = (t & 1) ? 1.0 : -1.0;
        double b = 0.0;
        if (L.pos[vz] < 0) b -= P.mu * xfixed(L, vz);
        if (L.pos[vt] < 0) b -= sg * xfixed(L, vt);
        return b;
    }
    const int r = id - 2 * nf - nfric, row = r >> 1, side = r & 1;
    return side ? (-P.ubA[row] + L.rowfix[row]) : (P.lbA[row] - L.rowfix[row]);
}

// slack n'x - b of constraint id evaluated by ONE lane (x read from the LDS mirror)
__device__ __forceinline__ double gi_cons_slack_lane(const GiCtx &C, int id) {
    const SolveProblem &P = *C.P;
    const GiLds &L = C.L;
    const int nf = C.nf, nfric = C.nfric;
    if (id < nf) return L.xs[id] - gi_cons_b(C, id);
    if (id < 2 * nf) return -L.xs[id - nf] - gi_cons_b(C, id);
    if (id < 2 * nf + nfric) {
        const int r = id - 2 * nf, ks = r >> 2, t = r & 3;
        const int k = ks / P.nfeet, sft = ks % P.nfeet;
        const int vz = k * P.nu + 3 * sft + 2, vt = k * P.nu + 3 * sft + (t >> 1);
        const double sg = (t & 1) ? 1.0 : -1.0;
        const int pz = L.pos[vz], pt = L.pos[vt];
        double s = 0.0;
        if (pz >= 0) s += P.mu * L.xs[pz];
        if (pt >= 0) s += sg * L.xs[pt];
        return s - gi_cons_b(C, id);
    }
    const int r = id - 2 * nf - nfric, row = r >> 1, side = r & 1;
    const double sg = side ? -1.0 : 1.0;
    double s = 0.0;
    for (int a = 0; a < nf; ++a) s += sg * rowA(P, row, L.fid[a]) * L.xs[a];
    return s - gi_cons_b(C, id);
}

// n'x of friction row id (id in [2nf, 2nf + nfric)) evaluated by ONE lane, without b: the
// register solver's sweep computes b once and subtracts it itself
__device__ __forceinline__ double gi_fric_nx_lane(const GiCtx &C, int id) {
    const SolveProblem &P = *C.P;
    const GiLds &L = C.L;
    const int r = id - 2 * C.nf, ks = r >> 2, t = r & 3;
    const int k = ks / P.nfeet, sft = ks % P.nfeet;
    const int pz = L.pos[k * P.nu + 3 * sft + 2], pt = L.pos[k * P.nu + 3 * sft + (t >> 1)];
    const double sg = (t & 1) ? 1.0 : -1.0;
    double s = 0.0;
    if (pz >= 0) s += P.mu * L.xs[pz];
    if (pt >= 0) s += sg * L.xs[pt];
    return s;
}

// d_j = (J' n_p)_j on lane j, and the slack n_p'x - b (uniform); x: lane i holds x_i
__device__ __forceinline__ void gi_cons_project(const GiCtx &C, int id, double x, double &dj, double &sp) {
    const SolveProblem &P = *C.P;
    const GiLds &L = C.L;
    const int nf = C.nf, nfric = C.nfric, ld = L.ld, ln = lane();
    const double b = gi_cons_b(C, id);
    dj = 0.0;
    if (id < 2 * nf) {
        const int a = id < nf ? id : id - nf;
        const double sg = id < nf ? 1.0 : -1.0;
        if (ln < nf) dj = sg * L.J[ln * ld + a];
        sp = sg * readlane(x, a) - b;
    } else if (id < 2 * nf + nfric) {
        const int r = id - 2 * nf, ks = r >> 2, t = r & 3;
        const int k = ks / P.nfeet, sft = ks % P.nfeet;
        const int pz = L.pos[k * P.nu + 3 * sft + 2], pt = L.pos[k * P.nu + 3 * sft + (t >> 1)];
        const double sg = (t & 1) ? 1.0 : -1.0;
        double nx_ = 0.0;
        if (pz >= 0) { if (ln < nf) dj += P.mu * L.J[ln * ld + pz]; nx_ += P.mu * readlane(x, pz); }
        if (pt >= 0) { if (ln < nf) dj += sg * L.J[ln * ld + pt]; nx_ += sg * readlane(x, pt); }
        sp = nx_ - b;
    } else {
        const int r = id - 2 * nf - nfric, row = r >> 1, side = r & 1;
        const double sg = side ? -1.0 : 1.0;
        double acc = 0.0, part = 0.0;
        for (int a = 0; a < nf; ++a) {
            const double na = sg * rowA(P, row, L.fid[a]);
            if (ln < nf) acc += L.J[ln * ld + a] * na;
        }
        for (int a = ln; a < nf; a += kWave) part += sg * rowA(P, row, L.fid[a]) * L.xs[a];
        dj = acc;
        sp = wave_sum(part) - b;
    }
}

// ---------------------------------------------------------------- stage 1: setup
// MPCQP_ELIDE_FZ: leave out a contact foot's fz lower bound that its friction pyramid implies
// (see gi_setup); 0 keeps it (A/B builds -- the oracle then needs p["elide_fz"] = 0)
#ifndef MPCQP_ELIDE_FZ
#define MPCQP_ELIDE_FZ 1
#endif
// Fixed variables, free index map, constraint states.  Leaves C.nf, C.mt, C.status.
__device__ __forceinline__ void gi_setup(GiCtx &C) {
    const SolveProblem &P = *C.P;
    GiLds &L = C.L;
    const int nV = P.nV, mA = P.mA, ln = lane(), nfmax = C.nfmax;
    C.nfric = P.friction ? 4 * P.N * P.nfeet : 0;
    C.status = ST_OK;
    C.c0 = 0.0;
    int nf = 0;
    for (int base = 0; base < nV; base += kWave) {
        const int v = base + ln;
        const bool valid = v < nV;
        double lo = -kInfty, hi = kInfty;
        if (valid) var_bounds(P, v, lo, hi);
        const bool bad = valid && lo > hi;
        const bool freev = valid && lo != hi;
        if (__any(bad)) C.status = ST_INFEASIBLE;
        const unsigned long long m = __ballot(freev);
        const int before = __popcll(m & ((1ull << ln) - 1ull));
        if (valid) {
            L.pos[v] = freev ? nf + before : -1;
            if (L.xfull) L.xfull[v] = freev ? 0.0 : lo;
            if (freev && nf + before < nfmax) L.fid[nf + before] = v;
        }
        nf += __popcll(m);
    }
    wave_sync();
    C.nf = nf;
    if (nf > nfmax || (!C.wide && nf > kWave)) C.status = ST_BAD_DIMS;
    const int nfric = C.nfric;
    const int mt = 2 * nf + nfric + 2 * mA;
    C.mt = mt;
    if (C.status != ST_OK) return;
    for (int id = ln; id < mt; id += kWave) {
        unsigned char s = 0;
        if (id < 2 * nf) {
            double lo, hi;
            const int v = L.fid[id < nf ? id : id - nf];
            var_bounds(P, v, lo, hi);
            s = (id < nf) ? (lo > -kInfty ? 1 : 0) : (hi < kInfty ? 1 : 0);
            // the lower bound fz >= lo <= 0 of a foot in contact is implied by its friction
            // pyramid (mu fz -+ fx >= 0 sum to fz >= 0 when mu > 0; at mu = 0 the rows only pin
            // fx, fy and the bound stays): left out, the same feasible set and
            // minimiser without the degenerate apex where five constraints meet in 3-D (the
            // dual loop's add / drop cycles there: config C's mean passes 5.9 -> 2.8 in the
            // oracle); the oracle does the same (orc_friction::elide_fz)
            if (MPCQP_ELIDE_FZ && id < nf && nfric > 0 && s == 1 && lo <= 0.0 && P.mu > 0.0) {
                const int k = v / P.nu, c = v % P.nu;
                if (c % 3 == 2 && c / 3 < P.nfeet && ((P.contact >> (2 * k + c / 3)) & 1ull)) s = 0;
            }
        } else if (id < 2 * nf + nfric) {
            const int r = id - 2 * nf, ks = r >> 2, t = r & 3;
            const int k = ks / P.nfeet, sft = ks % P.nfeet;
            if ((P.contact >> (2 * k + sft)) & 1ull) {
                const int vz = k * P.nu + 3 * sft + 2, vt = k * P.nu + 3 * sft + (t >> 1);
                const double sg = (t & 1) ? 1.0 : -1.0;
                if (L.pos[vz] >= 0 || L.pos[vt] >= 0) s = 1;
                else {
                    const double bb = -(P.mu * xfixed(L, vz) + sg * xfixed(L, vt));
                    if (bb > kFeasTol * (1.0 + fabs(bb))) s = 4;  // 0 >= b violated
                }
            }
        } else {
            const int r = id - 2 * nf - nfric, row = r >> 1, side = r & 1;
            const double lo = P.lbA ? P.lbA[row] : -kInfty, hi = P.ubA ? P.ubA[row] : kInfty;
            bool anyfree = false;
            double fix = 0.0;
            for (int v = 0; v < nV; ++v) {
                const double a = rowA(P, row, v);
                if (L.pos[v] >= 0) anyfree |= (a != 0.0);
                else fix += a * xfixed(L, v);
            }
            if (side == 0) L.rowfix[row] = fix;
            if (lo > hi) s = 4;
            else if (!anyfree) {
                bool ok = true;
                if (lo == hi) { const double bb = lo - fix; ok = fabs(bb) <= kFeasTol * (1.0 + fabs(bb)); }
                else if (side == 0 && lo > -kInfty) { const double bb = lo - fix; ok = !(bb > kFeasTol * (1.0 + fabs(bb))); }
                else if (side == 1 && hi < kInfty) { const double bb = fix - hi; ok = !(bb > kFeasTol * (1.0 + fabs(bb))); }
                s = ok ? 0 : 4;
            } else if (lo == hi) s = side == 0 ? 3 : 0;
            else if (side == 0) s = lo > -kInfty ? 1 : 0;
            else s = hi < kInfty ? 1 : 0;
        }
        L.st[id] = s;
    }
    wave_sync();
    bool infe = false;
    for (int id = ln; id < mt; id += kWave) infe |= (L.st[id] == 4);
    if (__any(infe)) C.status = ST_INFEASIBLE;
    if (L.cb) {  // b of the bound constraints, once (the dual loop's sweeps read it)
        for (int id = ln; id < 2 * nf; id += kWave) L.cb[id] = gi_cons_b(C, id);
        wave_sync();
    }
}

// ---------------------------------------------------------------- stage 2: gather
// H_FF (lower triangle suffices) into R, g = f_F + H_FB x_B, c0 = fixed-part objective.
__device__ __forceinline__ void gi_gather(GiCtx &C) {
    const SolveProblem &P = *C.P;
    GiLds &L = C.L;
    const int nV = P.nV, nf = C.nf, ld = L.ld, ln = lane();
    if (C.status != ST_OK) return;
    for (int b = 0; b < nf; ++b) {
        const int vb = L.fid[b];
        for (int a = ln; a < nf; a += kWave) L.R[b * ld + a] = P.H[(size_t)vb * nV + L.fid[a]];
    }
    for (int a = ln; a < nf; a += kWave) {
        const int va = L.fid[a];
        double s = P.f[va];
        for (int j = 0; j < nV; ++j)
            if (L.pos[j] < 0 && L.xfull[j] != 0.0) s += P.H[(size_t)j * nV + va] * L.xfull[j];
        L.g[a] = s;
    }
    double cl = 0.0;
    for (int i = ln; i < nV; i += kWave)
        if (L.pos[i] < 0 && L.xfull[i] != 0.0) {
            double s = 0.0;
            for (int j = 0; j < nV; ++j)
                if (L.pos[j] < 0) s += P.H[(size_t)j * nV + i] * L.xfull[j];
            cl += 0.5 * L.xfull[i] * s + P.f[i] * L.xfull[i];
        }
    C.c0 = wave_sum(cl);
    wave_sync();
}

// ---------------------------------------------------------------- stage 3: factor + loop
__device__ __forceinline__ void gi_run(GiCtx &C) {
    const SolveProblem &P = *C.P;
    GiLds &L = C.L;
    const int nf = C.nf, ld = L.ld, ln = lane(), mt = C.mt, nfric = C.nfric;
    double fval = 0.0, x = 0.0, u = 0.0;
    int iters = 0, q = 0, act = -1, eqs = 0;
    int status = C.status;
    MPCQP_STAMP_INIT(tst);

    if (status == ST_OK && nf > 0) {
        // Cholesky H_FF = L L' in place (lower), left-looking by column
        for (int k = 0; k < nf; ++k) {
            double piv = L.R[k * ld + k];
            for (int l = 0; l < k; ++l) piv -= L.R[l * ld + k] * L.R[l * ld + k];
            if (!(piv > 0.0)) { status = ST_NOT_PD; break; }
            const double lkk = sqrt(piv);
            for (int i = k + 1 + ln; i < nf; i += kWave) {
                double s = L.R[k * ld + i];
                for (int l = 0; l < k; ++l) s -= L.R[l * ld + i] * L.R[l * ld + k];
                L.R[k * ld + i] = s / lkk;
            }
            wave_sync();
            if (ln == 0) L.R[k * ld + k] = lkk;
            wave_sync();
        }
    } else if (status == ST_OK) {
        // nothing free: cost of the fixed point only
        const int nV = P.nV;
        double cl = 0.0;
        if (P.H)
            for (int i = ln; i < nV; i += kWave) {
                double s = 0.0;
                for (int j = 0; j < nV; ++j) s += P.H[(size_t)j * nV + i] * L.xfull[j];
                cl += 0.5 * L.xfull[i] * s + P.f[i] * L.xfull[i];
            }
        C.c0 = wave_sum(cl);
    }
    MPCQP_STAMP(C.stamps, 5, tst); MPCQP_CUT(C.cut, 4);

    if (status == ST_OK && nf > 0) {
        // J = L^-T: lane c computes column c of L^-1 and stores Linv(i, c) at J[i*ld + c],
        // which is J(c, i) in column-major order.
        for (int c = ln; c < nf; c += kWave) {
            for (int i = 0; i < c; ++i) L.J[i * ld + c] = 0.0;
            for (int i = c; i < nf; ++i) {
                double s = (i == c) ? 1.0 : 0.0;
                for (int l = c; l < i; ++l) s -= L.R[l * ld + i] * L.J[l * ld + c];
                L.J[i * ld + c] = s / L.R[i * ld + i];
            }
        }
        wave_sync();
        MPCQP_STAMP(C.stamps, 6, tst); MPCQP_CUT(C.cut, 5);
        // unconstrained minimum x = -J J' g
        double w = 0.0;
        if (ln < nf)
            for (int i = 0; i < nf; ++i) w += L.J[ln * ld + i] * L.g[i];
        double s = 0.0;
        for (int j = 0; j < nf; ++j) {
            const double wj = readlane(w, j);
            if (ln < nf) s += L.J[j * ld + ln] * wj;
        }
        x = (ln < nf) ? -s : 0.0;
        fval = wave_sum((ln < nf) ? 0.5 * L.g[ln] * x : 0.0);
        if (ln < nf) L.xs[ln] = x;
        wave_sync();
    }
    MPCQP_STAMP(C.stamps, 7, tst); MPCQP_CUT(C.cut, 6);

    const int max_iter = P.max_iter > 0 ? P.max_iter : 10 * (mt + nf + 1);
    int eq_next = 2 * nf + nfric;  // dense rows are the only equality candidates
    bool done = (status != ST_OK) || nf == 0;
    while (!done) {
        // ---- step 1: the constraint to add (pending equalities first, in row order)
        int p = -1;
        double sp = 0.0;
        bool adding_eq = false;
        while (eq_next < mt && L.st[eq_next] != 3) eq_next += 1;
        if (eq_next < mt) {
            p = eq_next;
            eq_next += 1;
            adding_eq = true;
        } else {
            double best = INFINITY;
            int bid = 0x7fffffff;
            for (int id = ln; id < mt; id += kWave) {
                if (L.st[id] != 1) continue;
                const double s = gi_cons_slack_lane(C, id);
                const double key = gi_sel_key(s, C.nfric > 0 && P.contact != 0ull);
                if (s < -kFeasTol * (1.0 + fabs(gi_cons_b(C, id))) && key < best) { best = key; bid = id; }
            }
            wave_argmin(best, bid);
            if (bid == 0x7fffffff) break;  // optimal
            p = bid;
        }
        double dj;
        gi_cons_project(C, p, x, dj, sp);
        if (ln == q) u = 0.0;
        // ---- step 2
        for (;;) {
            if (iters >= max_iter) { status = ST_ITER_LIMIT; done = true; break; }
            ++iters;
            double dd = ln < nf ? dj * dj : 0.0;
            double zn = (ln >= q && ln < nf) ? dj * dj : 0.0;
            wave_sum2(dd, zn);
            // z = J(:, q:) d(q:)   (lane i)
            double z = 0.0;
            for (int j = q; j < nf; ++j) {
                const double dv = readlane(dj, j);
                if (ln < nf) z += L.J[j * ld + ln] * dv;
            }
            // r = R^-1 d(0:q)   (back substitution; lane j ends with r_j)
            double r = 0.0, val = dj;
            for (int j = q - 1; j >= 0; --j) {
                const double rj = readlane(val, j) / L.R[j * ld + j];
                if (ln == j) r = rj;
                if (ln < j) val -= L.R[j * ld + ln] * rj;
            }
            const double rmax = wave_max(ln < q ? fabs(r) : 0.0);
            double t1 = INFINITY;
            int kslot = 0x7fffffff;
            if (!adding_eq && ln < q && !eqs && r > kRTol * rmax) { t1 = u / r; kslot = ln; }
            wave_argmin(t1, kslot);
            const bool dep = !(zn > kDepTol * dd);
            if (adding_eq && dep) {
                const double bp = gi_cons_b(C, p);
                if (fabs(sp) <= kFeasTol * (1.0 + fabs(bp))) break;  // consistent: skip
                status = ST_INFEASIBLE; done = true; break;
            }
            const double t2 = dep ? INFINITY : -sp / zn;
            const double t = t1 < t2 ? t1 : t2;
            if (isinf(t)) { status = ST_INFEASIBLE; done = true; break; }
            const double uq = readlane(u, q);
            if (isinf(t2)) {
                if (ln < q) u -= t * r;
                if (ln == q) u += t;
            } else {
                if (ln < nf) { x += t * z; L.xs[ln] = x; }
                fval += t * zn * (0.5 * t + uq);
                if (ln < q) u -= t * r;
                if (ln == q) u += t;
                if (t2 <= t1) {
                    // ---- full step: add p.  Givens chain on d from the bottom up to q+1.
                    double cj = 1.0, sj = 0.0;  // lane j keeps the rotation of pair (j-1, j)
                    double acc = readlane(dj, nf - 1);
                    for (int j = nf - 1; j > q; --j) {
                        const double a = readlane(dj, j - 1);
                        double c = 1.0, s = 0.0, h = a;
                        if (acc != 0.0) {
                            h = sqrt(a * a + acc * acc);
                            c = a / h;
                            s = acc / h;
                        }
                        if (ln == j) { cj = c; sj = s; }
                        acc = h;
                    }
                    const double rqq = (q < nf - 1) ? acc : readlane(dj, q);
                    double carry = (ln < nf) ? L.J[(nf - 1) * ld + ln] : 0.0;
                    for (int j = nf - 1; j > q; --j) {
                        const double c = readlane(cj, j), s = readlane(sj, j);
                        if (ln < nf) {
                            const double a = L.J[(j - 1) * ld + ln];
                            L.J[j * ld + ln] = -s * a + c * carry;
                            carry = c * a + s * carry;
                        }
                    }
                    if (ln < nf) L.J[q * ld + ln] = carry;
                    if (ln < q) L.R[q * ld + ln] = dj;
                    if (ln == q) { L.R[q * ld + q] = rqq; act = p; eqs = adding_eq ? 1 : 0; }
                    if (ln == 0) L.st[p] = adding_eq ? 3 : 2;
                    ++q;
                    wave_sync();
                    break;  // back to step 1
                }
            }
            // ---- drop slot kslot (uniform)
            const int k = kslot;
            const int dropped = readlane(act, k);
            if (ln == 0) L.st[dropped] = 1;
            {
                const int src = ln + 1 < kWave ? ln + 1 : ln;
                const double un = __shfl(u, src, kWave);
                const int an = __shfl(act, src, kWave);
                const int en = __shfl(eqs, src, kWave);
                if (ln >= k && ln < q) { u = un; act = an; eqs = en; }
            }
            // shift R columns k+1..q-1 left by one (rows 0..j+1)
            for (int j = k; j < q - 1; ++j) {
                const double v = (ln <= j + 1) ? L.R[(j + 1) * ld + ln] : 0.0;
                wave_sync();
                if (ln <= j + 1) L.R[j * ld + ln] = v;
                wave_sync();
            }
            --q;
            // restore triangularity with Givens on rows (j, j+1), also applied to J columns
            for (int j = k; j < q; ++j) {
                const double a = L.R[j * ld + j], bb = L.R[j * ld + j + 1];
                if (bb == 0.0) continue;
                const double h = sqrt(a * a + bb * bb);
                const double c = a / h, s = bb / h;
                const int l = j + 1 + ln;
                double r0 = 0.0, r1 = 0.0;
                if (l < q) { r0 = L.R[l * ld + j]; r1 = L.R[l * ld + j + 1]; }
                double j0 = 0.0, j1 = 0.0;
                if (ln < nf) { j0 = L.J[j * ld + ln]; j1 = L.J[(j + 1) * ld + ln]; }
                wave_sync();
                if (l < q) { L.R[l * ld + j] = c * r0 + s * r1; L.R[l * ld + j + 1] = -s * r0 + c * r1; }
                if (ln < nf) { L.J[j * ld + ln] = c * j0 + s * j1; L.J[(j + 1) * ld + ln] = -s * j0 + c * j1; }
                if (ln == 0) { L.R[j * ld + j] = h; L.R[j * ld + j + 1] = 0.0; }
                wave_sync();
            }
            // p remains the target: refresh d and its slack
            gi_cons_project(C, p, x, dj, sp);
        }
    }
    MPCQP_STAMP(C.stamps, 8, tst); MPCQP_CUT(C.cut, 7);
    C.status = status;
    C.x = x;
    C.u = u;
    C.fval = fval;
    C.act = act;
    C.q = q;
    C.iters = iters;
}

// ---------------------------------------------------------------- stage 4: outputs
__device__ __forceinline__ void gi_write(GiCtx &C, const SolveOut &O) {
    const SolveProblem &P = *C.P;
    GiLds &L = C.L;
    const int nV = P.nV, mA = P.mA, nf = C.nf, ln = lane(), nfric = C.nfric;
    const bool have_map = nf <= C.nfmax && nf <= kWave;
    double *xo = O.stage ? O.stage : O.x;
    if (O.stage) wave_sync();
    for (int v = ln; v < nV; v += kWave) {
        const int pv = L.pos[v];
        if (pv < 0 || !have_map) xo[v] = (pv < 0) ? xfixed(L, v) : 0.0;
    }
    if (have_map && ln < nf) xo[L.fid[ln]] = C.x;
    if (O.stage) {
        wave_sync();
        for (int v = ln; v < nV; v += kWave) stream_store(O.x + v, O.stage[v]);
    }
    if (ln == 0) {
        stream_store(O.cost, C.fval + C.c0);
        stream_store(O.status, C.status);
        stream_store(O.iters, C.iters);
    }
    if (O.y) {
        // multipliers: y_b (nV) then y_A (mA) with H x + f = y_b + A' y_A, built in LDS
        for (int v = ln; v < nV + mA; v += kWave) L.ys[v] = 0.0;
        if (L.xfull && have_map && ln < nf) L.xfull[L.fid[ln]] = C.x;  // full primal in LDS
        wave_sync();
        if (C.status == ST_OK && ln < C.q) {
            const int id = C.act;
            const double u = C.u;
            if (id < nf) L.ys[L.fid[id]] = u;
            else if (id < 2 * nf) L.ys[L.fid[id - nf]] = -u;
            else if (id >= 2 * nf + nfric) {
                const int r = id - 2 * nf - nfric;
                L.ys[nV + (r >> 1)] = (r & 1) ? -u : u;
            }
        }
        wave_sync();
        for (int v = ln; v < nV; v += kWave)
            if (L.pos[v] < 0) {  // fixed variables: the remaining gradient
                double s = P.f[v];
                for (int j = 0; j < nV; ++j) s += P.H[(size_t)j * nV + v] * L.xfull[j];
                for (int r2 = 0; r2 < mA; ++r2) s -= rowA(P, r2, v) * L.ys[nV + r2];
                L.ys[v] = s;
            }
        wave_sync();
        for (int v = ln; v < nV + mA; v += kWave) O.y[v] = L.ys[v];
    }
}

// Stand-alone solve of one instance from H, f in global memory (LDS: gi_lds_bytes).
__device__ __forceinline__ void wave_gi_solve(const SolveProblem &P, const SolveOut &O,
                                     unsigned char *smem, int nfmax) {
    GiCtx C;
    C.wide = 0;
    C.stamps = nullptr;
    C.cut = 0;
    C.P = &P;
    C.L = gi_carve(smem, nfmax, P.nV, P.mA);
    C.nfmax = nfmax;
    gi_setup(C);
    gi_gather(C);
    gi_run(C);
    gi_write(C, O);
}

}  // namespace mpcqp
