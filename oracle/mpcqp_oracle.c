/*
 * mpcqp_oracle.c -- CPU restatement of the reference MPC-QP hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see mpcqp_oracle.h): the parity oracle for the HIP path and the
 * timed CPU baseline (kind "port").  Never linked into the product library.
 *
 * Parity: unpinned w.r.t. the reference binary (unbuildable here: Eigen/qpOASES absent, no
 * reference fixtures exist).  Cross-checked against an independent numpy/scipy restatement
 * and the SURVEY.md section 8c known-answer values -- see tests/golden/.
 *
 * Compiled with -ffp-contract=off so every rounding is the one written here.
 */
#include "mpcqp_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define IDX(i, j, ld) ((size_t)(j) * (size_t)(ld) + (size_t)(i))

/* ---------------------------------------------------------------- small dense helpers */
/* C(m x n) = A(m x k) * B(k x n), all column-major, C must not alias A or B */
static void mm(int m, int k, int n, const double *A, const double *B, double *C) {
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < m; ++i) {
            double s = 0.0;
            for (int l = 0; l < k; ++l) s += A[IDX(i, l, m)] * B[IDX(l, j, k)];
            C[IDX(i, j, m)] = s;
        }
}

static void eye(int n, double *A) {
    memset(A, 0, sizeof(double) * (size_t)n * n);
    for (int i = 0; i < n; ++i) A[IDX(i, i, n)] = 1.0;
}

/* solve A X = B in place of B (A n x n destroyed), Gaussian elimination with partial
 * pivoting -- the algorithm of Eigen's PartialPivLU::solve (max-|.| pivot per column). */
static int lu_solve(int n, double *A, int nrhs, double *B) {
    for (int k = 0; k < n; ++k) {
        int p = k;
        double amax = fabs(A[IDX(k, k, n)]);
        for (int i = k + 1; i < n; ++i) {
            double v = fabs(A[IDX(i, k, n)]);
            if (v > amax) { amax = v; p = i; }
        }
        if (amax == 0.0) return -1;
        if (p != k) {
            for (int j = 0; j < n; ++j) {
                double t = A[IDX(k, j, n)]; A[IDX(k, j, n)] = A[IDX(p, j, n)]; A[IDX(p, j, n)] = t;
            }
            for (int j = 0; j < nrhs; ++j) {
                double t = B[IDX(k, j, n)]; B[IDX(k, j, n)] = B[IDX(p, j, n)]; B[IDX(p, j, n)] = t;
            }
        }
        const double piv = A[IDX(k, k, n)];
        for (int i = k + 1; i < n; ++i) {
            const double l = A[IDX(i, k, n)] / piv;
            A[IDX(i, k, n)] = l;
            for (int j = k + 1; j < n; ++j) A[IDX(i, j, n)] -= l * A[IDX(k, j, n)];
            for (int j = 0; j < nrhs; ++j) B[IDX(i, j, n)] -= l * B[IDX(k, j, n)];
        }
    }
    for (int j = 0; j < nrhs; ++j)
        for (int i = n - 1; i >= 0; --i) {
            double s = B[IDX(i, j, n)];
            for (int l = i + 1; l < n; ++l) s -= A[IDX(i, l, n)] * B[IDX(l, j, n)];
            B[IDX(i, j, n)] = s / A[IDX(i, i, n)];
        }
    return 0;
}

/* ------------------------------------------------ matrix exponential (Eigen 3.3 algorithm)
 * Restates Eigen/unsupported MatrixExponential for double: Pade degree by the 1-norm of the
 * argument (thresholds of Higham 2005 as tabulated by Eigen), degree 13 with scaling by
 * frexp(norm/5.371920351148152) squarings.  Used by QPSolver::discretizeSystem
 * (src/QPSolver.cpp:26) and linear_mpc_example (src/linear_mpc_example.cpp:37). */
static void lincomb(int nn, double *out, const double *c, const double *const *M, int cnt,
                    double cI, int n) {
    for (int t = 0; t < nn; ++t) {
        double s = 0.0;
        for (int q = 0; q < cnt; ++q) s += c[q] * M[q][t];
        out[t] = s;
    }
    if (cI != 0.0)
        for (int i = 0; i < n; ++i) out[IDX(i, i, n)] += cI;
}

int orc_expm(int n, const double *Ain, double *E) {
    const int nn = n * n;
    double *A = malloc(sizeof(double) * nn * 8);
    if (!A) return -1;
    double *A2 = A + nn, *A4 = A2 + nn, *A6 = A4 + nn, *A8 = A6 + nn, *U = A8 + nn,
           *V = U + nn, *T = V + nn;
    memcpy(A, Ain, sizeof(double) * nn);

    double l1 = 0.0;
    for (int j = 0; j < n; ++j) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += fabs(A[IDX(i, j, n)]);
        if (s > l1) l1 = s;
    }
    int squarings = 0;
    if (l1 < 1.495585217958292e-002) { /* pade3 */
        const double b[] = {120., 60., 12., 1.};
        mm(n, n, n, A, A, A2);
        const double *M1[] = {A2};
        const double c1[] = {b[3]};
        lincomb(nn, T, c1, M1, 1, b[1], n);
        mm(n, n, n, A, T, U);
        const double c2[] = {b[2]};
        lincomb(nn, V, c2, M1, 1, b[0], n);
    } else if (l1 < 2.539398330063230e-001) { /* pade5 */
        const double b[] = {30240., 15120., 3360., 420., 30., 1.};
        mm(n, n, n, A, A, A2);
        mm(n, n, n, A2, A2, A4);
        const double *M2[] = {A4, A2};
        const double c1[] = {b[5], b[3]};
        lincomb(nn, T, c1, M2, 2, b[1], n);
        mm(n, n, n, A, T, U);
        const double c2[] = {b[4], b[2]};
        lincomb(nn, V, c2, M2, 2, b[0], n);
    } else if (l1 < 9.504178996162932e-001) { /* pade7 */
        const double b[] = {17297280., 8648640., 1995840., 277200., 25200., 1512., 56., 1.};
        mm(n, n, n, A, A, A2);
        mm(n, n, n, A2, A2, A4);
        mm(n, n, n, A4, A2, A6);
        const double *M3[] = {A6, A4, A2};
        const double c1[] = {b[7], b[5], b[3]};
        lincomb(nn, T, c1, M3, 3, b[1], n);
        mm(n, n, n, A, T, U);
        const double c2[] = {b[6], b[4], b[2]};
        lincomb(nn, V, c2, M3, 3, b[0], n);
    } else if (l1 < 2.097847961257068e+000) { /* pade9 */
        const double b[] = {17643225600., 8821612800., 2075673600., 302702400., 30270240.,
                            2162160.,     110880.,     3960.,       90.,        1.};
        mm(n, n, n, A, A, A2);
        mm(n, n, n, A2, A2, A4);
        mm(n, n, n, A4, A2, A6);
        mm(n, n, n, A6, A2, A8);
        const double *M4[] = {A8, A6, A4, A2};
        const double c1[] = {b[9], b[7], b[5], b[3]};
        lincomb(nn, T, c1, M4, 4, b[1], n);
        mm(n, n, n, A, T, U);
        const double c2[] = {b[8], b[6], b[4], b[2]};
        lincomb(nn, V, c2, M4, 4, b[0], n);
    } else { /* pade13 with scaling */
        const double maxnorm = 5.371920351148152;
        frexp(l1 / maxnorm, &squarings);
        if (squarings < 0) squarings = 0;
        for (int t = 0; t < nn; ++t) A[t] = ldexp(A[t], -squarings);
        const double b[] = {64764752532480000., 32382376266240000., 7771770303897600.,
                            1187353796428800.,  129060195264000.,   10559470521600.,
                            670442572800.,      33522128640.,       1323241920.,
                            40840800.,          960960.,            16380.,
                            182.,               1.};
        mm(n, n, n, A, A, A2);
        mm(n, n, n, A2, A2, A4);
        mm(n, n, n, A4, A2, A6);
        const double *M3[] = {A6, A4, A2};
        const double c1[] = {b[13], b[11], b[9]};
        lincomb(nn, V, c1, M3, 3, 0.0, n);
        mm(n, n, n, A6, V, T);
        const double c2[] = {b[7], b[5], b[3]};
        lincomb(nn, A8, c2, M3, 3, b[1], n); /* A8 reused as scratch */
        for (int t = 0; t < nn; ++t) T[t] += A8[t];
        mm(n, n, n, A, T, U);
        const double c3[] = {b[12], b[10], b[8]};
        lincomb(nn, T, c3, M3, 3, 0.0, n);
        mm(n, n, n, A6, T, V);
        const double c4[] = {b[6], b[4], b[2]};
        lincomb(nn, A8, c4, M3, 3, b[0], n);
        for (int t = 0; t < nn; ++t) V[t] += A8[t];
    }
    /* numer = U + V; denom = -U + V; result = denom.partialPivLu().solve(numer) */
    for (int t = 0; t < nn; ++t) {
        E[t] = U[t] + V[t];
        T[t] = -U[t] + V[t];
    }
    int rc = lu_solve(n, T, n, E);
    for (int s = 0; s < squarings; ++s) {
        mm(n, n, n, E, E, A2);
        memcpy(E, A2, sizeof(double) * nn);
    }
    free(A);
    return rc;
}

/* Eigen MatrixPower<...>::computeIntPower for a non-negative integer exponent:
 * res = I; tmp = A; while(true){ if (fmod(pp,2) >= 1) res = tmp*res; pp /= 2; if (pp<1) break;
 * tmp *= tmp; }   (used by Ad.pow(k), src/QPSolver.cpp:45,75) */
void orc_matpow(int n, const double *A, int p, double *out) {
    const int nn = n * n;
    double *tmp = malloc(sizeof(double) * nn * 2);
    double *w = tmp + nn;
    eye(n, out);
    memcpy(tmp, A, sizeof(double) * nn);
    double pp = fabs((double)p);
    while (1) {
        if (fmod(pp, 2.0) >= 1.0) {
            mm(n, n, n, tmp, out, w);
            memcpy(out, w, sizeof(double) * nn);
        }
        pp /= 2.0;
        if (pp < 1.0) break;
        mm(n, n, n, tmp, tmp, w);
        memcpy(tmp, w, sizeof(double) * nn);
    }
    free(tmp);
}

/* QPSolver::discretizeSystem, src/QPSolver.cpp:21-29:
 *   M = [[Ac, Bc],[0, 0]];  expM = (M*Ts).exp();  Ad = expM[0:NX,0:NX];  Bd = expM[0:NX,NX:] */
int orc_discretize(int nx, int nu, double Ts, const double *Ac, const double *Bc, double *Ad,
                   double *Bd) {
    if (nx <= 0 || nu <= 0) return ORC_BAD_DIMS;
    const int n = nx + nu;
    double *M = calloc((size_t)n * n * 2, sizeof(double));
    double *E = M + n * n;
    for (int j = 0; j < nx; ++j)
        for (int i = 0; i < nx; ++i) M[IDX(i, j, n)] = Ac[IDX(i, j, nx)] * Ts;
    for (int j = 0; j < nu; ++j)
        for (int i = 0; i < nx; ++i) M[IDX(i, nx + j, n)] = Bc[IDX(i, j, nx)] * Ts;
    int rc = orc_expm(n, M, E);
    for (int j = 0; j < nx; ++j)
        for (int i = 0; i < nx; ++i) Ad[IDX(i, j, nx)] = E[IDX(i, j, n)];
    for (int j = 0; j < nu; ++j)
        for (int i = 0; i < nx; ++i) Bd[IDX(i, j, nx)] = E[IDX(i, nx + j, n)];
    free(M);
    return rc ? ORC_NOT_PD : ORC_OK;
}

/* linear_mpc_example's discretizeSystem, src/linear_mpc_example.cpp:35-46:
 *   Ad = (A*Ts).exp();  Bd = sum_{i<100} Ad * (I - A*tau/steps)^-1 * Bc * (Ts/steps),
 *   tau = i*Ts/steps   (an approximate quadrature; kept verbatim, including its 1/steps^2) */
int orc_discretize_quadrature(int nx, int nu, double Ts, const double *Ac, const double *Bc,
                              double *Ad, double *Bd) {
    const int steps = 100;
    const int nn = nx * nx;
    double *M = malloc(sizeof(double) * (nn * 3 + nx * nu * 2));
    double *Minv = M + nn, *W = Minv + nn, *T1 = W + nn, *T2 = T1 + nx * nu;
    for (int t = 0; t < nn; ++t) M[t] = Ac[t] * Ts;
    orc_expm(nx, M, Ad);
    memset(Bd, 0, sizeof(double) * nx * nu);
    for (int i = 0; i < steps; ++i) {
        const double tau = i * Ts / steps;
        for (int t = 0; t < nn; ++t) W[t] = -Ac[t] * tau / steps;
        for (int d = 0; d < nx; ++d) W[IDX(d, d, nx)] += 1.0;
        eye(nx, Minv);
        lu_solve(nx, W, nx, Minv);
        mm(nx, nx, nu, Minv, Bc, T1);
        mm(nx, nx, nu, Ad, T1, T2);
        for (int t = 0; t < nx * nu; ++t) Bd[t] += T2[t] * (Ts / steps);
    }
    free(M);
    return ORC_OK;
}

/* QPSolver::buildQPParams, src/QPSolver.cpp:31-81, restated with the reference's exact
 * output layouts (column-major):
 *   A_aug (NX(N+1) x NX): block i = Ad * block i-1                         (:36-40)
 *   B_aug (NX(N+1) x NU N): block (i,j) = Ad.pow(i-j-1) * Bd, j < i        (:42-47)
 *   Q_bar = blkdiag(Q x N, P), R_bar = blkdiag(R x N)                       (:50-56)
 *   H = 2 (B_aug' Q_bar B_aug + R_bar)                                      (:58)
 *   f = 2 B_aug' Q_bar (A_aug xi0 - vec(xi_ref))                            (:59-60)
 *   A_eq = B_aug.bottomRows(NX N), b_eq = A_aug.bottomRows(NX N) xi0        (:63-64)
 *   lb = u_min, ub = u_max                                                  (:67-68)
 *   A_ineq (2 NX N x NU N), rows 2 i NX.. = B_aug block row i+1, others 0;
 *   lbA/ubA = x_min/x_max - Ad.pow(i+1) xi0 on filled rows, -/+INFTY else  (:71-80) */
int orc_build_qp(int NX, int NU, int N, const double *Ad, const double *Bd, const double *Q,
                 const double *R, const double *P, const double *x_min, const double *x_max,
                 double u_min, double u_max, const double *xi0, const double *xi_ref, double *H,
                 double *f, double *A_eq, double *b_eq, double *lb, double *ub, double *A_ineq,
                 double *lbA, double *ubA) {
    if (NX <= 0 || NU <= 0 || N <= 0) return ORC_BAD_DIMS;
    const int XB = NX * (N + 1), nV = NU * N;
    double *Aaug = calloc((size_t)XB * NX, sizeof(double));
    double *Baug = calloc((size_t)XB * nV, sizeof(double));
    double *Qbar = calloc((size_t)XB * XB, sizeof(double));
    double *T = calloc((size_t)nV * XB, sizeof(double));
    double *pw = malloc(sizeof(double) * NX * NX);
    double *blk = malloc(sizeof(double) * NX * (NX > NU ? NX : NU));
    double *v = malloc(sizeof(double) * XB);

    for (int d = 0; d < NX; ++d) Aaug[IDX(d, d, XB)] = 1.0;
    for (int i = 1; i <= N; ++i)
        for (int c = 0; c < NX; ++c)
            for (int r = 0; r < NX; ++r) {
                double s = 0.0;
                for (int l = 0; l < NX; ++l)
                    s += Ad[IDX(r, l, NX)] * Aaug[IDX((i - 1) * NX + l, c, XB)];
                Aaug[IDX(i * NX + r, c, XB)] = s;
            }
    for (int i = 1; i <= N; ++i)
        for (int j = 0; j < i; ++j) {
            orc_matpow(NX, Ad, i - j - 1, pw);
            mm(NX, NX, NU, pw, Bd, blk);
            for (int c = 0; c < NU; ++c)
                for (int r = 0; r < NX; ++r)
                    Baug[IDX(i * NX + r, j * NU + c, XB)] = blk[IDX(r, c, NX)];
        }
    for (int i = 0; i < N; ++i)
        for (int c = 0; c < NX; ++c)
            for (int r = 0; r < NX; ++r) Qbar[IDX(i * NX + r, i * NX + c, XB)] = Q[IDX(r, c, NX)];
    for (int c = 0; c < NX; ++c)
        for (int r = 0; r < NX; ++r) Qbar[IDX(N * NX + r, N * NX + c, XB)] = P[IDX(r, c, NX)];

    /* T = B_aug' * Q_bar  (nV x XB) */
    for (int c = 0; c < XB; ++c)
        for (int r = 0; r < nV; ++r) {
            double s = 0.0;
            for (int l = 0; l < XB; ++l) s += Baug[IDX(l, r, XB)] * Qbar[IDX(l, c, XB)];
            T[IDX(r, c, nV)] = s;
        }
    /* H = 2 * (T * B_aug + R_bar) */
    for (int c = 0; c < nV; ++c)
        for (int r = 0; r < nV; ++r) {
            double s = 0.0;
            for (int l = 0; l < XB; ++l) s += T[IDX(r, l, nV)] * Baug[IDX(l, c, XB)];
            double rb = 0.0;
            if (r / NU == c / NU) rb = R[IDX(r % NU, c % NU, NU)];
            H[IDX(r, c, nV)] = 2.0 * (s + rb);
        }
    /* v = A_aug * xi0 - vec(xi_ref);  f = 2 * T * v */
    for (int r = 0; r < XB; ++r) {
        double s = 0.0;
        for (int l = 0; l < NX; ++l) s += Aaug[IDX(r, l, XB)] * xi0[l];
        v[r] = s - xi_ref[r];
    }
    for (int r = 0; r < nV; ++r) {
        double s = 0.0;
        for (int l = 0; l < XB; ++l) s += 2.0 * T[IDX(r, l, nV)] * v[l];
        f[r] = s;
    }
    const int NE = NX * N;
    if (A_eq)
        for (int c = 0; c < nV; ++c)
            for (int r = 0; r < NE; ++r) A_eq[IDX(r, c, NE)] = Baug[IDX(NX + r, c, XB)];
    if (b_eq)
        for (int r = 0; r < NE; ++r) {
            double s = 0.0;
            for (int l = 0; l < NX; ++l) s += Aaug[IDX(NX + r, l, XB)] * xi0[l];
            b_eq[r] = s;
        }
    if (lb)
        for (int r = 0; r < nV; ++r) lb[r] = u_min;
    if (ub)
        for (int r = 0; r < nV; ++r) ub[r] = u_max;
    const int NI = 2 * NX * N;
    if (A_ineq) memset(A_ineq, 0, sizeof(double) * (size_t)NI * nV);
    if (lbA)
        for (int r = 0; r < NI; ++r) lbA[r] = -ORC_INFTY;
    if (ubA)
        for (int r = 0; r < NI; ++r) ubA[r] = ORC_INFTY;
    for (int i = 0; i < N; ++i) {
        if (A_ineq)
            for (int c = 0; c < nV; ++c)
                for (int r = 0; r < NX; ++r)
                    A_ineq[IDX(2 * i * NX + r, c, NI)] = Baug[IDX((i + 1) * NX + r, c, XB)];
        if (lbA || ubA) {
            orc_matpow(NX, Ad, i + 1, pw);
            for (int r = 0; r < NX; ++r) {
                double s = 0.0;
                for (int l = 0; l < NX; ++l) s += pw[IDX(r, l, NX)] * xi0[l];
                if (lbA) lbA[2 * i * NX + r] = x_min[r] - s;
                if (ubA) ubA[2 * i * NX + r] = x_max[r] - s;
            }
        }
    }
    free(Aaug); free(Baug); free(Qbar); free(T); free(pw); free(blk); free(v);
    return ORC_OK;
}

/* QPSolver::updateState, src/QPSolver.cpp:108-111:  xi = Ad*xi + Bd*u */
void orc_plant_step(int nx, int nu, const double *Ad, const double *Bd, double *x,
                    const double *u) {
    double y[64];
    for (int r = 0; r < nx; ++r) {
        double s = 0.0;
        for (int l = 0; l < nx; ++l) s += Ad[IDX(r, l, nx)] * x[l];
        double t = 0.0;
        for (int l = 0; l < nu; ++l) t += Bd[IDX(r, l, nx)] * u[l];
        y[r] = s + t;
    }
    memcpy(x, y, sizeof(double) * nx);
}

/* ---------------------------------------------------------------- dense QP: Goldfarb-Idnani
 * The reference hands its QP to qpOASES (src/QPSolver.cpp:87-104).  As handed over that QP is
 * infeasible; the corrected QP (bounds + A_ineq rows, row-major, no A_eq) is
 * strictly convex, so its optimum is unique and solver-independent.  Both this oracle and
 * the GPU solve it with the Goldfarb-Idnani (1983) dual active-set method on the free
 * variables (lb == ub variables eliminated), in the J = L^-T Q / R factored form, with the
 * same constraint ordering and tolerances:
 *   constraint ids: [lower bounds (free pos)] [upper bounds] [friction (k,s,t)] [rows (r,side)]
 *   most-violated selection, ties -> lowest id.                                           */
#define GI_FEAS_TOL 1e-11 /* violation threshold, relative to (1 + |b|)               */
#define GI_DEP_TOL 1e-20  /* |d2|^2 <= tol*|d|^2  => n_p linearly dependent (z = 0)   */
#define GI_R_TOL 1e-12    /* r_j > tol * max|r|  counts as a blocking multiplier       */

typedef struct {
    int n, m;     /* free vars, one-sided constraints */
    double *N;    /* m x n normals, row-major (normal of c at N + c*n) */
    double *b;    /* m */
    int *is_eq;   /* m */
    int *src;     /* m: original constraint id (see ordering above) */
    int qsel;     /* friction rows present: selection keys quantized (gi_sel_key) */
} gi_cons;

/* The most-violated selection's key when the QP has friction rows: the violation with its low
 * 20 mantissa bits cleared, so violations within ~2^-32 relative tie and the lowest id wins, as
 * for exact ties.  A pyramid's +- rows are exactly tied whenever the tangential force is zero
 * (symmetric commands), and rounding alone would otherwise pick one of them -- differently in
 * the library's solvers and here (same minimiser, different pass counts).  The library's
 * one-wave and workgroup solvers use the same key (gi_sel_key, gi_solver.hpp). */
static double gi_sel_key(double s) {
    uint64_t u;
    memcpy(&u, &s, sizeof u);
    u &= ~(uint64_t)0xFFFFF;
    memcpy(&s, &u, sizeof u);
    return s;
}

/* Speculative primal-dual active-set start for problems whose constraints are all bounds (the
 * GPU kernels' "crash").  From the unconstrained minimum x0 (H^-1 = J J'):
 * the working set A starts as every violated bound (at most kmax: the ones already active, then
 * the lowest variable ids); the minimiser with A's bounds as equalities is
 *   x = x0 - J J_A' w,   M w = x0_A - b_A,   M = J_A J_A' = (H^-1)_AA,
 * M solved by Gauss-Jordan without pivoting (M is positive definite), multipliers
 * lambda_a = -side_a w_a, f = f0 + w'(x0_A - b_A) / 2.  The next working set drops the
 * negative multipliers and adds the bounds x violates (GI_FEAS_TOL, as the dual loop's test);
 * an unchanged set is the optimum of the strictly convex QP (KKT within the tolerance), the
 * same point the dual active-set loop reaches.  Gives up (returns 0, x / fval untouched) after
 * pmax working sets or a non-positive pivot: the caller then runs Goldfarb-Idnani from x0.
 * *solves counts the working sets that needed a solve (the reported iterations). */
/* Solver flops of the instance being solved on this thread (orc_srbm_batch's sflops output),
 * counted the textbook way per working-set solve and per dual pass -- the same formulas the
 * paired kernel's diagnostic counter applies (mpcqp/flops.py crash_ws_flops / pass_flops). */
static _Thread_local double t_sflops;
static double crash_ws_flops(int nf, int k) {
    /* Gram M = J_A J_A' (k(k+1)/2 entries, nf-long dots), Gauss-Jordan with one right-hand side,
     * w, y = J_A' w, x = x0 - J y, f */
    return (double)k * (k + 1) * nf + (double)(k - 1) * k * (k + 1) + 2.0 * k * nf +
           2.0 * nf * nf + nf + 3.0 * k;
}
static double pass_flops(int nf, int q, int friction_row) {
    const double r = (double)(nf - q > 0 ? nf - q : 0);
    return (double)q * q + 4.0 * nf + 2.0 * nf * r + 2.0 * nf + 3.0 * q + 4.0 * nf * r +
           (friction_row ? 2.0 * nf : 0.0);
}

static int box_crash(int n, const double *J, const double *x0, double fval0, const gi_cons *C,
                     int kmax, int pmax, double *x, double *fval, double *u_cons, int *solves) {
    int *lo_c = malloc(sizeof(int) * 2 * n), *up_c = lo_c + n;
    int *side = calloc((size_t)2 * n, sizeof(int)), *nw = side + n;
    int *A = malloc(sizeof(int) * (n + 1));
    double *lam = calloc((size_t)n, sizeof(double)), *xc = malloc(sizeof(double) * n);
    double *M = malloc(sizeof(double) * (size_t)n * n), *r = malloc(sizeof(double) * 3 * n);
    double *r0 = r + n, *y = r + 2 * n;
    double fv = fval0;
    int ok = 0, it = 0, ns = 0;
    for (int j = 0; j < n; ++j) { lo_c[j] = up_c[j] = -1; xc[j] = x0[j]; }
    for (int c = 0; c < C->m; ++c) {
        const int s = C->src[c];
        if (C->is_eq[c] || s >= 2 * n) goto out; /* not a bounds-only problem */
        if (s < n) lo_c[s] = c; else up_c[s - n] = c;
    }
    for (;;) {
        int changed = 0, cnt = 0;
        for (int j = 0; j < n; ++j) {
            nw[j] = side[j];
            if (side[j] == 0) {
                if (lo_c[j] >= 0) {
                    const double b = C->b[lo_c[j]];
                    if (xc[j] - b < -GI_FEAS_TOL * (1.0 + fabs(b))) nw[j] = 1;
                }
                if (nw[j] == 0 && up_c[j] >= 0) {
                    const double b = C->b[up_c[j]]; /* -ub */
                    if (-xc[j] - b < -GI_FEAS_TOL * (1.0 + fabs(b))) nw[j] = -1;
                }
            } else if (lam[j] < 0.0) {
                nw[j] = 0;
            }
            changed |= nw[j] != side[j];
            cnt += nw[j] != 0;
        }
        if (!changed) { ok = 1; break; } /* (it = 0: x0 violates nothing) */
        if (it >= pmax) break;
        if (cnt > kmax) { /* kept bounds first, then new ones by variable id */
            int kept = 0;
            for (int j = 0; j < n; ++j) kept += side[j] != 0 && nw[j] != 0;
            int room = kmax - kept;
            for (int j = 0; j < n; ++j)
                if (side[j] == 0 && nw[j] != 0) {
                    if (room > 0) --room;
                    else nw[j] = 0;
                }
        }
        int k = 0;
        for (int j = 0; j < n; ++j) {
            side[j] = nw[j];
            if (side[j]) A[k++] = j;
        }
        ++it;
        if (k == 0) {
            for (int j = 0; j < n; ++j) { xc[j] = x0[j]; lam[j] = 0.0; }
            fv = fval0;
            continue;
        }
        ++ns;
        t_sflops += crash_ws_flops(n, k);
        for (int i = 0; i < k; ++i) {
            for (int m = 0; m < k; ++m) {
                double s = 0.0;
                for (int c = 0; c < n; ++c) s += J[IDX(A[i], c, n)] * J[IDX(A[m], c, n)];
                M[IDX(i, m, k)] = s;
            }
            const int a = A[i];
            const double b = side[a] > 0 ? C->b[lo_c[a]] : -C->b[up_c[a]];
            r[i] = r0[i] = x0[a] - b;
        }
        int pd = 1;
        for (int j = 0; j < k && pd; ++j) {
            const double d = M[IDX(j, j, k)];
            if (!(d > 0.0)) { pd = 0; break; }
            const double inv = 1.0 / d;
            for (int i = 0; i < k; ++i) {
                if (i == j) continue;
                const double l = M[IDX(i, j, k)] * inv;
                for (int m = j + 1; m < k; ++m) M[IDX(i, m, k)] -= l * M[IDX(j, m, k)];
                r[i] -= l * r[j];
            }
        }
        if (!pd) break;
        double wr = 0.0;
        for (int i = 0; i < k; ++i) {
            r[i] = r[i] / M[IDX(i, i, k)]; /* w */
            wr += r[i] * r0[i];
        }
        for (int c = 0; c < n; ++c) {
            double s = 0.0;
            for (int i = 0; i < k; ++i) s += J[IDX(A[i], c, n)] * r[i];
            y[c] = s;
        }
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int c = 0; c < n; ++c) s += J[IDX(j, c, n)] * y[c];
            xc[j] = x0[j] - s;
            lam[j] = 0.0;
        }
        for (int i = 0; i < k; ++i) {
            const int a = A[i];
            xc[a] = side[a] > 0 ? C->b[lo_c[a]] : -C->b[up_c[a]];
            lam[a] = -(double)side[a] * r[i];
        }
        fv = fval0 + 0.5 * wr;
    }
    if (ok) {
        for (int j = 0; j < n; ++j) x[j] = xc[j];
        *fval = fv;
        if (u_cons) {
            for (int c = 0; c < C->m; ++c) u_cons[c] = 0.0;
            for (int j = 0; j < n; ++j)
                if (side[j]) u_cons[side[j] > 0 ? lo_c[j] : up_c[j]] = lam[j];
        }
    }
out:
    *solves = ns;
    free(lo_c); free(side); free(A); free(lam); free(xc); free(M); free(r);
    return ok;
}

static int gi_solve(int n, double *Hf /* n x n, destroyed */, const double *g, gi_cons *C,
                    int max_iter, double *x, double *fval_out, int *iters_out,
                    double *u_out /* m */, int crash_kmax, int crash_pmax) {
    const int m = C->m;
    double *J = calloc((size_t)n * n, sizeof(double));
    double *Rm = calloc((size_t)n * n, sizeof(double));
    double *d = malloc(sizeof(double) * (n + 1));
    double *z = malloc(sizeof(double) * (n + 1));
    double *r = malloc(sizeof(double) * (n + 1));
    double *u = malloc(sizeof(double) * (n + 2));
    double *w = malloc(sizeof(double) * (n + 1));
    int *act = malloc(sizeof(int) * (n + 1));
    char *isact = calloc((size_t)m + 1, 1);
    int status = ORC_OK, iters = 0, q = 0;
    double fval = 0.0;

    /* Cholesky Hf = L L' (lower, in place) */
    for (int k = 0; k < n; ++k) {
        double piv = Hf[IDX(k, k, n)];
        for (int l = 0; l < k; ++l) piv -= Hf[IDX(k, l, n)] * Hf[IDX(k, l, n)];
        if (!(piv > 0.0)) { status = ORC_NOT_PD; goto done; }
        const double lkk = sqrt(piv);
        Hf[IDX(k, k, n)] = lkk;
        for (int i = k + 1; i < n; ++i) {
            double s = Hf[IDX(i, k, n)];
            for (int l = 0; l < k; ++l) s -= Hf[IDX(i, l, n)] * Hf[IDX(k, l, n)];
            Hf[IDX(i, k, n)] = s / lkk;
        }
    }
    /* J = L^-T: column c of L^-1 by forward substitution, J(c, i) = Linv(i, c) */
    for (int c = 0; c < n; ++c) {
        for (int i = 0; i < c; ++i) w[i] = 0.0;
        for (int i = c; i < n; ++i) {
            double s = (i == c) ? 1.0 : 0.0;
            for (int l = c; l < i; ++l) s -= Hf[IDX(i, l, n)] * w[l];
            w[i] = s / Hf[IDX(i, i, n)];
        }
        for (int i = 0; i < n; ++i) J[IDX(c, i, n)] = w[i];
    }
    /* unconstrained minimum x = -J J' g, fval = 1/2 g'x */
    for (int j = 0; j < n; ++j) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += J[IDX(i, j, n)] * g[i];
        w[j] = s;
    }
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += J[IDX(i, j, n)] * w[j];
        x[i] = -s;
    }
    for (int i = 0; i < n; ++i) fval += 0.5 * g[i] * x[i];

    if (crash_kmax > 0 && m > 0) {
        int solves = 0;
        if (box_crash(n, J, x, fval, C, crash_kmax, crash_pmax, x, &fval, u_out, &solves)) {
            *fval_out = fval;
            *iters_out = solves;
            free(J); free(Rm); free(d); free(z); free(r); free(u); free(w); free(act);
            free(isact);
            return ORC_OK;
        }
        iters = solves; /* gave up: Goldfarb-Idnani from the unconstrained minimum */
    }

    /* equality constraints first (full steps, never dropped), then the dual loop */
    int eq_next = 0;
    for (;;) {
        int p = -1;
        double sp = 0.0;
        int adding_eq = 0;
        while (eq_next < m && !C->is_eq[eq_next]) ++eq_next;
        if (eq_next < m) {
            p = eq_next++;
            adding_eq = 1;
            const double *np = C->N + (size_t)p * n;
            sp = -C->b[p];
            for (int i = 0; i < n; ++i) sp += np[i] * x[i];
        } else {
            /* step 1: most violated inactive inequality */
            double best = 0.0;
            for (int c = 0; c < m; ++c) {
                if (isact[c] || C->is_eq[c]) continue;
                const double *nc = C->N + (size_t)c * n;
                double s = -C->b[c];
                for (int i = 0; i < n; ++i) s += nc[i] * x[i];
                const double key = C->qsel ? gi_sel_key(s) : s;
                if (s < -GI_FEAS_TOL * (1.0 + fabs(C->b[c])) && (p < 0 || key < best)) {
                    best = key;
                    sp = s;
                    p = c;
                }
            }
            if (p < 0) break; /* optimal */
        }
        const double *np = C->N + (size_t)p * n;
        u[q] = 0.0;
        /* step 2 */
        for (;;) {
            if (iters >= max_iter) { status = ORC_ITER_LIMIT; goto done; }
            ++iters;
            t_sflops += pass_flops(n, q, C->src[p] >= 2 * n);
            double dd = 0.0, zn = 0.0;
            for (int j = 0; j < n; ++j) {
                double s = 0.0;
                for (int i = 0; i < n; ++i) s += J[IDX(i, j, n)] * np[i];
                d[j] = s;
                dd += s * s;
                if (j >= q) zn += s * s;
            }
            for (int i = 0; i < n; ++i) {
                double s = 0.0;
                for (int j = q; j < n; ++j) s += J[IDX(i, j, n)] * d[j];
                z[i] = s;
            }
            for (int j = q - 1; j >= 0; --j) {
                double s = d[j];
                for (int l = j + 1; l < q; ++l) s -= Rm[IDX(j, l, n)] * r[l];
                r[j] = s / Rm[IDX(j, j, n)];
            }
            double rmax = 0.0;
            for (int j = 0; j < q; ++j)
                if (fabs(r[j]) > rmax) rmax = fabs(r[j]);
            double t1 = INFINITY;
            int k = -1;
            if (!adding_eq)
                for (int j = 0; j < q; ++j) {
                    if (C->is_eq[act[j]]) continue;
                    if (r[j] > GI_R_TOL * rmax) {
                        const double ratio = u[j] / r[j];
                        if (ratio < t1) { t1 = ratio; k = j; }
                    }
                }
            double t2 = INFINITY;
            if (zn > GI_DEP_TOL * dd) t2 = -sp / zn;
            if (adding_eq && !(zn > GI_DEP_TOL * dd)) {
                /* dependent equality: consistent -> skip, else infeasible */
                if (fabs(sp) <= GI_FEAS_TOL * (1.0 + fabs(C->b[p]))) break;
                status = ORC_INFEASIBLE;
                goto done;
            }
            const double t = (t1 < t2) ? t1 : t2;
            if (isinf(t)) { status = ORC_INFEASIBLE; goto done; }
            if (isinf(t2)) {
                /* dual step only, then drop k */
                for (int j = 0; j < q; ++j) u[j] -= t * r[j];
                u[q] += t;
            } else {
                for (int i = 0; i < n; ++i) x[i] += t * z[i];
                fval += t * zn * (0.5 * t + u[q]);
                for (int j = 0; j < q; ++j) u[j] -= t * r[j];
                u[q] += t;
                if (t2 <= t1) {
                    /* full step: add p.  Givens on d from the bottom up to q+1 */
                    for (int j = n - 1; j > q; --j) {
                        const double a = d[j - 1], bb = d[j];
                        if (bb == 0.0) continue;
                        const double h = sqrt(a * a + bb * bb);
                        const double c = a / h, s = bb / h;
                        d[j - 1] = h;
                        d[j] = 0.0;
                        for (int i = 0; i < n; ++i) {
                            const double x0 = J[IDX(i, j - 1, n)], x1 = J[IDX(i, j, n)];
                            J[IDX(i, j - 1, n)] = c * x0 + s * x1;
                            J[IDX(i, j, n)] = -s * x0 + c * x1;
                        }
                    }
                    for (int i = 0; i <= q; ++i) Rm[IDX(i, q, n)] = d[i];
                    act[q] = p;
                    isact[p] = 1;
                    ++q;
                    break; /* back to step 1 */
                }
            }
            /* drop constraint in slot k */
            isact[act[k]] = 0;
            for (int j = k; j < q - 1; ++j) {
                act[j] = act[j + 1];
                u[j] = u[j + 1];
                for (int i = 0; i <= j + 1; ++i) Rm[IDX(i, j, n)] = Rm[IDX(i, j + 1, n)];
            }
            u[q - 1] = u[q];
            --q;
            for (int j = k; j < q; ++j) {
                const double a = Rm[IDX(j, j, n)], bb = Rm[IDX(j + 1, j, n)];
                if (bb == 0.0) continue;
                const double h = sqrt(a * a + bb * bb);
                const double c = a / h, s = bb / h;
                Rm[IDX(j, j, n)] = h;
                Rm[IDX(j + 1, j, n)] = 0.0;
                for (int l = j + 1; l < q; ++l) {
                    const double x0 = Rm[IDX(j, l, n)], x1 = Rm[IDX(j + 1, l, n)];
                    Rm[IDX(j, l, n)] = c * x0 + s * x1;
                    Rm[IDX(j + 1, l, n)] = -s * x0 + c * x1;
                }
                for (int i = 0; i < n; ++i) {
                    const double x0 = J[IDX(i, j, n)], x1 = J[IDX(i, j + 1, n)];
                    J[IDX(i, j, n)] = c * x0 + s * x1;
                    J[IDX(i, j + 1, n)] = -s * x0 + c * x1;
                }
            }
            /* p stays the target; refresh its slack */
            sp = -C->b[p];
            for (int i = 0; i < n; ++i) sp += np[i] * x[i];
        }
    }
done:
    if (u_out) {
        for (int c = 0; c < m; ++c) u_out[c] = 0.0;
        if (status == ORC_OK)
            for (int j = 0; j < q; ++j) u_out[act[j]] = u[j];
    }
    *fval_out = fval;
    *iters_out = iters;
    free(J); free(Rm); free(d); free(z); free(r); free(u); free(w); free(act); free(isact);
    return status;
}

static int solve_qp_impl(int n, const double *H, const double *f, int mA, const double *A,
                         int a_colmajor, const double *lb, const double *ub, const double *lbA,
                         const double *ubA, const orc_friction *fric, int max_iter, double *x,
                         double *cost, int *iters, double *lam_bounds, double *lam_rows,
                         int crash_kmax, int crash_pmax);

int orc_solve_qp(int n, const double *H, const double *f, int mA, const double *A,
                 int a_colmajor, const double *lb, const double *ub, const double *lbA,
                 const double *ubA, const orc_friction *fric, int max_iter, double *x,
                 double *cost, int *iters, double *lam_bounds, double *lam_rows) {
    return solve_qp_impl(n, H, f, mA, A, a_colmajor, lb, ub, lbA, ubA, fric, max_iter, x, cost,
                         iters, lam_bounds, lam_rows, 0, 0);
}

static int solve_qp_impl(int n, const double *H, const double *f, int mA, const double *A,
                         int a_colmajor, const double *lb, const double *ub, const double *lbA,
                         const double *ubA, const orc_friction *fric, int max_iter, double *x,
                         double *cost, int *iters, double *lam_bounds, double *lam_rows,
                         int crash_kmax, int crash_pmax) {
    if (n <= 0 || mA < 0) return ORC_BAD_DIMS;
    int *pos = malloc(sizeof(int) * n);
    int *fid = malloc(sizeof(int) * n);
    double *xB = calloc((size_t)n, sizeof(double));
    int nf = 0, status = ORC_OK;
    for (int i = 0; i < n; ++i) {
        const double l = lb ? lb[i] : -ORC_INFTY, u = ub ? ub[i] : ORC_INFTY;
        if (l > u) status = ORC_INFEASIBLE;
        if (l == u) { pos[i] = -1; xB[i] = l; }
        else { pos[i] = nf; fid[nf++] = i; }
    }
    if (status != ORC_OK) { free(pos); free(fid); free(xB); return status; }

    /* reduced problem */
    double *Hf = malloc(sizeof(double) * (size_t)(nf ? nf : 1) * (nf ? nf : 1));
    double *g = malloc(sizeof(double) * (nf + 1));
    double c0 = 0.0;
    for (int a = 0; a < nf; ++a)
        for (int b = 0; b < nf; ++b) Hf[IDX(a, b, nf)] = H[IDX(fid[a], fid[b], n)];
    for (int a = 0; a < nf; ++a) {
        double s = f[fid[a]];
        for (int j = 0; j < n; ++j)
            if (pos[j] < 0) s += H[IDX(fid[a], j, n)] * xB[j];
        g[a] = s;
    }
    for (int i = 0; i < n; ++i)
        if (pos[i] < 0) {
            double s = 0.0;
            for (int j = 0; j < n; ++j)
                if (pos[j] < 0) s += H[IDX(i, j, n)] * xB[j];
            c0 += 0.5 * xB[i] * s + f[i] * xB[i];
        }

    /* one-sided constraints in the canonical order */
    const int nfric = (fric && fric->enabled) ? 4 * fric->N * fric->nfeet : 0;
    const int mmax = 2 * nf + nfric + 2 * mA;
    gi_cons C;
    C.n = nf;
    C.m = 0;
    C.N = calloc((size_t)(mmax ? mmax : 1) * (nf ? nf : 1), sizeof(double));
    C.b = malloc(sizeof(double) * (mmax + 1));
    C.is_eq = malloc(sizeof(int) * (mmax + 1));
    C.src = malloc(sizeof(int) * (mmax + 1));
    C.qsel = nfric > 0 && fric->contact_mask != 0;
    double *full = malloc(sizeof(double) * n);
#define ADD_CONS(normal_full, bval, eqflag, srcid)                                          \
    do {                                                                                    \
        double bb_ = (bval);                                                                \
        double *row_ = C.N + (size_t)C.m * nf;                                              \
        double nrm_ = 0.0;                                                                  \
        for (int i_ = 0; i_ < n; ++i_) {                                                    \
            if (pos[i_] < 0) bb_ -= (normal_full)[i_] * xB[i_];                             \
            else { row_[pos[i_]] = (normal_full)[i_]; nrm_ += fabs((normal_full)[i_]); }    \
        }                                                                                   \
        if (nrm_ == 0.0) {                                                                  \
            const double viol_ = (eqflag) ? fabs(bb_) : bb_;                                \
            if (viol_ > GI_FEAS_TOL * (1.0 + fabs(bb_))) status = ORC_INFEASIBLE;          \
        } else {                                                                            \
            C.b[C.m] = bb_; C.is_eq[C.m] = (eqflag); C.src[C.m] = (srcid); ++C.m;           \
        }                                                                                   \
    } while (0)

    for (int a = 0; a < nf; ++a)
        if (lb && lb[fid[a]] > -ORC_INFTY) {
            if (nfric && fric->elide_fz && fric->mu > 0.0 && lb[fid[a]] <= 0.0) {
                const int k = fid[a] / fric->nu, c = fid[a] % fric->nu;
                if (c % 3 == 2 && c / 3 < fric->nfeet && ((fric->contact_mask >> (2 * k + c / 3)) & 1ull))
                    continue; /* implied by the foot's pyramid rows */
            }
            memset(full, 0, sizeof(double) * n);
            full[fid[a]] = 1.0;
            ADD_CONS(full, lb[fid[a]], 0, a);
        }
    for (int a = 0; a < nf; ++a)
        if (ub && ub[fid[a]] < ORC_INFTY) {
            memset(full, 0, sizeof(double) * n);
            full[fid[a]] = -1.0;
            ADD_CONS(full, -ub[fid[a]], 0, nf + a);
        }
    if (nfric)
        for (int k = 0; k < fric->N; ++k)
            for (int s = 0; s < fric->nfeet; ++s) {
                if (!((fric->contact_mask >> (2 * k + s)) & 1ull)) continue;
                const int base = k * fric->nu + 3 * s;
                for (int t = 0; t < 4; ++t) {
                    memset(full, 0, sizeof(double) * n);
                    full[base + 2] = fric->mu;
                    full[base + (t >> 1)] = (t & 1) ? 1.0 : -1.0;
                    ADD_CONS(full, 0.0, 0, 2 * nf + (k * fric->nfeet + s) * 4 + t);
                }
            }
    for (int rr = 0; rr < mA; ++rr) {
        for (int i = 0; i < n; ++i)
            full[i] = a_colmajor ? A[IDX(rr, i, mA)] : A[(size_t)rr * n + i];
        const double lo = lbA ? lbA[rr] : -ORC_INFTY, hi = ubA ? ubA[rr] : ORC_INFTY;
        if (lo > hi) status = ORC_INFEASIBLE;
        if (lo == hi) {
            ADD_CONS(full, lo, 1, 2 * nf + nfric + 2 * rr);
        } else {
            if (lo > -ORC_INFTY) ADD_CONS(full, lo, 0, 2 * nf + nfric + 2 * rr);
            if (hi < ORC_INFTY) {
                for (int i = 0; i < n; ++i) full[i] = -full[i];
                ADD_CONS(full, -hi, 0, 2 * nf + nfric + 2 * rr + 1);
            }
        }
    }
#undef ADD_CONS

    double *xf = calloc((size_t)nf + 1, sizeof(double));
    double *uc = calloc((size_t)C.m + 1, sizeof(double));
    double fv = 0.0;
    int it = 0;
    if (status == ORC_OK && nf > 0)
        status = gi_solve(nf, Hf, g, &C, max_iter > 0 ? max_iter : 10 * (C.m + nf + 1), xf,
                          &fv, &it, uc, crash_kmax, crash_pmax);
    for (int i = 0; i < n; ++i) x[i] = pos[i] < 0 ? xB[i] : xf[pos[i]];
    if (cost) *cost = fv + c0;
    if (iters) *iters = it;
    if (lam_bounds || lam_rows) {
        /* y such that H x + f = y_bounds + A' y_rows (qpOASES sign convention) */
        if (lam_bounds) memset(lam_bounds, 0, sizeof(double) * n);
        if (lam_rows && mA) memset(lam_rows, 0, sizeof(double) * mA);
        for (int c = 0; c < C.m; ++c) {
            const int s = C.src[c];
            if (s < nf) { if (lam_bounds) lam_bounds[fid[s]] += uc[c]; }
            else if (s < 2 * nf) { if (lam_bounds) lam_bounds[fid[s - nf]] -= uc[c]; }
            else if (s >= 2 * nf + nfric) {
                const int rr = (s - 2 * nf - nfric) >> 1, side = (s - 2 * nf - nfric) & 1;
                if (lam_rows) lam_rows[rr] += side ? -uc[c] : uc[c];
            }
        }
        if (lam_bounds) /* fixed variables: the whole remaining gradient */
            for (int i = 0; i < n; ++i)
                if (pos[i] < 0) {
                    double s = f[i];
                    for (int j = 0; j < n; ++j) s += H[IDX(i, j, n)] * x[j];
                    if (lam_rows)
                        for (int rr = 0; rr < mA; ++rr)
                            s -= (a_colmajor ? A[IDX(rr, i, mA)] : A[(size_t)rr * n + i]) *
                                 lam_rows[rr];
                    lam_bounds[i] = s;
                }
    }
    free(pos); free(fid); free(xB); free(Hf); free(g); free(C.N); free(C.b); free(C.is_eq);
    free(C.src); free(full); free(xf); free(uc);
    return status;
}

/* ---------------------------------------------------------------- SRBM models */
/* mpcQP::buildSystemModel, include/mpcQP.h:139-181 (0-based indices; the reference's
 * placeholder physics is reproduced verbatim: lever-arm terms in rows 1-3, -1 at (12,13),
 * Bc = -m I in rows 10-12; inB is computed there but unused, so it is not needed here). */
void orc_model_literal(double dx, double dy, double dz, double m, double *Ac, double *Bc) {
    memset(Ac, 0, sizeof(double) * 13 * 13);
    memset(Bc, 0, sizeof(double) * 13 * 3);
    Ac[IDX(0, 7, 13)] = dz; Ac[IDX(0, 8, 13)] = dy;
    Ac[IDX(1, 6, 13)] = dz; Ac[IDX(1, 8, 13)] = dx;
    Ac[IDX(2, 6, 13)] = dy; Ac[IDX(2, 7, 13)] = dx;
    Ac[IDX(3, 9, 13)] = 1.0; Ac[IDX(4, 10, 13)] = 1.0; Ac[IDX(5, 11, 13)] = 1.0;
    Ac[IDX(11, 12, 13)] = -1.0;
    Bc[IDX(9, 0, 13)] = -m; Bc[IDX(10, 1, 13)] = -m; Bc[IDX(11, 2, 13)] = -m;
}

static void inv3(const double *A, double *Ai) { /* column-major 3x3 inverse (adjugate) */
    const double a = A[0], b = A[3], c = A[6], d = A[1], e = A[4], f = A[7], g = A[2],
                 h = A[5], i = A[8];
    const double A00 = e * i - f * h, A01 = -(d * i - f * g), A02 = d * h - e * g;
    const double det = a * A00 + b * A01 + c * A02;
    const double id = 1.0 / det;
    Ai[0] = A00 * id; Ai[3] = -(b * i - c * h) * id; Ai[6] = (b * f - c * e) * id;
    Ai[1] = A01 * id; Ai[4] = (a * i - c * g) * id;  Ai[7] = -(a * f - c * d) * id;
    Ai[2] = A02 * id; Ai[5] = -(a * h - b * g) * id; Ai[8] = (a * e - b * d) * id;
}

/* Convex-MPC single-rigid-body model (build's definition):
 * state x = [rpy(0:3), p(3:6), omega(6:9), v(9:12), g(12)] as the reference's xi
 * (include/mpcQP.h:67-71, g = -9.8), input u = [f_L(3), f_R(3)] world-frame GRFs.
 *   d rpy/dt = Rz(yaw)' omega;  dp/dt = v;  dv/dt = (f_L + f_R)/m + g e_z;
 *   d omega/dt = I_w^-1 (r_L x f_L + r_R x f_R),  I_w = Rz Ib Rz'.
 * lin = {yaw, r_L(3), r_R(3)} with r_s = foot_s - CoM (world). */
void orc_model_srbm(const double *lin, double m, const double *Ib, double *Ac, double *Bc) {
    memset(Ac, 0, sizeof(double) * 13 * 13);
    memset(Bc, 0, sizeof(double) * 13 * 6);
    const double cy = cos(lin[0]), sy = sin(lin[0]);
    /* Rz' */
    Ac[IDX(0, 6, 13)] = cy;  Ac[IDX(0, 7, 13)] = sy;
    Ac[IDX(1, 6, 13)] = -sy; Ac[IDX(1, 7, 13)] = cy;
    Ac[IDX(2, 8, 13)] = 1.0;
    Ac[IDX(3, 9, 13)] = 1.0; Ac[IDX(4, 10, 13)] = 1.0; Ac[IDX(5, 11, 13)] = 1.0;
    Ac[IDX(11, 12, 13)] = 1.0;
    /* I_w^-1 = Rz Ib^-1 Rz' */
    double Ibi[9], Rz[9] = {cy, sy, 0, -sy, cy, 0, 0, 0, 1}, T[9], Iwi[9];
    inv3(Ib, Ibi);
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) {
            double s = 0.0;
            for (int l = 0; l < 3; ++l) s += Rz[IDX(i, l, 3)] * Ibi[IDX(l, j, 3)];
            T[IDX(i, j, 3)] = s;
        }
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) {
            double s = 0.0;
            for (int l = 0; l < 3; ++l) s += T[IDX(i, l, 3)] * Rz[IDX(j, l, 3)];
            Iwi[IDX(i, j, 3)] = s;
        }
    for (int ft = 0; ft < 2; ++ft) {
        const double *rr = lin + 1 + 3 * ft;
        const double X[9] = {0, rr[2], -rr[1], -rr[2], 0, rr[0], rr[1], -rr[0], 0}; /* [r]x */
        for (int j = 0; j < 3; ++j)
            for (int i = 0; i < 3; ++i) {
                double s = 0.0;
                for (int l = 0; l < 3; ++l) s += Iwi[IDX(i, l, 3)] * X[IDX(l, j, 3)];
                Bc[IDX(6 + i, 3 * ft + j, 13)] = s;
            }
        for (int i = 0; i < 3; ++i) Bc[IDX(9 + i, 3 * ft + i, 13)] = 1.0 / m;
    }
}

/* MPC::calculateGait, include/MPCController.h:61-75, evaluated at each horizon step:
 * t_k = phase0 + k*Ts; phase = fmod(t_k, swing+stance); phase < swing => left swings
 * (right in contact) else left in contact.  bit 2k = left contact, bit 2k+1 = right. */
uint64_t orc_gait_contact_mask(int N, double Ts, double phase0, float swing_time,
                               float stance_time) {
    const double cycle = (double)(swing_time + stance_time); /* float sum, as the reference */
    uint64_t mask = 0;
    for (int k = 0; k < N && k < 32; ++k) {
        const double t = phase0 + (double)k * Ts;
        const double ph = fmod(t, cycle);
        if (ph < (double)swing_time) mask |= 1ull << (2 * k + 1);
        else mask |= 1ull << (2 * k);
    }
    return mask;
}

void orc_srbm_bounds(const orc_srbm_cfg *cfg, uint64_t contact, double *lb, double *ub) {
    const int nu = cfg->nu;
    for (int k = 0; k < cfg->N; ++k) {
        if (cfg->model == 1) {
            for (int c = 0; c < nu; ++c) { lb[k * nu + c] = cfg->u_min; ub[k * nu + c] = cfg->u_max; }
            continue;
        }
        for (int s = 0; s < 2; ++s) {
            const int b = k * nu + 3 * s;
            if ((contact >> (2 * k + s)) & 1ull) {
                lb[b + 0] = -cfg->fxy_max; ub[b + 0] = cfg->fxy_max;
                lb[b + 1] = -cfg->fxy_max; ub[b + 1] = cfg->fxy_max;
                lb[b + 2] = cfg->fz_min;   ub[b + 2] = cfg->fz_max;
            } else {
                for (int c = 0; c < 3; ++c) { lb[b + c] = 0.0; ub[b + c] = 0.0; }
            }
        }
    }
}

/* One instance of the batched pipeline: linearise -> discretise -> condense -> solve.
 * Condensing here is the reference's literal dense product (orc_build_qp). */
static int srbm_one(const orc_srbm_cfg *cfg, const double *x0, const double *xref,
                    const double *lin, uint64_t contact, double *U, double *cost, int *iters,
                    double *Hout, double *fout) {
    const int nx = cfg->nx, nu = cfg->nu, N = cfg->N, nV = nu * N;
    double Ac[13 * 13], Bc[13 * 6], Ad[13 * 13], Bd[13 * 6];
    if (nx != 13 || (cfg->model == 0 && nu != 6) || (cfg->model == 1 && nu != 3))
        return ORC_BAD_DIMS;
    if (cfg->model == 1) orc_model_literal(lin[0], lin[1], lin[2], cfg->mass, Ac, Bc);
    else orc_model_srbm(lin, cfg->mass, cfg->Ib, Ac, Bc);
    orc_discretize(nx, nu, cfg->Ts, Ac, Bc, Ad, Bd);
    double *H = Hout ? Hout : malloc(sizeof(double) * nV * nV);
    double *f = fout ? fout : malloc(sizeof(double) * nV);
    double *lb = malloc(sizeof(double) * nV * 2), *ub = lb + nV;
    orc_build_qp(nx, nu, N, Ad, Bd, cfg->Q, cfg->R, cfg->P, NULL, NULL, 0, 0, x0, xref, H, f,
                 NULL, NULL, NULL, NULL, NULL, NULL, NULL);
    orc_srbm_bounds(cfg, contact, lb, ub);
    orc_friction fr = {cfg->friction && cfg->model == 0, nu, N, 2, cfg->mu, contact, cfg->elide_fz};
    int nfree = 0;
    for (int v = 0; v < nV; ++v) nfree += lb[v] != ub[v];
    const int wg = nfree > cfg->crash_split;
    int st = solve_qp_impl(nV, H, f, 0, NULL, 0, lb, ub, NULL, NULL, &fr, cfg->max_iter, U,
                           cost, iters, NULL, NULL, wg ? cfg->crash_kmax_wg : cfg->crash_kmax,
                           wg ? cfg->crash_pmax_wg : cfg->crash_pmax);
    if (!Hout) free(H);
    if (!fout) free(f);
    free(lb);
    return st;
}

int orc_srbm_batch(const orc_srbm_cfg *cfg, int B, const double *x0, const double *xref,
                   const double *lin, const uint64_t *contact, double *U, double *cost,
                   int *status, int *iters, double *H_out, double *f_out, int nthreads,
                   double *sflops) {
    const int nx = cfg->nx, nV = cfg->nu * cfg->N;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
    for (int b = 0; b < B; ++b) {
        int it = 0;
        double c = 0.0;
        t_sflops = 0.0;
        const int st = srbm_one(cfg, x0 + (size_t)b * nx, xref + (size_t)b * nx * (cfg->N + 1),
                                lin + (size_t)b * 8, contact[b], U + (size_t)b * nV, &c, &it,
                                H_out ? H_out + (size_t)b * nV * nV : NULL,
                                f_out ? f_out + (size_t)b * nV : NULL);
        if (cost) cost[b] = c;
        if (status) status[b] = st;
        if (iters) iters[b] = it;
        if (sflops) sflops[b] = t_sflops;
    }
    (void)nthreads;
    return ORC_OK;
}

/* dense model, one instance (config E) -- see mpcqp_oracle.h */
static int dense_one(const orc_dense_cfg *cfg, const double *x0, const double *xref,
                     const double *AB, double *U, double *cost, int *iters, double *Hout,
                     double *fout) {
    const int nx = cfg->nx, nu = cfg->nu, N = cfg->N, nV = nu * N;
    double *Ad = malloc(sizeof(double) * nx * (nx + nu)), *Bd = Ad + nx * nx;
    orc_discretize(nx, nu, cfg->Ts, AB, AB + nx * nx, Ad, Bd);
    double *H = Hout ? Hout : malloc(sizeof(double) * nV * nV);
    double *f = fout ? fout : malloc(sizeof(double) * nV);
    double *lb = malloc(sizeof(double) * nV * 2), *ub = lb + nV;
    orc_build_qp(nx, nu, N, Ad, Bd, cfg->Q, cfg->R, cfg->P, NULL, NULL, 0, 0, x0, xref, H, f,
                 NULL, NULL, NULL, NULL, NULL, NULL, NULL);
    for (int v = 0; v < nV; ++v) { lb[v] = cfg->u_min; ub[v] = cfg->u_max; }
    int st = solve_qp_impl(nV, H, f, 0, NULL, 0, lb, ub, NULL, NULL, NULL, cfg->max_iter, U,
                           cost, iters, NULL, NULL, cfg->crash_kmax, cfg->crash_pmax);
    if (!Hout) free(H);
    if (!fout) free(f);
    free(lb);
    free(Ad);
    return st;
}

int orc_dense_batch(const orc_dense_cfg *cfg, int B, const double *x0, const double *xref,
                    const double *AB, double *U, double *cost, int *status, int *iters,
                    double *H_out, double *f_out, int nthreads) {
    const int nx = cfg->nx, nV = cfg->nu * cfg->N, ab = cfg->nx * (cfg->nx + cfg->nu);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int b = 0; b < B; ++b) {
        int it = 0;
        double c = 0.0;
        const int st = dense_one(cfg, x0 + (size_t)b * nx, xref + (size_t)b * nx * (cfg->N + 1),
                                 AB + (size_t)b * ab, U + (size_t)b * nV, &c, &it,
                                 H_out ? H_out + (size_t)b * nV * nV : NULL,
                                 f_out ? f_out + (size_t)b * nV : NULL);
        if (cost) cost[b] = c;
        if (status) status[b] = st;
        if (iters) iters[b] = it;
    }
    (void)nthreads;
    return ORC_OK;
}

int orc_srbm_plant(const orc_srbm_cfg *cfg, const double *lin, double *x, const double *u) {
    double Ac[13 * 13], Bc[13 * 6], Ad[13 * 13], Bd[13 * 6];
    orc_model_srbm(lin, cfg->mass, cfg->Ib, Ac, Bc);
    const int rc = orc_discretize(13, 6, cfg->Ts, Ac, Bc, Ad, Bd);
    if (rc) return rc;
    orc_plant_step(13, 6, Ad, Bd, x, u);
    return ORC_OK;
}

/* ---- state estimator: stateEstimator::update, include/stateEstimator.h:217-337
 * One linear Kalman step of the 12-state estimator [p(3), v(3), foot positions(6)] with 14
 * measurements [-eePos (+foot radius on z), -eeVel, feetHeights(2) = 0].  Restated as
 * written, quirks included: dt*9.81f/20.f (float literal), q_(6:12) = dt I, the `y << ps, vs,
 * feetHeights_` of a 4-vector keeping its first two (zero) entries, accel = R(zyx)' a + g,
 * the symmetrisation and the det(P(0:2,0:2)) > 1e-6 decoupling.  R(zyx) is ocs2's
 * getRotationMatrixFromZyxEulerAngles (Rz Ry Rx; ocs2 is not vendored, restated). */
static void quat_to_zyx(const double *q /* x y z w */, double *zyx) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    double as = -2. * (x * z - w * y);
    if (as > .99999) as = .99999;
    zyx[0] = atan2(2 * (x * y + w * z), w * w + x * x - y * y - z * z);
    zyx[1] = asin(as);
    zyx[2] = atan2(2 * (y * z + w * x), w * w - x * x - y * y + z * z);
}
static void rot_zyx(const double *e, double *R /* col-major */) {
    const double c1 = cos(e[0]), c2 = cos(e[1]), c3 = cos(e[2]);
    const double s1 = sin(e[0]), s2 = sin(e[1]), s3 = sin(e[2]);
    R[IDX(0, 0, 3)] = c1 * c2; R[IDX(0, 1, 3)] = c1 * s2 * s3 - s1 * c3; R[IDX(0, 2, 3)] = c1 * s2 * c3 + s1 * s3;
    R[IDX(1, 0, 3)] = c2 * s1; R[IDX(1, 1, 3)] = s1 * s2 * s3 + c1 * c3; R[IDX(1, 2, 3)] = s1 * s2 * c3 - c1 * s3;
    R[IDX(2, 0, 3)] = -s2;     R[IDX(2, 1, 3)] = c2 * s3;                R[IDX(2, 2, 3)] = c2 * c3;
}

int orc_kf_update(double dt, double *xhat, double *P, const double *eePos, const double *eeVel,
                  const unsigned char *contact, const double *quat, const double *acc) {
    double A[144] = {0}, B[36] = {0}, Cm[168] = {0}, qd[12], rd[14], y[14];
    for (int i = 0; i < 12; ++i) A[IDX(i, i, 12)] = 1.0;
    for (int i = 0; i < 3; ++i) {
        A[IDX(i, 3 + i, 12)] = dt;
        B[IDX(i, i, 12)] = 0.5 * dt * dt;
        B[IDX(3 + i, i, 12)] = dt;
    }
    for (int i = 0; i < 3; ++i) {
        Cm[IDX(i, i, 14)] = 1.0; Cm[IDX(3 + i, i, 14)] = 1.0;          /* c1 blocks */
        Cm[IDX(6 + i, 3 + i, 14)] = 1.0; Cm[IDX(9 + i, 3 + i, 14)] = 1.0; /* c2 blocks */
    }
    for (int i = 0; i < 6; ++i) Cm[IDX(i, 6 + i, 14)] = -1.0;
    Cm[IDX(12, 8, 14)] = 1.0;
    Cm[IDX(13, 11, 14)] = 1.0;
    for (int i = 0; i < 3; ++i) {
        qd[i] = (dt / 20.f) * 0.02;
        qd[3 + i] = (dt * 9.81f / 20.f) * 0.02;
    }
    for (int i = 6; i < 12; ++i) qd[i] = dt * 0.002;
    for (int i = 0; i < 6; ++i) rd[i] = 0.005;
    for (int i = 6; i < 12; ++i) rd[i] = 0.1;
    rd[12] = rd[13] = 0.01;
    for (int f = 0; f < 2; ++f) {
        const double k = contact[f] ? 1.0 : 100.0;
        for (int d = 0; d < 3; ++d) {
            qd[6 + 3 * f + d] *= k;
            rd[3 * f + d] *= k;
            rd[6 + 3 * f + d] *= k;
            y[3 * f + d] = -eePos[3 * f + d] + (d == 2 ? 0.02 : 0.0);
            y[6 + 3 * f + d] = -eeVel[3 * f + d];
        }
        rd[12 + f] *= k;
    }
    y[12] = y[13] = 0.0;
    double zyx[3], R[9], accw[3];
    quat_to_zyx(quat, zyx);
    rot_zyx(zyx, R);
    for (int i = 0; i < 3; ++i) {
        double s = 0.0;
        for (int l = 0; l < 3; ++l) s += R[IDX(l, i, 3)] * acc[l]; /* R' a */
        accw[i] = s + (i == 2 ? -9.81 : 0.0);
    }
    double xn[12], T[144], Pm[144];
    for (int i = 0; i < 12; ++i) {
        double s = 0.0;
        for (int l = 0; l < 12; ++l) s += A[IDX(i, l, 12)] * xhat[l];
        for (int l = 0; l < 3; ++l) s += B[IDX(i, l, 12)] * accw[l];
        xn[i] = s;
    }
    mm(12, 12, 12, A, P, T);
    for (int j = 0; j < 12; ++j)
        for (int i = 0; i < 12; ++i) {
            double s = 0.0;
            for (int l = 0; l < 12; ++l) s += T[IDX(i, l, 12)] * A[IDX(j, l, 12)];
            Pm[IDX(i, j, 12)] = s + (i == j ? qd[i] : 0.0);
        }
    double PC[168], S[196], ey[14], X[14 * 13];
    for (int j = 0; j < 14; ++j) /* PC = Pm C' (12 x 14) */
        for (int i = 0; i < 12; ++i) {
            double s = 0.0;
            for (int l = 0; l < 12; ++l) s += Pm[IDX(i, l, 12)] * Cm[IDX(j, l, 14)];
            PC[IDX(i, j, 12)] = s;
        }
    for (int j = 0; j < 14; ++j)
        for (int i = 0; i < 14; ++i) {
            double s = 0.0;
            for (int l = 0; l < 12; ++l) s += Cm[IDX(i, l, 14)] * PC[IDX(l, j, 12)];
            S[IDX(i, j, 14)] = s + (i == j ? rd[i] : 0.0);
        }
    for (int i = 0; i < 14; ++i) {
        double s = 0.0;
        for (int l = 0; l < 12; ++l) s += Cm[IDX(i, l, 14)] * xn[l];
        ey[i] = y[i] - s;
    }
    for (int i = 0; i < 14; ++i) X[IDX(i, 0, 14)] = ey[i];
    for (int j = 0; j < 12; ++j)
        for (int i = 0; i < 14; ++i) X[IDX(i, 1 + j, 14)] = Cm[IDX(i, j, 14)];
    if (lu_solve(14, S, 13, X)) return ORC_NOT_PD;
    for (int i = 0; i < 12; ++i) {
        double s = 0.0;
        for (int l = 0; l < 14; ++l) s += PC[IDX(i, l, 12)] * X[IDX(l, 0, 14)];
        xhat[i] = xn[i] + s;
    }
    double K[144], Pn[144]; /* K = I - PC sC */
    for (int j = 0; j < 12; ++j)
        for (int i = 0; i < 12; ++i) {
            double s = 0.0;
            for (int l = 0; l < 14; ++l) s += PC[IDX(i, l, 12)] * X[IDX(l, 1 + j, 14)];
            K[IDX(i, j, 12)] = (i == j ? 1.0 : 0.0) - s;
        }
    mm(12, 12, 12, K, Pm, Pn);
    for (int j = 0; j < 12; ++j)
        for (int i = 0; i < 12; ++i) P[IDX(i, j, 12)] = (Pn[IDX(i, j, 12)] + Pn[IDX(j, i, 12)]) / 2.0;
    const double det = P[IDX(0, 0, 12)] * P[IDX(1, 1, 12)] - P[IDX(0, 1, 12)] * P[IDX(1, 0, 12)];
    if (det > 0.000001) {
        for (int j = 2; j < 12; ++j)
            for (int i = 0; i < 2; ++i) { P[IDX(i, j, 12)] = 0.0; P[IDX(j, i, 12)] = 0.0; }
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 2; ++i) P[IDX(i, j, 12)] /= 10.;
    }
    return ORC_OK;
}

/* ---- leg kinematics: foot contact points of the two 3-DoF legs.
 * The reference computes them with Pinocchio from PF_TRON1A's URDF
 * (include/pinocchio_kinematics.h:30-43), which is not in the repository; the chain is
 * restated from MPCParam's kinematicValues (include/MPCParam.h:13-38) with the usual
 * point-foot axes (abad about x, hip and knee about y -- build-chosen), and the left leg's
 * lateral sign convention of MPCParam.h:66-72.  At q = 0 it reproduces the reference's
 * static_foot_offset_{left,right} exactly (the pinned known answer).
 *   p_body = abad + Rx(q0) (hip + Ry(q1) (knee + Ry(q2) (foot + contact)))
 *   feet   = R(rpy) p_body, R = Rz(yaw) Ry(pitch) Rx(roll)  (world frame, foot minus base) */
static const double K_ABAD[3] = {0.05556, 0.105, -0.2602}, K_HIP[3] = {-0.077, 0.02050, 0.0},
                    K_KNEE[3] = {-0.1500, -0.02050, -0.25981}, K_FOOT[3] = {0.145, 0.0, -0.2598},
                    K_CONTACT[3] = {0.0, 0.0, -0.032};

void orc_fk_feet(const double *q, const double *rpy, double *feet) {
    const double cr = cos(rpy[0]), sr = sin(rpy[0]), cp = cos(rpy[1]), sp = sin(rpy[1]),
                 cyw = cos(rpy[2]), syw = sin(rpy[2]);
    for (int leg = 0; leg < 2; ++leg) {
        const double sg = leg == 0 ? -1.0 : 1.0;
        const double *ql = q + 3 * leg;
        double v[3] = {K_FOOT[0] + K_CONTACT[0], K_FOOT[1] + K_CONTACT[1], K_FOOT[2] + K_CONTACT[2]};
        /* knee: Ry(q2) v + knee */
        double c = cos(ql[2]), s = sin(ql[2]), t0 = c * v[0] + s * v[2], t2 = -s * v[0] + c * v[2];
        v[0] = t0 + K_KNEE[0]; v[1] = v[1] + sg * K_KNEE[1]; v[2] = t2 + K_KNEE[2];
        /* hip: Ry(q1) v + hip */
        c = cos(ql[1]); s = sin(ql[1]); t0 = c * v[0] + s * v[2]; t2 = -s * v[0] + c * v[2];
        v[0] = t0 + K_HIP[0]; v[1] = v[1] + sg * K_HIP[1]; v[2] = t2 + K_HIP[2];
        /* abad: Rx(q0) v + abad */
        c = cos(ql[0]); s = sin(ql[0]);
        const double t1 = c * v[1] - s * v[2];
        t2 = s * v[1] + c * v[2];
        v[0] = v[0] + K_ABAD[0]; v[1] = t1 + sg * K_ABAD[1]; v[2] = t2 + K_ABAD[2];
        /* world: Rz Ry Rx v */
        const double a1 = v[1] * cr - v[2] * sr, a2 = v[1] * sr + v[2] * cr;   /* Rx */
        const double b0 = v[0] * cp + a2 * sp, b2 = -v[0] * sp + a2 * cp;      /* Ry */
        feet[3 * leg + 0] = b0 * cyw - a1 * syw;                               /* Rz */
        feet[3 * leg + 1] = b0 * syw + a1 * cyw;
        feet[3 * leg + 2] = b2;
    }
}
